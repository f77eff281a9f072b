import csv,collections,sys
src=sys.argv[1]
for r in csv.DictReader(open(src+'/trace/run_kernel_stats.csv')):
    print('%-30s %4s %9.1f us %6.2f%%'%(r['Name'][:30], r['Calls'], float(r['AverageNs'])/1e3, float(r['Percentage'])))
acc=collections.defaultdict(lambda: collections.defaultdict(list))
for sub in ('occ','f64'):
    try:
        for r in csv.DictReader(open(f'{src}/{sub}/run_counter_collection.csv')):
            acc[r['Kernel_Name'][:40]][r['Counter_Name']].append(float(r['Counter_Value']))
    except FileNotFoundError: pass
for k,d in acc.items():
    if 'bnb_bound' in k or 'bnb_root' in k or 'qp' in k:
        m={c:sum(v)/len(v) for c,v in d.items()}
        print(k[:30], 'lane_util %.3f'%(m['SQ_THREAD_CYCLES_VALU']/64/m['SQ_ACTIVE_INST_VALU']), 'valu_issue %.3f'%(m['SQ_ACTIVE_INST_VALU']/m['SQ_WAVE_CYCLES']), 'wait %.3f'%(m['SQ_WAIT_ANY']/m['SQ_WAVE_CYCLES']), 'stall %.3f'%(m['SQ_WAIT_INST_ANY']/m['SQ_WAVE_CYCLES']), 'waves/cu %.2f'%(4*m['SQ_WAVE_CYCLES']/(m['GRBM_GUI_ACTIVE']/8)/256), 'valu %.3g f64 %.3g salu %.3g lds %.3g'%(m.get('SQ_INSTS_VALU',0), m.get('SQ_INSTS_VALU_FMA_F64',0)+m.get('SQ_INSTS_VALU_MUL_F64',0)+m.get('SQ_INSTS_VALU_ADD_F64',0)+m.get('SQ_INSTS_VALU_TRANS_F64',0), m.get('SQ_INSTS_SALU',0), m.get('SQ_INSTS_LDS',0)))
