set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
B=(python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/trace -o run -- "${B[@]}" > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -T -f csv -d $OUT/occ -o run -- "${B[@]}" > $OUT/occ.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT64 -T -f csv -d $OUT/f64 -o run -- "${B[@]}" > $OUT/f64.log 2>&1
echo done
