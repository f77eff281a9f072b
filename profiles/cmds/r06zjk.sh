#!/bin/bash
# r06zj: hash-stamped PMC profiles of library 75abee51 for C3, C4, the centralised bench and the
# naive-ADMM min_1_norm line, summarised on the box
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zj
for w in admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096 admm_n10_N10_l1_P32; do
  timeout -k 10 600 bash profiles/profile_all.sh /tmp/$R $w > gpurun_out/${R}_${w}_prof.log 2>&1 || exit 3
  python3 profiles/summarize.py /tmp/$R/$w $R $w >> gpurun_out/${R}_${w}_prof.log 2>&1 || exit 4
  mkdir -p gpurun_out/${R}_sum && cp profiles/${R}_${w}_summary.json profiles/${R}_${w}_kernel_stats.csv gpurun_out/${R}_sum/ || exit 5
  rm -rf /tmp/$R/$w
done
# r06zk: the bench lines of library 75abee51 with their CPU baselines (every host core + one),
# rooflines from the committed r06zi / r06zj summaries: C2 default, min_1_norm, C3, C4, centralised,
# and the naive-ADMM min_1_norm line (C3 with quadratic_cost=False)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zk
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench_default.jsonl 2> gpurun_out/${R}_bench_default.err || exit 1
timeout -k 10 300 python bench.py --cost l1 --steps 5 --warmup 1 > gpurun_out/${R}_bench_l1.jsonl 2> gpurun_out/${R}_bench_l1.err || exit 2
timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 > gpurun_out/${R}_bench_admm.jsonl 2> gpurun_out/${R}_bench_admm.err || exit 3
timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 > gpurun_out/${R}_bench_gadmm.jsonl 2> gpurun_out/${R}_bench_gadmm.err || exit 4
timeout -k 10 500 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 > gpurun_out/${R}_bench_cent.jsonl 2> gpurun_out/${R}_bench_cent.err || exit 5
timeout -k 10 300 python bench.py --controller admm --cost l1 --n 10 --N 10 --platoons 64 --steps 1 --warmup 0 > gpurun_out/${R}_bench_admm_l1.jsonl 2> gpurun_out/${R}_bench_admm_l1.err || exit 6
