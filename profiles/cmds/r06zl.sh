#!/bin/bash
# r06zl: decentralised min_1_norm at n = 10, N = 10 (a configs[4] sweep point; the wave interior point
# of DESIGN section 3) on library 75abee51 -- hash-stamped profile, then the bench line with its CPU baselines
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zl
w=decent_n10_N10_l1_P256
timeout -k 10 600 bash profiles/run_profiles.sh /tmp/$R/$w --cost l1 --N 10 --platoons 256 --steps 1 --warmup 1 --no-cpu --streams 1 > gpurun_out/${R}_${w}_prof.log 2>&1 || exit 1
python3 profiles/summarize.py /tmp/$R/$w $R $w >> gpurun_out/${R}_${w}_prof.log 2>&1 || exit 2
mkdir -p gpurun_out/${R}_sum && cp profiles/${R}_${w}_summary.json profiles/${R}_${w}_kernel_stats.csv gpurun_out/${R}_sum/ || exit 3
timeout -k 10 400 python bench.py --cost l1 --N 10 --platoons 256 --steps 2 --warmup 1 > gpurun_out/${R}_bench_l1_N10.jsonl 2> gpurun_out/${R}_bench_l1_N10.err || exit 4
