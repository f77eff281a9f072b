#!/bin/bash
# r06zo: decentralised min_1_norm n = 10, N = 10 bench line with its CPU baselines (single-vehicle
# oracle samples past N = 8), library 75abee51; a heartbeat file while the CPU legs run
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zo
(while true; do date +%T >> gpurun_out/${R}_heartbeat.txt; sleep 40; done) &
HB=$!
timeout -k 10 500 python bench.py --cost l1 --N 10 --platoons 256 --steps 2 --warmup 1 > gpurun_out/${R}_bench_l1_N10.jsonl 2> gpurun_out/${R}_bench_l1_N10.err
rc=$?
kill $HB
exit $rc
