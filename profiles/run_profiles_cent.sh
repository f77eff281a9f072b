#!/usr/bin/env bash
# Centralised MLD (bench.py --controller cent) on the GPU box, from the repo root:
# bench lines (with the bounded oracle CPU sample) and a rocprofv3 kernel trace of the search kernel.
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_cent}
mkdir -p "$OUT"
timeout -k 10 300 python3 bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 1 \
    --max-nodes 30000 --cpu-budget 20 > "$OUT/bench_n10.log" 2>&1
timeout -k 10 200 python3 bench.py --controller cent --n 5 --N 5 --platoons 4096 --steps 1 --warmup 1 \
    --max-nodes 30000 --cpu-budget 20 > "$OUT/bench_n5.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- python3 bench.py \
    --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --max-nodes 30000 --no-cpu \
    > "$OUT/trace.log" 2>&1
echo cent profiles done
