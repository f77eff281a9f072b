#!/bin/bash
# r06zb: the naive-ADMM min_1_norm closed loop (C3 shape with quadratic_cost=False) at small batches,
# with a heartbeat file (the bench prints only at its end)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zb
(while true; do date +%T >> gpurun_out/${R}_heartbeat.txt; sleep 50; done) &
HB=$!
for P in 16 64; do
  timeout -k 10 400 python bench.py --controller admm --cost l1 --n 10 --N 10 --platoons $P --steps 1 --warmup 0 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_l1.jsonl 2>> gpurun_out/${R}.err || { kill $HB; exit 1; }
  echo "P $P done $(date +%T)" >> gpurun_out/${R}_bench_admm_l1.jsonl
done
kill $HB
