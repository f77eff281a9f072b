#!/bin/bash
# round 6: GPU suite + smoke on this tree (pass-through nodes, LP refill level lists in buckets via
# level_slot, naive-ADMM min_1_norm stall acceptance); same-box A/B: (a) C2 with / without the
# pass-through nodes (HVP_PASS_THROUGH=0), (b) the min_1_norm line with the pivot buckets against one
# list (HVP_SPLIT_LEVELS=1)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06n
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${R}_gpu_tests.txt 2>&1
echo "suite rc=$?" >> gpurun_out/${R}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.txt 2>&1 || exit 2
for pt in 1 0 1 0; do
  HVP_PASS_THROUGH=$pt timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_pass_ab.jsonl 2>> gpurun_out/${R}_bench.err || exit 3
  echo "pass $pt done" >> gpurun_out/${R}_bench_pass_ab.jsonl
done
for sp in 2 1 2 1; do
  HVP_SPLIT_LEVELS=$sp timeout -k 10 300 python bench.py --cost l1 --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_l1_split_ab.jsonl 2>> gpurun_out/${R}_bench.err || exit 4
  echo "split $sp done" >> gpurun_out/${R}_bench_l1_split_ab.jsonl
done
