#!/bin/bash
# round 6: the C3 root level with its incumbent leaves as a list of their own (k_bnb_leaf_coop):
# ADMM + long-horizon tests, then same-box A/B of C3 against the inline leaves (HVP_COOP_LEAF_LIST=0)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06t
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_admm.py tests/test_sweep.py tests/test_gpu_overflow.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for ll in 1 0 1 0; do
  HVP_COOP_LEAF_LIST=$ll timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 2
  echo "leaf_list $ll done" >> gpurun_out/${R}_bench_admm_ab.jsonl
done
