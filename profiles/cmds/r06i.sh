#!/bin/bash
# round 6: the N = 3 min_1_norm refill failure on the last green library (round 5's final tree) and
# on this tree (pass-through nodes, the naive-ADMM min_1_norm stall acceptance); then the GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06i
timeout -k 10 120 python -u oldtree/diag_old.py > gpurun_out/${R}_old.log 2>&1 || exit 1
TAG=cur timeout -k 10 120 python -u profiles/diag_l1_small.py > gpurun_out/${R}_cur.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${R}_gpu_tests.txt 2>&1
echo "suite rc=$?" >> gpurun_out/${R}_gpu_tests.txt
