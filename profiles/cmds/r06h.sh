#!/bin/bash
# round 6: bisect the N = 3 min_1_norm refill regression (variant libraries of the N = 3 unit)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "" _vA _vB; do
  HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve$v.so TAG="lib$v" timeout -k 10 120 python -u profiles/diag_l1_small.py || exit 1
done
