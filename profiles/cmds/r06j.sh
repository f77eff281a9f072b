#!/bin/bash
# round 6: N = 3 min_1_norm refill failure -- which refill setting brings it back
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06j
for cfg in "HVP_LP_REFILL=64" "HVP_LP_REFILL=1" "HVP_LP_INV_BATCH=1" "HVP_LP_INV_BATCH=64" "HVP_LP_REFILL=64 HVP_LP_INV_BATCH=1" "HVP_SPLIT_LEVELS=1 HVP_LP_ROOT_REFILL=0"; do
  env $cfg TAG="$cfg" timeout -k 10 120 python -u profiles/diag_l1_small.py >> gpurun_out/${R}.log 2>&1 || exit 1
done
