#!/bin/bash
# round 6: the min_1_norm line's 6 % regression against round 5 (r06o): round 5's tree, the committed
# hvp_lane.h (vA, N = 5 unit), this tree with the committed LP refill kernel (vE, one list), this tree
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06p
L=$PWD/hybrid-vehicle-platoon_amd/lib
for t in old vA vE new old vA vE new; do
  B=bench.py; unset HVP_LIB HVP_SPLIT_LEVELS
  case $t in old) B=oldtree/bench.py;; vA) export HVP_LIB=$L/libhvpsolve_vA.so;; vE) export HVP_LIB=$L/libhvpsolve_vE.so HVP_SPLIT_LEVELS=1;; esac
  timeout -k 10 300 python $B --cost l1 --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_l1_ab.jsonl 2>> gpurun_out/${R}.err || exit 1
  echo "$t done" >> gpurun_out/${R}_l1_ab.jsonl
done
