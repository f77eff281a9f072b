#!/bin/bash
# r06zc: the refill threshold re-swept on round 6's kernel (N = 5 unit built with -DHVP_REFILL_MIN=48 / 56;
# shipped: 64, generations of 64 nodes), C2 default bench, same box
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zc
L=$PWD/hybrid-vehicle-platoon_amd/lib
for v in 64 48 56 64 48 56; do
  unset HVP_LIB; [ $v != 64 ] && export HVP_LIB=$L/libhvpsolve_rm$v.so
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_c2_ab.jsonl 2>> gpurun_out/${R}.err || exit 1
  echo "min $v done" >> gpurun_out/${R}_c2_ab.jsonl
done
