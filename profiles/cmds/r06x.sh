#!/bin/bash
# round 6: pass-through nodes compacted out of each level before the refill kernel (k_level_compact,
# variant library libhvpsolve_cmp.so = this tree's N = 5 unit): parity tests with the pass-through
# nodes on, then same-box C2 A/B: variant on / variant off / committed library (base) off
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06x
L=$PWD/hybrid-vehicle-platoon_amd/lib
HVP_PASS_THROUGH=1 HVP_LIB=$L/libhvpsolve_cmp.so timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_overflow.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for v in on off base on off base; do
  unset HVP_PASS_THROUGH; export HVP_LIB=$L/libhvpsolve_cmp.so
  case $v in on) export HVP_PASS_THROUGH=1;; base) export HVP_LIB=$L/libhvpsolve_base.so;; esac
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_c2_ab.jsonl 2>> gpurun_out/${R}.err || exit 2
  echo "$v done" >> gpurun_out/${R}_c2_ab.jsonl
done
