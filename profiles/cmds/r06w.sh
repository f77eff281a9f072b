#!/bin/bash
# round 6: pass-through nodes finished inside the claim (variant library libhvpsolve_pc.so, N = 5
# unit) against the committed form (a pass node holds its lane for one generation) and against no
# pass-through (HVP_PASS_THROUGH=0); C2 default bench, same box; then the parity tests on the variant
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06w
L=$PWD/hybrid-vehicle-platoon_amd/lib
for v in pc cur off pc cur off; do
  unset HVP_LIB HVP_PASS_THROUGH
  case $v in pc) export HVP_LIB=$L/libhvpsolve_pc.so;; off) export HVP_PASS_THROUGH=0;; esac
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_c2_ab.jsonl 2>> gpurun_out/${R}.err || exit 1
  echo "$v done" >> gpurun_out/${R}_c2_ab.jsonl
done
unset HVP_PASS_THROUGH
HVP_LIB=$L/libhvpsolve_pc.so timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_overflow.py -m gpu > gpurun_out/${R}_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/${R}_tests.log
