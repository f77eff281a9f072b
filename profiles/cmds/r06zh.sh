#!/bin/bash
# r06zh: the naive-ADMM min_1_norm node LP reaching its LDS buffer through a module-scope variable
# (ds_* instead of flat instructions in the outlined function) -- L1 GPU tests, then same-box A/B
# against the library before it (build_prev/, 61861168)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zh
sha256sum hybrid-vehicle-platoon_amd/lib/libhvpsolve.so build_prev/libhvpsolve.so > gpurun_out/${R}_sha.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_l1.py tests/test_admm_l1.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
for v in new old new old; do
  unset HVP_LIB; [ $v = old ] && export HVP_LIB=$PWD/build_prev/libhvpsolve.so
  timeout -k 10 300 python -u bench.py --controller admm --cost l1 --n 10 --N 10 --platoons 16 --steps 1 --warmup 0 --no-cpu >> gpurun_out/${R}_admm_l1_ab.jsonl 2>> gpurun_out/${R}.err || exit 3
  echo "lib $v" >> gpurun_out/${R}_admm_l1_ab.jsonl
done
