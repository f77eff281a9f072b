#!/bin/bash
# r06zd: the wave interior point (min_1_norm past N = 8, naive-ADMM min_1_norm) with its row vectors in
# LDS and the Newton matrix assembled in chunks -- L1 GPU tests, then same-box A/B against the round's
# earlier library (build_old/, 249633e6) on decent min_1_norm at N = 10 and naive-ADMM min_1_norm
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zd
sha256sum hybrid-vehicle-platoon_amd/lib/libhvpsolve.so build_old/libhvpsolve.so > gpurun_out/${R}_sha.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_l1.py tests/test_admm_l1.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
for v in new old new old; do
  unset HVP_LIB; [ $v = old ] && export HVP_LIB=$PWD/build_old/libhvpsolve.so
  timeout -k 10 300 python -u bench.py --cost l1 --N 10 --platoons 256 --steps 2 --warmup 1 --no-cpu >> gpurun_out/${R}_l1_N10_ab.jsonl 2>> gpurun_out/${R}.err || exit 2
  echo "lib $v" >> gpurun_out/${R}_l1_N10_ab.jsonl
  timeout -k 10 300 python -u bench.py --controller admm --cost l1 --n 10 --N 10 --platoons 16 --steps 1 --warmup 0 --no-cpu >> gpurun_out/${R}_admm_l1_ab.jsonl 2>> gpurun_out/${R}.err || exit 3
  echo "lib $v" >> gpurun_out/${R}_admm_l1_ab.jsonl
done
