# r06f: diagnosis of the min_1_norm N = 3 status regression (pivot buckets on vs one list,
# HVP_SPLIT_LEVELS=1), the naive-ADMM min_1_norm tests with the tightened interior-point test, and
# the same-box A/Bs: 16-lane cooperative QP at configs[1] (coop5 build) vs the per-lane refill path
set -o pipefail
export TMPDIR=/tmp
R=r06f
HVP_SPLIT_LEVELS=1 timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_l1.py -m gpu > gpurun_out/${R}_l1_split1.txt 2>&1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_l1.py -m gpu -k "branch_and_bound_fixture" > gpurun_out/${R}_l1_default.txt 2>&1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_admm_l1.py -m gpu > gpurun_out/${R}_admm_l1.txt 2>&1
for lib in coop5 new coop5 new; do
  if [ $lib = coop5 ]; then export HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_coop5.so; else unset HVP_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_coop5_ab.jsonl 2>> gpurun_out/${R}_bench.err || exit 4
  echo "$lib done" >> gpurun_out/${R}_bench_coop5_ab.jsonl
done
