# r05za: solve_qp force-inlined into the 16-lane kernels (no outlined coop functions): the GPU tests of the 16-lane
# paths (ADMM forms, long horizons), then same-box A/B of C3 and C4 against the previous library
set -o pipefail
export TMPDIR=/tmp
R=r05za
L=$PWD/hybrid-vehicle-platoon_amd/lib
timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_admm.py tests/test_gadmm.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for lib in new prev new prev; do
  if [ $lib = new ]; then unset HVP_LIB; else export HVP_LIB=$L/libhvpsolve_$lib.so; fi
  timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 2
  echo "admm $lib done" >> gpurun_out/${R}_bench_admm_ab.jsonl
  timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 2 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_gadmm_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 3
  echo "gadmm $lib done" >> gpurun_out/${R}_bench_gadmm_ab.jsonl
done
