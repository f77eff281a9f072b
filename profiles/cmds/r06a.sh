# r06a: warm-record write-back skipped when the warm start needed no add / drop (hvp_coop.h solve):
# ADMM / switching-ADMM GPU tests, then C3 and C4 bench lines against round 5's library (HVP_LIB,
# rebuilt from commit bfd061e's sources with the ABI-5 header, same box)
set -o pipefail
export TMPDIR=/tmp
R=r06a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_admm.py tests/test_gadmm.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for lib in new old new old; do
  if [ $lib = old ]; then export HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_prev.so; else unset HVP_LIB; fi
  timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 2
  echo "admm $lib done" >> gpurun_out/${R}_bench_admm_ab.jsonl
  timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 2 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_gadmm_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 3
  echo "gadmm $lib done" >> gpurun_out/${R}_bench_gadmm_ab.jsonl
done
