# r06b: the full GPU suite with naive-ADMM min_1_norm (tests/test_admm_l1.py) and smoke; then the
# 16-lane cooperative QP at configs[1] (N = 5, -DHVP_COOP_MIN_N=5 build of the N = 5 unit,
# lib/libhvpsolve_coop5.so) against the per-lane refill path, default bench, same box
set -o pipefail
export TMPDIR=/tmp
R=r06b
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${R}_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.txt 2>&1 || exit 2
for lib in coop5 new coop5 new; do
  if [ $lib = coop5 ]; then export HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_coop5.so; else unset HVP_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_coop5_ab.jsonl 2>> gpurun_out/${R}_bench.err || exit 3
  echo "$lib done" >> gpurun_out/${R}_bench_coop5_ab.jsonl
done
