# r06e: the GPU suite without the naive-ADMM min_1_norm file (its tolerance fix is building) and smoke;
# A/B on one box: (a) the 16-lane cooperative QP at configs[1] (-DHVP_COOP_MIN_N=5 build of the N = 5
# unit) against the per-lane refill path, (b) the min_1_norm line with the pivot buckets against one
# list (HVP_SPLIT_LEVELS=1)
set -o pipefail
export TMPDIR=/tmp
R=r06e
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu --deselect tests/test_admm_l1.py > gpurun_out/${R}_gpu_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.txt 2>&1 || exit 2
for lib in coop5 new coop5 new; do
  if [ $lib = coop5 ]; then export HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_coop5.so; else unset HVP_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_coop5_ab.jsonl 2>> gpurun_out/${R}_bench.err || exit 4
  echo "$lib done" >> gpurun_out/${R}_bench_coop5_ab.jsonl
done
unset HVP_LIB
for sp in 2 1 2 1; do
  HVP_SPLIT_LEVELS=$sp timeout -k 10 300 python bench.py --cost l1 --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_l1_split_ab.jsonl 2>> gpurun_out/${R}_bench.err || exit 5
  echo "split $sp done" >> gpurun_out/${R}_bench_l1_split_ab.jsonl
done
