# r03y: LevelList / reservation loops over the static bucket count (refill scratch 192 -> 140 B):
# lane-path GPU parity, same-box A/B against the library before the buckets, kernel trace
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03y_gputests.log 2>&1 || exit 1
OLD=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_old.so
for r in a b; do
  HVP_LIB=$OLD timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03y_bench_old_$r.jsonl 2> gpurun_out/r03y_bench_old_$r.err || exit 2
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03y_bench_new_$r.jsonl 2> gpurun_out/r03y_bench_new_$r.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r03y/new -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r03y_trace_new.log 2>&1 || exit 4
