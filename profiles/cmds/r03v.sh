# r03v: same-box A/B of the library before the bucketed level lists (6d25a76, lib/libhvpsolve_old.so)
# against HEAD (4 buckets): default bench twice each, and a kernel trace of each (root kernel time)
set -o pipefail
export TMPDIR=/tmp
OLD=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_old.so
for r in a b; do
  HVP_LIB=$OLD timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03v_bench_old_$r.jsonl 2> gpurun_out/r03v_bench_old_$r.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03v_bench_new_$r.jsonl 2> gpurun_out/r03v_bench_new_$r.err || exit 2
done
HVP_LIB=$OLD timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r03v/old -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r03v_trace_old.log 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r03v/new -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r03v_trace_new.log 2>&1 || exit 4
