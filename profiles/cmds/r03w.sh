# r03w: same-box A/B after moving the root's children to bucket 0 and the segments to shifts:
# library before the level buckets (6d25a76) vs HEAD with 4 and 2 buckets; kernel trace of HEAD
set -o pipefail
export TMPDIR=/tmp
OLD=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_old.so
for r in a b; do
  HVP_LIB=$OLD timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03w_bench_old_$r.jsonl 2> gpurun_out/r03w_bench_old_$r.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03w_bench_b4_$r.jsonl 2> gpurun_out/r03w_bench_b4_$r.err || exit 2
  HVP_SPLIT_LEVELS=2 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03w_bench_b2_$r.jsonl 2> gpurun_out/r03w_bench_b2_$r.err || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r03w/new -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r03w_trace_new.log 2>&1 || exit 4
