# r03l: re-profile HEAD on the default C2 workload (kernel trace + separate PMC passes) + default bench
set -o pipefail
timeout -k 10 300 python bench.py > gpurun_out/r03l_bench_default.jsonl 2> gpurun_out/r03l_bench_default.err || exit 3
bash profiles/run_profiles.sh gpurun_out/r03l/decent_n10_N5 --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 || exit 4
