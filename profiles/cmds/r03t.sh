# r03t: re-profile HEAD (split level lists, centralised early stop): kernel trace + separate PMC
# passes of the default C2 workload and of the centralised C2-size workload, then the default bench
set -o pipefail
bash profiles/run_profiles.sh gpurun_out/r03t/decent_n10_N5 --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 || exit 1
bash profiles/run_profiles.sh gpurun_out/r03t/cent_n10_N5 --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu || exit 2
timeout -k 10 400 python bench.py > gpurun_out/r03t_bench_default.jsonl 2> gpurun_out/r03t_bench_default.err || exit 3
