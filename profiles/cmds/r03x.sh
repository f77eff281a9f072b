# r03x: HEAD (2 buckets by default, root children in bucket 0, per-bucket loops in key / write):
# full GPU suite, smoke, a same-box A/B against the library before the buckets, the re-profile of
# HEAD (decent C2 and cent C2-size workloads: kernel trace + separate PMC passes), default bench
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03x_gputests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03x_smoke.log 2>&1 || exit 2
OLD=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_old.so
HVP_LIB=$OLD timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03x_bench_old.jsonl 2> gpurun_out/r03x_bench_old.err || exit 3
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03x_bench_new.jsonl 2> gpurun_out/r03x_bench_new.err || exit 4
bash profiles/run_profiles.sh gpurun_out/r03x/decent_n10_N5 --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 || exit 5
bash profiles/run_profiles.sh gpurun_out/r03x/cent_n10_N5 --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu || exit 6
timeout -k 10 400 python bench.py > gpurun_out/r03x_bench_default.jsonl 2> gpurun_out/r03x_bench_default.err || exit 7
