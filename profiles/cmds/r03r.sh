# r03r: (1) centralised early stop (dual bound past the incumbent): cent GPU tests, the C2-size
# cent bench with it (r03q = without), QPs per search depth of the two heaviest platoons;
# (2) decentralised level lists in two halves by the parent's active-set steps: lane parity /
# overflow tests and the default bench with and without (HVP_SPLIT_LEVELS=0)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_cent.py tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r_gputests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03r_bench_split.jsonl 2> gpurun_out/r03r_bench_split.err || exit 2
HVP_SPLIT_LEVELS=0 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03r_bench_nosplit.jsonl 2> gpurun_out/r03r_bench_nosplit.err || exit 3
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03r_bench_split2.jsonl 2> gpurun_out/r03r_bench_split2.err || exit 4
timeout -k 10 300 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu > gpurun_out/r03r_bench_cent.jsonl 2> gpurun_out/r03r_bench_cent.err || exit 5
HVP_CENT_DEBUG=6 timeout -k 10 240 python profiles/cmds/diag_cent_heavy.py --seeds 426 3139 --max-nodes 2000000 > gpurun_out/r03r_heavy.jsonl 2> gpurun_out/r03r_heavy.err || exit 6
# (3) the refill kernel at 3 waves per SIMD (168 VGPRs, 492 B/lane scratch), same source
HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_w3.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03r_bench_w3.jsonl 2> gpurun_out/r03r_bench_w3.err || exit 7
