# r03p: warm-start equality test + PMC profile of the C4 workload after the switching-ADMM warm start
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gadmm.py -m gpu -x -q -k warm_start --timeout 240 --timeout-method thread > gpurun_out/r03p_gputests.log 2>&1 || exit 1
bash profiles/run_profiles.sh gpurun_out/r03p/gadmm_n20_N10 --controller gadmm --n 20 --N 10 --platoons 2048 --steps 1 --warmup 0 --no-cpu || exit 4
timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 1 --warmup 1 --no-cpu > gpurun_out/r03p_bench_gadmm.jsonl 2> gpurun_out/r03p_bench.err || exit 3
