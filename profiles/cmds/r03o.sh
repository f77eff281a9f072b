# r03o: switching ADMM warm start (hinge states + active set + factors) across ADMM iterations: A/B bench at C4 + gadmm tests
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gadmm.py tests/test_admm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03o_gputests.log 2>&1 || exit 1
HVP_GADMM_WARM=0 timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 1 --warmup 1 --no-cpu > gpurun_out/r03o_bench_cold.jsonl 2> gpurun_out/r03o_bench.err || exit 3
timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 1 --warmup 1 --no-cpu > gpurun_out/r03o_bench_warm.jsonl 2>> gpurun_out/r03o_bench.err || exit 4
