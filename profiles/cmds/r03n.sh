# r03n: branch-free most-violated scan: default bench + decentralised parity tests
set -o pipefail
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03n_bench.jsonl 2> gpurun_out/r03n_bench.err || exit 3
timeout -k 10 300 python bench.py --no-cpu --streams 1 > gpurun_out/r03n_bench_s1.jsonl 2>> gpurun_out/r03n_bench.err || exit 4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03n_gputests.log 2>&1 || exit 1
