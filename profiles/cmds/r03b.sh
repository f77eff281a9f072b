set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_l1.py tests/test_integration_stub.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03b_gputests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --cost l1 --platoons 4096 --steps 5 --warmup 1 --no-cpu --method enum > gpurun_out/r03b_l1_enum.jsonl 2> gpurun_out/r03b_l1_enum.err || exit 2
timeout -k 10 200 python bench.py --cost l1 --platoons 4096 --steps 5 --warmup 1 --no-cpu --method bnb > gpurun_out/r03b_l1_bnb.jsonl 2> gpurun_out/r03b_l1_bnb.err || exit 3
timeout -k 10 200 python bench.py --cost l1 --N 10 --platoons 1024 --steps 2 --warmup 1 --no-cpu > gpurun_out/r03b_l1_N10.jsonl 2> gpurun_out/r03b_l1_N10.err || exit 4
