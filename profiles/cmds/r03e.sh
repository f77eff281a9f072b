# r03e: min_1_norm benches at the C2 size after the 2-wave L1 kernels
set -o pipefail
timeout -k 10 300 python bench.py --cost l1 --platoons 16384 --steps 5 --warmup 1 --no-cpu --method bnb > gpurun_out/r03e_l1_bnb16k.jsonl 2> gpurun_out/r03e_l1_bnb16k.err || exit 3
timeout -k 10 300 python bench.py --cost l1 --platoons 16384 --steps 3 --warmup 1 --no-cpu --method enum > gpurun_out/r03e_l1_enum16k.jsonl 2> gpurun_out/r03e_l1_enum16k.err || exit 4
timeout -k 10 300 python -u -m pytest tests/test_gpu_l1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e_gputests.log 2>&1 || exit 1
