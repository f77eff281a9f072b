# r03c: full GPU suite after the min_1_norm branch and bound; L1 benches at the C2 size
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03c_gputests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03c_smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py --cost l1 --platoons 16384 --steps 5 --warmup 1 --no-cpu --method bnb > gpurun_out/r03c_l1_bnb16k.jsonl 2> gpurun_out/r03c_l1_bnb16k.err || exit 3
timeout -k 10 300 python bench.py --cost l1 --platoons 16384 --steps 3 --warmup 1 --no-cpu --method enum > gpurun_out/r03c_l1_enum16k.jsonl 2> gpurun_out/r03c_l1_enum16k.err || exit 4
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r03c_default.jsonl 2> gpurun_out/r03c_default.err || exit 5
