# r03q: full GPU suite + smoke + default bench at HEAD (re-entry check after the container was
# re-created), then the centralised bench with the heaviest searches named and the heaviest
# platoons alone (QP cap 30M, QPs per search depth)
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03q_gputests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03q_smoke.log 2>&1 || exit 2
timeout -k 10 300 python bench.py > gpurun_out/r03q_bench_default.jsonl 2> gpurun_out/r03q_bench.err || exit 3
timeout -k 10 300 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu > gpurun_out/r03q_bench_cent.jsonl 2> gpurun_out/r03q_bench_cent.err || exit 4
HVP_CENT_DEBUG=6 timeout -k 10 400 python profiles/cmds/diag_cent_heavy.py --from-bench gpurun_out/r03q_bench_cent.jsonl --top 3 --max-nodes 30000000 --save gpurun_out/r03q_heavy.npz > gpurun_out/r03q_heavy.jsonl 2> gpurun_out/r03q_heavy.err || exit 5
