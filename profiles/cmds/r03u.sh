# r03u: bucketed level lists 2 vs 4 (HVP_SPLIT_LEVELS), lane-path parity at both, then r03s
# (heavy centralised platoons) and r03t (profile of HEAD with the default 2 buckets)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u_gputests2.log 2>&1 || exit 1
HVP_SPLIT_LEVELS=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u_gputests4.log 2>&1 || exit 2
for r in a b; do
  for nb in 2 4 1; do
    HVP_SPLIT_LEVELS=$nb timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r03u_bench_b${nb}_$r.jsonl 2> gpurun_out/r03u_bench_b${nb}_$r.err || exit 3
  done
done
bash profiles/cmds/r03s.sh || exit 4
bash profiles/cmds/r03t.sh || exit 5
