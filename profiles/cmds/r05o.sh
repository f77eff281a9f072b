# r05o: k_node_order (warm-started nodes of a level first): ADMM GPU tests, then same-box A/B of C3
# with and without the order (HVP_ADMM_NODE_ORDER=0)
set -o pipefail
export TMPDIR=/tmp
R=r05o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_admm.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for o in 1 0 1 0; do
  HVP_ADMM_NODE_ORDER=$o timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_ab.jsonl 2>> gpurun_out/${R}_bench_admm_ab.err || exit 2
  echo "order $o done" >> gpurun_out/${R}_bench_admm_ab.jsonl
done
