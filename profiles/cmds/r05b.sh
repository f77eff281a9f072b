# r05b: the switching-ADMM polish (gadmm/admm GPU tests), the one-scan-per-trip simplex (L1 GPU tests),
# the whole GPU suite + smoke, the default bench line, then the L1 bench over the rebuild batch and
# the refill threshold
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gadmm.py tests/test_admm.py tests/test_gpu_l1.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05b_admm_l1_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05b_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05b_smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r05b_bench_default.jsonl 2> gpurun_out/r05b_bench_default.err || exit 4
for b in 12 8 16 24; do
  HVP_LP_INV_BATCH=$b timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05b_bench_l1_inv$b.jsonl 2> gpurun_out/r05b_bench_l1_inv$b.err || exit 5
done
for m in 16 48; do
  HVP_LP_REFILL=$m timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05b_bench_l1_refill$m.jsonl 2> gpurun_out/r05b_bench_l1_refill$m.err || exit 6
done
