# r05d: straggler eviction in the QP refill kernel (HVP_REFILL_EVICT, restart-style requeue): the
# decentralised parity / overflow / root-refill tests, then a same-box A/B of the default bench over
# the eviction threshold (0 = off), alternating twice
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gpu_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1 || exit 1
for r in a b; do
  for e in 0 2 4 8; do
    HVP_REFILL_EVICT=$e timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r05d_bench_e${e}_$r.jsonl 2> gpurun_out/r05d_bench_e${e}_$r.err || exit 2
  done
done
HVP_REFILL_EVICT=0 timeout -k 10 300 python bench.py --no-cpu --streams 1 > gpurun_out/r05d_bench_e0_s1.jsonl 2> gpurun_out/r05d_bench_e0_s1.err || exit 3
HVP_REFILL_EVICT=4 timeout -k 10 300 python bench.py --no-cpu --streams 1 > gpurun_out/r05d_bench_e4_s1.jsonl 2> gpurun_out/r05d_bench_e4_s1.err || exit 4
