# r04i: the whole GPU suite + smoke at HEAD (interior-point solvers inlined), then the same-box
# A/B of the refill event's argument variants (see r04h.sh) and the L1 simplex rolled / unrolled
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
for r in a b; do
  for v in v11 v10 v01 rr; do
    HVP_LIB=$L/libhvpsolve_$v.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04i_bench_${v}_$r.jsonl 2> gpurun_out/r04i_bench_${v}_$r.err || exit 3
  done
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04i_bench_v00_$r.jsonl 2> gpurun_out/r04i_bench_v00_$r.err || exit 4
done
# L1: node LPs through the refill kernel (default, refill at 32 free lanes) on one and two streams,
# its refill threshold, the grid-stride kernel (HVP_LP_REFILL=0), the wave interior point
for s in 1 2; do
  timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 --streams $s > gpurun_out/r04i_bench_l1_refill32_s$s.jsonl 2> gpurun_out/r04i_bench_l1_refill32_s$s.err || exit 5
done
for m in 0 16 48; do
  HVP_LP_REFILL=$m timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 --streams 1 > gpurun_out/r04i_bench_l1_refill${m}_s1.jsonl 2> gpurun_out/r04i_bench_l1_refill${m}_s1.err || exit 6
done
HVP_LP_ROOT_REFILL=0 timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 --streams 1 > gpurun_out/r04i_bench_l1_rootkernel_s1.jsonl 2> gpurun_out/r04i_bench_l1_rootkernel_s1.err || exit 8
HVP_L1_SIMPLEX=0 timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 > gpurun_out/r04i_bench_l1_ipm_s2.jsonl 2> gpurun_out/r04i_bench_l1_ipm_s2.err || exit 7
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r04i_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04i_smoke.log 2>&1 || exit 12
