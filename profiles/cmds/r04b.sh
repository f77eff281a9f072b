# r04b: (1) the root level through the refill kernel (k_inst_prep root nodes, refill at k = 0, dive
# list at K = N), (2) the refill kernel's event constants through laundered device pointers (scratch
# 140 -> 24 B/lane, SGPR lane spills 128 -> 38), (3) keyed switching-ADMM warm records, (4) interior-
# point fallback of the naive / switching ADMM QPs, (5) min_1_norm LPs by the per-lane simplex.
# Same-box A/B of the default bench first (libhvpsolve_r03.so = round 3's HEAD, _rr = (1) only, the
# in-tree build = all), kernel traces, the L1 bench against the wave interior point, then the GPU
# tests (verbose, 150 s per test: a slow test names itself and dumps its stacks).
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
for r in a b; do
  HVP_LIB=$L/libhvpsolve_r03.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04b_bench_r03_$r.jsonl 2> gpurun_out/r04b_bench_r03_$r.err || exit 2
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04b_bench_new_$r.jsonl 2> gpurun_out/r04b_bench_new_$r.err || exit 3
  HVP_LIB=$L/libhvpsolve_rr.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04b_bench_rr_$r.jsonl 2> gpurun_out/r04b_bench_rr_$r.err || exit 4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r04b_trace_new -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r04b_trace_new.log 2>&1 || exit 6
HVP_LIB=$L/libhvpsolve_r03.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r04b_trace_r03 -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r04b_trace_r03.log 2>&1 || exit 7
timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 5 --warmup 1 > gpurun_out/r04b_bench_l1_simplex.jsonl 2> gpurun_out/r04b_bench_l1_simplex.err || exit 9
HVP_L1_SIMPLEX=0 timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 5 --warmup 1 > gpurun_out/r04b_bench_l1_ipm.jsonl 2> gpurun_out/r04b_bench_l1_ipm.err || exit 10
timeout -k 10 400 python -u -m pytest tests/test_gpu_l1.py tests/test_envdev.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r04b_l1_tests.log 2>&1 || exit 8
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gadmm.py tests/test_admm.py tests/test_gpu_api.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 || exit 1
