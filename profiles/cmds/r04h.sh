# r04h: (1) the N = 10 leaf-fallback solve with the interior-point solvers force-inlined (r04g:
# the outlined Solver<10>::solve build hangs), the GPU tests of the parity / overflow / ADMM / API
# files; (2) same-box A/B of where the refill kernel's event reads the workspace descriptor /
# constants (libhvpsolve_v<W><C>: W = 1 workspace by value, C = 1 constants by value; in-tree =
# v00, both through laundered device pointers; _rr = round 4's first root-refill build), default
# bench twice each in rotation; (3) L1: the simplex with rolled term scans (in-tree) vs unrolled
# (_lpu), one and two streams
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
HVP_LEAF_GI_CAP=2 timeout -k 10 45 python -u profiles/cmds/diag_leafcap.py > gpurun_out/r04h_leafcap.jsonl 2> gpurun_out/r04h_leafcap.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gadmm.py tests/test_admm.py tests/test_gpu_api.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04h_tests.log 2>&1 || exit 2
for r in a b; do
  for v in v11 v10 v01 rr; do
    HVP_LIB=$L/libhvpsolve_$v.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04h_bench_${v}_$r.jsonl 2> gpurun_out/r04h_bench_${v}_$r.err || exit 3
  done
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04h_bench_v00_$r.jsonl 2> gpurun_out/r04h_bench_v00_$r.err || exit 4
done
for s in 1 2; do
  timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 --streams $s > gpurun_out/r04h_bench_l1_rolled_s$s.jsonl 2> gpurun_out/r04h_bench_l1_rolled_s$s.err || exit 5
  HVP_LIB=$L/libhvpsolve_lpu.so timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 --streams $s > gpurun_out/r04h_bench_l1_unrolled_s$s.jsonl 2> gpurun_out/r04h_bench_l1_unrolled_s$s.err || exit 6
done
