# r05f: the per-instance QP part instance-major (AoS, one padded row per instance) against the
# field-major layout (libhvpsolve_base.so): decentralised parity tests, same-box A/B of the default
# bench, and HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of a one-stream run of each
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1 || exit 1
for r in a b; do
  HVP_LIB=$L/libhvpsolve_base.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r05f_bench_base_$r.jsonl 2> gpurun_out/r05f_bench_base_$r.err || exit 2
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r05f_bench_aos_$r.jsonl 2> gpurun_out/r05f_bench_aos_$r.err || exit 3
done
for v in base aos; do
  if [ $v = base ]; then export HVP_LIB=$L/libhvpsolve_base.so; else unset HVP_LIB; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c -T -f csv -d gpurun_out/r05f_pmc_${v}_$c -o run -- python3 bench.py --platoons 16384 --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/r05f_pmc_${v}_$c.log 2>&1 || exit 4
  done
done
unset HVP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r05f_trace_aos -o run -- python3 bench.py --platoons 16384 --steps 3 --warmup 1 --no-cpu --streams 1 > gpurun_out/r05f_trace_aos.log 2>&1 || exit 5
