# r05g: the LP refill kernel at two waves per SIMD (-DHVP_LP_WAVES=2: 572 B of scratch per lane)
# against one (the shipped build), min_1_norm C2 bench, same box, alternating
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
for r in a b; do
  timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05g_bench_l1_w1_$r.jsonl 2> gpurun_out/r05g_bench_l1_w1_$r.err || exit 1
  HVP_LIB=$L/libhvpsolve_lpw2.so timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05g_bench_l1_w2_$r.jsonl 2> gpurun_out/r05g_bench_l1_w2_$r.err || exit 2
done
