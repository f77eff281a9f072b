# r04j: same-box A/B of the refill kernel's round-3 body (descriptor and constants by value, level
# list hoisted; libhvpsolve_vr3) against the in-tree laundered one and round 4's first root-refill
# build (libhvpsolve_rr), default bench three times each in rotation
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
for r in a b c; do
  for v in vr3 rr; do
    HVP_LIB=$L/libhvpsolve_$v.so timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04j_bench_${v}_$r.jsonl 2> gpurun_out/r04j_bench_${v}_$r.err || exit 2
  done
  timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r04j_bench_v00_$r.jsonl 2> gpurun_out/r04j_bench_v00_$r.err || exit 3
done
