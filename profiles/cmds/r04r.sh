# r04r: same-box A/B of the C5 sweep's N = 15 points (r04q: 9-17 % below round 2's r02w on another
# box): round 3's library (libhvpsolve_r03, built from 73d8649) vs the shipped one, alternating
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
for r in a b; do
  HVP_LIB=$L/libhvpsolve_r03.so PYTHONPATH=$PWD/hybrid-vehicle-platoon_amd timeout -k 10 300 python -u -m hvp.sweep --N 15 --ep-len 50 > gpurun_out/r04r_sweep_N15_r03_$r.jsonl 2> gpurun_out/r04r_sweep_N15_r03_$r.err || exit 1
  PYTHONPATH=$PWD/hybrid-vehicle-platoon_amd timeout -k 10 300 python -u -m hvp.sweep --N 15 --ep-len 50 > gpurun_out/r04r_sweep_N15_new_$r.jsonl 2> gpurun_out/r04r_sweep_N15_new_$r.err || exit 2
done
