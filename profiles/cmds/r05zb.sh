# r05zb: same-box A/B of the C2 headline: the round's final library (prev = d9d54767), the same
# sources without the bucket spill (-DHVP_SPILL=0), and the round-5 mid-round library dc99c3ae
set -o pipefail
export TMPDIR=/tmp
R=r05zb
L=$PWD/hybrid-vehicle-platoon_amd/lib
for v in prev nospill old prev nospill old; do
  if [ $v = old ]; then D=build_oldpkg; unset HVP_LIB; else D=.; export HVP_LIB=$L/libhvpsolve_$v.so; fi
  (cd $D && timeout -k 10 300 python bench.py --no-cpu --no-roofline-pass) >> gpurun_out/${R}_bench_default_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 1
  echo "c2 $v done" >> gpurun_out/${R}_bench_default_ab.jsonl
done
