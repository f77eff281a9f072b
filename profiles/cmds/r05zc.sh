# r05zc: the round's library -- the whole GPU suite and smoke, then the hash-stamped PMC profiles of
# the decentralised workloads (one stream, the timed three-stream configuration, min_1_norm) that
# bench.py's roofline reads (summarised with profiles/summarize.py)
set -o pipefail
export TMPDIR=/tmp
R=r05zc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass > gpurun_out/${R}_bench_admm_quick.jsonl 2>&1 || exit 4
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit 2
timeout -k 10 1000 bash profiles/profile_all.sh gpurun_out/$R decent_n10_N5_P16384 decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384 > gpurun_out/${R}_prof.log 2>&1 || exit 3
L=$PWD/hybrid-vehicle-platoon_amd/lib
for v in final prev old final prev old; do
  if [ $v = old ]; then D=build_oldpkg; unset HVP_LIB; elif [ $v = prev ]; then D=.; export HVP_LIB=$L/libhvpsolve_prev.so; else D=.; unset HVP_LIB; fi
  (cd $D && timeout -k 10 300 python bench.py --no-cpu --no-roofline-pass) >> gpurun_out/${R}_bench_default_ab.jsonl 2>> gpurun_out/${R}_bench_ab.err || exit 5
  echo "c2 $v done" >> gpurun_out/${R}_bench_default_ab.jsonl
done
