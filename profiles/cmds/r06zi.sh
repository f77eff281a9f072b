#!/bin/bash
# r06zi: library 75abee51 (the naive-ADMM min_1_norm node LP reaching its LDS buffer through a
# module-scope variable) -- the whole GPU suite and smoke, the same-box naive-ADMM min_1_norm A/B
# against 61861168 (build_prev/), then hash-stamped profiles of the decentralised workloads
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zi
sha256sum hybrid-vehicle-platoon_amd/lib/libhvpsolve.so build_prev/libhvpsolve.so > gpurun_out/${R}_sha.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit 2
for v in new old new old; do
  unset HVP_LIB; [ $v = old ] && export HVP_LIB=$PWD/build_prev/libhvpsolve.so
  timeout -k 10 300 python -u bench.py --controller admm --cost l1 --n 10 --N 10 --platoons 16 --steps 1 --warmup 0 --no-cpu >> gpurun_out/${R}_admm_l1_ab.jsonl 2>> gpurun_out/${R}.err || exit 3
  echo "lib $v" >> gpurun_out/${R}_admm_l1_ab.jsonl
done
unset HVP_LIB
for w in decent_n10_N5_P16384 decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384; do
  timeout -k 10 600 bash profiles/profile_all.sh /tmp/$R $w > gpurun_out/${R}_${w}_prof.log 2>&1 || exit 4
  python3 profiles/summarize.py /tmp/$R/$w $R $w >> gpurun_out/${R}_${w}_prof.log 2>&1 || exit 5
  mkdir -p gpurun_out/${R}_sum && cp profiles/${R}_${w}_summary.json profiles/${R}_${w}_kernel_stats.csv gpurun_out/${R}_sum/ || exit 6
  rm -rf /tmp/$R/$w
done
