#!/bin/bash
# r06zn: same-box C2 A/B of the final library (75abee51) against the round's first library (249633e6,
# build_ab/): only the min_1_norm wave interior point changed between them
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zn
for v in new old new old; do
  unset HVP_LIB; [ $v = old ] && export HVP_LIB=$PWD/build_ab/libhvpsolve.so
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_c2_ab.jsonl 2>> gpurun_out/${R}.err || exit 1
  echo "lib $v" >> gpurun_out/${R}_c2_ab.jsonl
done
