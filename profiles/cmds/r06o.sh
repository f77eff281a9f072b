#!/bin/bash
# round 6: same-box A/B of round 5's final tree (oldtree/: its bench.py, package and library, built
# from commit 890d640) against this tree: the min_1_norm line and C2
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06o
for t in old new old new; do
  if [ $t = old ]; then B=oldtree/bench.py; else B=bench.py; fi
  timeout -k 10 300 python $B --cost l1 --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_l1_ab.jsonl 2>> gpurun_out/${R}.err || exit 1
  echo "$t done" >> gpurun_out/${R}_l1_ab.jsonl
done
for t in old new old new; do
  if [ $t = old ]; then B=oldtree/bench.py; else B=bench.py; fi
  timeout -k 10 300 python $B --steps 10 --warmup 2 --no-cpu --no-roofline-pass >> gpurun_out/${R}_c2_ab.jsonl 2>> gpurun_out/${R}.err || exit 2
  echo "$t done" >> gpurun_out/${R}_c2_ab.jsonl
done
