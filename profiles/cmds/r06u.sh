#!/bin/bash
# round 6: kernel traces of C3 with the incumbent leaves as a list (k_bnb_leaf_coop) and inline
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06u
for ll in 1 0; do
  HVP_COOP_LEAF_LIST=$ll timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${R}_ll$ll -o run -- python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 2 --warmup 1 --no-cpu --no-roofline-pass > gpurun_out/${R}_ll$ll.log 2>&1 || exit 1
done
