#!/bin/bash
# round 6: C3 on one engine (--streams 1): kernel trace and the lane-utilisation counters with the
# incumbent leaves as a list (k_bnb_leaf_coop) and inline (HVP_COOP_LEAF_LIST=0)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06v
B="python bench.py --controller admm --n 10 --N 10 --platoons 512 --streams 1 --steps 1 --warmup 1 --no-cpu --no-roofline-pass"
for ll in 1 0; do
  export HVP_COOP_LEAF_LIST=$ll
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${R}_ll$ll/trace -o run -- $B > gpurun_out/${R}_ll${ll}_trace.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU -T -f csv -d gpurun_out/${R}_ll$ll/occ -o run -- $B > gpurun_out/${R}_ll${ll}_occ.log 2>&1 || exit 2
done
