#!/bin/bash
# r06zj: hash-stamped PMC profiles of library 75abee51 for C3, C4, the centralised bench and the
# naive-ADMM min_1_norm line, summarised on the box
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zj
for w in admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096 admm_n10_N10_l1_P32; do
  timeout -k 10 600 bash profiles/profile_all.sh /tmp/$R $w > gpurun_out/${R}_${w}_prof.log 2>&1 || exit 3
  python3 profiles/summarize.py /tmp/$R/$w $R $w >> gpurun_out/${R}_${w}_prof.log 2>&1 || exit 4
  mkdir -p gpurun_out/${R}_sum && cp profiles/${R}_${w}_summary.json profiles/${R}_${w}_kernel_stats.csv gpurun_out/${R}_sum/ || exit 5
  rm -rf /tmp/$R/$w
done
