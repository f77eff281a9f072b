#!/bin/bash
# r06ze: the round's final library (wave interior point with LDS row vectors) -- the whole GPU suite and
# smoke, then hash-stamped PMC profiles of the decentralised workloads, summarised on the box
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06ze
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit 2
for w in decent_n10_N5_P16384 decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384; do
  timeout -k 10 600 bash profiles/profile_all.sh /tmp/$R $w > gpurun_out/${R}_${w}_prof.log 2>&1 || exit 3
  python3 profiles/summarize.py /tmp/$R/$w $R $w >> gpurun_out/${R}_${w}_prof.log 2>&1 || exit 4
  mkdir -p gpurun_out/${R}_sum && cp profiles/${R}_${w}_summary.json profiles/${R}_${w}_kernel_stats.csv gpurun_out/${R}_sum/ || exit 5
  rm -rf /tmp/$R/$w
done
