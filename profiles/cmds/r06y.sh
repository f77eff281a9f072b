#!/bin/bash
# r06y: the round's library -- the whole GPU suite and smoke, then the hash-stamped PMC profiles of
# the decentralised workloads (one stream, the timed three-stream configuration, min_1_norm) that
# bench.py's roofline reads (summarised with profiles/summarize.py)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06y
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit 2
timeout -k 10 900 bash profiles/profile_all.sh gpurun_out/$R decent_n10_N5_P16384 decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384 > gpurun_out/${R}_prof.log 2>&1 || exit 3
