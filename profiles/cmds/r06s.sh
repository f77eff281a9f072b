#!/bin/bash
# round 6: GPU suite + smoke after reverting the min_1_norm LP buckets (the LP refill kernel of round
# 5) and keeping the naive-ADMM min_1_norm interior point's best loose iterate; the min_1_norm and C2
# lines (one sample each)
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06s
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${R}_gpu_tests.txt 2>&1
echo "suite rc=$?" >> gpurun_out/${R}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.txt 2>&1 || exit 2
timeout -k 10 300 python bench.py --cost l1 --steps 10 --warmup 2 --no-cpu --no-roofline-pass > gpurun_out/${R}_bench_l1.jsonl 2>> gpurun_out/${R}.err || exit 3
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-roofline-pass > gpurun_out/${R}_bench_c2.jsonl 2>> gpurun_out/${R}.err || exit 4
