# r04q: the C5 sweep (12 (n, N) points x 100 seeds x 50 steps as one job) on the shipped library,
# as r02w measured it
set -o pipefail
export TMPDIR=/tmp
PYTHONPATH=$PWD/hybrid-vehicle-platoon_amd timeout -k 10 600 python -u -m hvp.sweep --ep-len 50 > gpurun_out/r04q_sweep_c5.jsonl 2> gpurun_out/r04q_sweep_c5.err || exit 1
