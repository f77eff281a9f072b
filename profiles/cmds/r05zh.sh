# r05zh: C5 sweep (12 (n, N) points x 100 seeds x 50 steps) on the round's final library -- the
# decentralised 16-lane path at N = 10 / 15 after the warm-start changes of the shared solver
set -o pipefail
export TMPDIR=/tmp
R=r05zh
PYTHONPATH=$PWD/hybrid-vehicle-platoon_amd timeout -k 10 600 python -u -m hvp.sweep --ep-len 50 > gpurun_out/${R}_sweep_c5.jsonl 2> gpurun_out/${R}_sweep_c5.err || exit 1
