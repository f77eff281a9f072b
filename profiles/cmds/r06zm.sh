# r06zm: C5 sweep (12 (n, N) points x 100 seeds x 50 steps) on the round's final library 75abee51
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=r06zm
PYTHONPATH=$PWD/hybrid-vehicle-platoon_amd timeout -k 10 600 python -u -m hvp.sweep --ep-len 50 > gpurun_out/${R}_sweep_c5.jsonl 2> gpurun_out/${R}_sweep_c5.err || exit 1
