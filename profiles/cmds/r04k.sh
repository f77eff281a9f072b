# r04k: the shipped library (refill kernel by value, HVP_REFILL_BYVAL): r04d part 1 (C2 decent and
# min_1_norm profiles + bench lines), then the whole GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
bash profiles/cmds/r04d.sh r04k 1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04k_smoke.log 2>&1 || exit 12
