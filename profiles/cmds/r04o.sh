# r04o: final check of the tree: the whole GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04o_smoke.log 2>&1 || exit 2
