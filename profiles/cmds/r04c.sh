# r04c: the whole GPU suite and smoke() on the current library
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r04c_gputests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04c_smoke.log 2>&1 || exit 2
