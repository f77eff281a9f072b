# r05a: switching-ADMM fallback with the active-set polish (hvp_gi.h gi_polish): the gadmm / admm GPU
# tests first, then the whole GPU suite, smoke and the default bench line
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gadmm.py tests/test_admm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05a_admm_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05a_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05a_smoke.log 2>&1 || exit 3
timeout -k 10 300 python bench.py > gpurun_out/r05a_bench_default.jsonl 2> gpurun_out/r05a_bench_default.err || exit 4
