# r04f: k_bnb_ipm split into its decentralised and ADMM kernels; the leaf-cap solve that hung in
# r04b / r04e, then the GPU tests of the parity / overflow / ADMM / API files
set -o pipefail
export TMPDIR=/tmp
HVP_LEAF_GI_CAP=2 timeout -k 10 60 python -u profiles/cmds/diag_leafcap.py > gpurun_out/r04f_leafcap.jsonl 2> gpurun_out/r04f_leafcap.err || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_overflow.py tests/test_gadmm.py tests/test_admm.py tests/test_gpu_api.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1 || exit 2
