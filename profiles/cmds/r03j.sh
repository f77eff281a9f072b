# r03j: cent L1 (LP stopping rule + rescue), parity, env, stub tests
set -o pipefail
timeout -k 10 120 python -u profiles/cmds/dbg_cent_l1.py 1 100000 cent_l1_gear_n2_N4.npz 0 > gpurun_out/r03j_dbg.log 2>&1 || exit 2
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_cent.py tests/test_envdev.py tests/test_integration_stub.py "tests/test_admm.py::test_region_hint_is_checked" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03j_gputests.log 2>&1 || exit 1
