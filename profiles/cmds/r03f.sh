# r03f: centralised min_1_norm, env lin_cost, region hint checks, small task budget, N > 8 leaf fallback
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_cent.py tests/test_envdev.py tests/test_integration_stub.py "tests/test_admm.py::test_region_hint_is_checked" tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "not cent_l1_n4_N5" > gpurun_out/r03f_gputests.log 2>&1 || exit 1
