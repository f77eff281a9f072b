# r03k: cent tests (alternative-optimum check for min_1_norm faces)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_cent.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03k_gputests.log 2>&1 || exit 1
