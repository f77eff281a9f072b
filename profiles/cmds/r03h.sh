# r03h: cent L1 node-count trace + parity/cent tests after the certified-infeasible leaf change
set -o pipefail
timeout -k 10 120 python -u profiles/cmds/dbg_cent_l1.py 1 100000 cent_l1_n3_N6.npz 0 > gpurun_out/r03h_dbg.log 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cent.py -m gpu -v --timeout 300 --timeout-method thread -k "not cent_l1_n4_N5" > gpurun_out/r03h_gputests.log 2>&1 || exit 1
