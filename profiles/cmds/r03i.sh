# r03i: trace of the failing bound LP of cent_l1_n3_N6 platoon 0
set -o pipefail
timeout -k 10 120 python -u profiles/cmds/dbg_cent_l1.py 4 100000 cent_l1_n3_N6.npz 0 > gpurun_out/r03i_dbg.log 2>&1 || exit 2
