# r03g: centralised min_1_norm LP trace (first LPs of one platoon)
set -o pipefail
timeout -k 10 120 python -u profiles/cmds/dbg_cent_l1.py 5 1 > gpurun_out/r03g_lp1.log 2>&1 || exit 1
timeout -k 10 120 python -u profiles/cmds/dbg_cent_l1.py 4 40 > gpurun_out/r03g_lp40.log 2>&1 || exit 2
