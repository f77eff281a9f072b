# r03s: the two heaviest centralised platoons (seeds 426, 3139): incumbent improvements of the
# search (HVP_CENT_DEBUG=6), then 3139 started from its optimal cost as incumbent (HVP_CENT_INC)
set -o pipefail
HVP_CENT_DEBUG=6 timeout -k 10 200 python profiles/cmds/diag_cent_heavy.py --seeds 3139 426 --max-nodes 2000000 > gpurun_out/r03s_heavy.jsonl 2> gpurun_out/r03s_heavy.err || exit 1
HVP_CENT_DEBUG=6 HVP_CENT_INC=1361956.8177621625 timeout -k 10 200 python profiles/cmds/diag_cent_heavy.py --seeds 3139 --max-nodes 2000000 > gpurun_out/r03s_heavy_inc.jsonl 2> gpurun_out/r03s_heavy_inc.err || exit 2
# seed 426 (past the 2M cap) alone with a 30M cap, no diagnostics: how many QPs it needs
timeout -k 10 240 python profiles/cmds/diag_cent_heavy.py --seeds 426 --max-nodes 30000000 > gpurun_out/r03s_heavy_426.jsonl 2> gpurun_out/r03s_heavy_426.err || exit 3
