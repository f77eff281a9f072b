# r04d: hash-stamped profiles of the shipped library (kernel trace + separate PMC passes per bench
# workload), summarised on the box so the bench lines that follow use them, then the bench lines.
#   part 1: C2 decent + min_1_norm; part 2: C3 naive ADMM, C4 switching ADMM, centralised + the
#   heaviest centralised platoon (seed 426) alone with a 30M QP cap
set -o pipefail
export TMPDIR=/tmp
R=${1:-r04d}
PART=${2:-1}
if [ "$PART" = 1 ]; then W="decent_n10_N5_P16384 decent_n10_N5_l1_P16384"; else W="admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096"; fi
bash profiles/profile_all.sh gpurun_out/$R $W || exit 1
mkdir -p gpurun_out/${R}_sum
for w in $W; do
  python profiles/summarize.py gpurun_out/$R/$w $R $w > /dev/null && cp profiles/${R}_${w}_* gpurun_out/${R}_sum/ || exit 1
done
if [ "$PART" = 1 ]; then
  timeout -k 10 400 python bench.py > gpurun_out/${R}_bench_default.jsonl 2> gpurun_out/${R}_bench_default.err || exit 2
  timeout -k 10 300 python bench.py --cost l1 --steps 5 --warmup 1 > gpurun_out/${R}_bench_l1.jsonl 2> gpurun_out/${R}_bench_l1.err || exit 3
else
  timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 > gpurun_out/${R}_bench_admm.jsonl 2> gpurun_out/${R}_bench_admm.err || exit 4
  timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 > gpurun_out/${R}_bench_gadmm.jsonl 2> gpurun_out/${R}_bench_gadmm.err || exit 5
  timeout -k 10 300 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 > gpurun_out/${R}_bench_cent.jsonl 2> gpurun_out/${R}_bench_cent.err || exit 6
  # seed 426 alone with a 30M QP cap: the split-task queue declines exports when full instead of
  # overflowing, so the search should end where r03s ended HVP_OVERFLOW at 22.1M QPs
  timeout -k 10 240 python profiles/cmds/diag_cent_heavy.py --seeds 426 --max-nodes 30000000 > gpurun_out/${R}_heavy_426.jsonl 2> gpurun_out/${R}_heavy_426.err || exit 7
fi
