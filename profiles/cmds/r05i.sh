# r05i: hash-stamped PMC profiles of the C3, C4 and centralised workloads (summarised on the box),
# then their bench lines with CPU baselines on every host core and on one
set -o pipefail
export TMPDIR=/tmp
R=r05i
W="admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096"
timeout -k 10 1200 bash profiles/profile_all.sh gpurun_out/$R $W > gpurun_out/${R}_prof.log 2>&1 || exit 1
mkdir -p gpurun_out/${R}_sum
for w in $W; do
  python profiles/summarize.py gpurun_out/$R/$w $R $w > /dev/null && cp profiles/${R}_${w}_* gpurun_out/${R}_sum/ || exit 2
done
timeout -k 10 400 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 > gpurun_out/${R}_bench_admm.jsonl 2> gpurun_out/${R}_bench_admm.err || exit 3
timeout -k 10 400 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 > gpurun_out/${R}_bench_gadmm.jsonl 2> gpurun_out/${R}_bench_gadmm.err || exit 4
timeout -k 10 400 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 > gpurun_out/${R}_bench_cent.jsonl 2> gpurun_out/${R}_bench_cent.err || exit 5
