# r05h: the round's library -- the whole GPU suite and smoke, then hash-stamped PMC profiles of the
# decentralised workloads (one stream, the timed three-stream configuration, min_1_norm),
# summarised on the box so the bench lines that follow carry their rooflines; the default and
# min_1_norm bench lines with their CPU baselines
set -o pipefail
export TMPDIR=/tmp
R=r05h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit 2
W="decent_n10_N5_P16384 decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384"
timeout -k 10 1200 bash profiles/profile_all.sh gpurun_out/$R $W > gpurun_out/${R}_prof.log 2>&1 || exit 3
mkdir -p gpurun_out/${R}_sum
for w in $W; do
  python profiles/summarize.py gpurun_out/$R/$w $R $w > /dev/null && cp profiles/${R}_${w}_* gpurun_out/${R}_sum/ || exit 4
done
timeout -k 10 400 python bench.py > gpurun_out/${R}_bench_default.jsonl 2> gpurun_out/${R}_bench_default.err || exit 5
timeout -k 10 300 python bench.py --cost l1 --steps 5 --warmup 1 > gpurun_out/${R}_bench_l1.jsonl 2> gpurun_out/${R}_bench_l1.err || exit 6
