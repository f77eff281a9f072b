# r04n: stream count of the default bench, 3 vs 4 streams (r04m: 3 streams 7.09-7.14M vs 2 streams
# 6.74-6.98M), twice each
set -o pipefail
export TMPDIR=/tmp
for r in a b; do
  for s in 3 4; do
    timeout -k 10 300 python bench.py --no-cpu --streams $s > gpurun_out/r04n_bench_s${s}_$r.jsonl 2> gpurun_out/r04n_bench_s${s}_$r.err || exit 2
  done
done
# the default line of the shipped library and bench (three streams, CPU baselines)
timeout -k 10 400 python bench.py > gpurun_out/r04n_bench_default.jsonl 2> gpurun_out/r04n_bench_default.err || exit 3
