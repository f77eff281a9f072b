# r04m: stream count of the default bench with the root level in the refill kernel (its root and
# dive phases fill 64 CUs; a third stream's levels could use the rest): 2 vs 3 streams, twice each
set -o pipefail
export TMPDIR=/tmp
for r in a b; do
  for s in 2 3; do
    timeout -k 10 300 python bench.py --no-cpu --streams $s > gpurun_out/r04m_bench_s${s}_$r.jsonl 2> gpurun_out/r04m_bench_s${s}_$r.err || exit 2
  done
done
