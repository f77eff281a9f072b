# r04p: stream count (engines) of the C3 / C4 / cent benches, 2 vs 3 (the decentralised bench
# moved to 3 in r04m)
set -o pipefail
export TMPDIR=/tmp
for s in 2 3; do
  timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --streams $s > gpurun_out/r04p_bench_admm_s$s.jsonl 2> gpurun_out/r04p_bench_admm_s$s.err || exit 2
done
for s in 2 3; do
  timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 --no-cpu --streams $s > gpurun_out/r04p_bench_gadmm_s$s.jsonl 2> gpurun_out/r04p_bench_gadmm_s$s.err || exit 3
done
for s in 2 3; do
  timeout -k 10 300 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu --streams $s > gpurun_out/r04p_bench_cent_s$s.jsonl 2> gpurun_out/r04p_bench_cent_s$s.err || exit 4
done
