# r05zi: engines (host threads + streams) per GPU for the ADMM benches, same box: C3 and C4 at 2, 3, 4
set -o pipefail
export TMPDIR=/tmp
R=r05zi
for s in 2 3 4 2 3 4; do
  timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass --streams $s >> gpurun_out/${R}_bench_admm_streams.jsonl 2>> gpurun_out/${R}_bench.err || exit 1
  timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 2 --warmup 1 --no-cpu --no-roofline-pass --streams $s >> gpurun_out/${R}_bench_gadmm_streams.jsonl 2>> gpurun_out/${R}_bench.err || exit 2
done
