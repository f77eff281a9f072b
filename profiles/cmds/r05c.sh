# r05c: L1 refill threshold sweep on the one-scan-per-trip simplex, then the PMC profiles of the
# default bench's own configuration (three streams) and of min_1_norm
set -o pipefail
export TMPDIR=/tmp
for m in 8 4 12; do
  HVP_LP_REFILL=$m timeout -k 10 300 python bench.py --cost l1 --no-cpu --steps 3 --warmup 1 > gpurun_out/r05c_bench_l1_refill$m.jsonl 2> gpurun_out/r05c_bench_l1_refill$m.err || exit 1
done
timeout -k 10 900 bash profiles/profile_all.sh gpurun_out/r05c_prof decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384 > gpurun_out/r05c_prof.log 2>&1 || exit 2
