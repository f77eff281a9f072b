# r04a: hash-stamped profiles of the library with the keyed switching-ADMM warm records: the
# switching-ADMM GPU tests, the five bench workloads (kernel trace + separate PMC passes, each summary
# stamped with the library's SHA-256) and their bench lines
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gadmm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04a_gadmm_tests.log 2>&1 || exit 9
bash profiles/profile_all.sh gpurun_out/r04a || exit 1
mkdir -p gpurun_out/r04a_sum
for w in decent_n10_N5_P16384 decent_n10_N5_l1_P16384 admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096; do
  python profiles/summarize.py gpurun_out/r04a/$w r04a $w > /dev/null && cp profiles/r04a_${w}_* gpurun_out/r04a_sum/ || exit 1
done
timeout -k 10 400 python bench.py > gpurun_out/r04a_bench_default.jsonl 2> gpurun_out/r04a_bench_default.err || exit 2
timeout -k 10 300 python bench.py --cost l1 --steps 5 --warmup 1 > gpurun_out/r04a_bench_l1.jsonl 2> gpurun_out/r04a_bench_l1.err || exit 3
timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 > gpurun_out/r04a_bench_admm.jsonl 2> gpurun_out/r04a_bench_admm.err || exit 4
timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 > gpurun_out/r04a_bench_gadmm.jsonl 2> gpurun_out/r04a_bench_gadmm.err || exit 5
timeout -k 10 300 python bench.py --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 > gpurun_out/r04a_bench_cent.jsonl 2> gpurun_out/r04a_bench_cent.err || exit 6
