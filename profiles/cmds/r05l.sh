# r05l: the naive-ADMM node records with multiplier drops in the warm start (hvp_coop.h warm_start;
# also the switching ADMM's per-QP records): the ADMM / switching-ADMM / overflow GPU tests, then
# same-box A/B of C3 over the records per (instance, depth) and C4 on the new warm start
set -o pipefail
export TMPDIR=/tmp
R=r05l
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_admm.py tests/test_gadmm.py tests/test_gpu_overflow.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for s in 0 256 512 0 256 512; do
  HVP_ADMM_NODE_SLOTS=$s timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_ab.jsonl 2>> gpurun_out/${R}_bench_admm_ab.err || exit 2
  echo "slots $s done" >> gpurun_out/${R}_bench_admm_ab.jsonl
done
timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 --no-cpu --no-roofline-pass > gpurun_out/${R}_bench_gadmm.jsonl 2> gpurun_out/${R}_bench_gadmm.err || exit 3
