# r05k: bucket spill + naive-ADMM node records (hvp_lane.h node_index): the GPU tests of both, and a
# same-box A/B of C3 (configs[2] at 1024 platoons) over the records per (instance, depth)
set -o pipefail
export TMPDIR=/tmp
R=r05k
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_admm.py tests/test_gpu_overflow.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
for s in 0 128 256 0 128 256; do
  HVP_ADMM_NODE_SLOTS=$s timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass >> gpurun_out/${R}_bench_admm_ab.jsonl 2>> gpurun_out/${R}_bench_admm_ab.err || exit 2
  echo "slots $s done" >> gpurun_out/${R}_bench_admm_ab.jsonl
done
