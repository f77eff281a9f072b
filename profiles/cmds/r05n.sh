# r05n: the warm start reads its record into LDS first, cold starts skip the extra setup: GPU tests of
# the ADMM forms, C3 / C4 bench lines (same box) and a PMC profile of C3
set -o pipefail
export TMPDIR=/tmp
R=r05n
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_admm.py tests/test_gadmm.py -m gpu > gpurun_out/${R}_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --controller admm --n 10 --N 10 --platoons 1024 --steps 3 --warmup 1 --no-cpu --no-roofline-pass > gpurun_out/${R}_bench_admm.jsonl 2> gpurun_out/${R}_bench_admm.err || exit 2
timeout -k 10 300 python bench.py --controller gadmm --n 20 --N 10 --platoons 4096 --steps 3 --warmup 1 --no-cpu --no-roofline-pass > gpurun_out/${R}_bench_gadmm.jsonl 2> gpurun_out/${R}_bench_gadmm.err || exit 3
timeout -k 10 800 bash profiles/profile_all.sh gpurun_out/${R} admm_n10_N10_P512 > gpurun_out/${R}_prof.log 2>&1 || exit 4
