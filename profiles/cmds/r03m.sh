# r03m: refill-kernel cycle split (instrumented build, HVP_REFILL_PROF): event vs trips, busy lanes
set -o pipefail
timeout -k 10 300 python bench.py --platoons 16384 --steps 2 --warmup 1 --no-cpu --streams 1 > gpurun_out/r03m_bench.jsonl 2> gpurun_out/r03m_bench.err || exit 3
