#!/usr/bin/env bash
# The bench workloads whose PMC summaries bench.py reads (roofline), one run_profiles.sh each.
# The tag's _P<platoons> is the launch size the bench's roofline pass uses: decent and cent time
# one handle over the whole batch; admm and gadmm time each of their 2 engines (S/2 platoons).
#   profiles/profile_all.sh OUTDIR
set -euo pipefail
O=${1:-gpurun_out/prof}
bash profiles/run_profiles.sh "$O/decent_n10_N5_P16384" --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1
bash profiles/run_profiles.sh "$O/decent_n10_N5_l1_P16384" --cost l1 --platoons 16384 --steps 2 --warmup 1 --no-cpu --streams 1
bash profiles/run_profiles.sh "$O/admm_n10_N10_P512" --controller admm --n 10 --N 10 --platoons 512 --steps 1 --warmup 1 --no-cpu --streams 1
bash profiles/run_profiles.sh "$O/gadmm_n20_N10_P2048" --controller gadmm --n 20 --N 10 --platoons 2048 --steps 1 --warmup 0 --no-cpu --streams 1
bash profiles/run_profiles.sh "$O/cent_n10_N5_P4096" --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu --streams 1
echo all profiles done
