#!/usr/bin/env bash
# The four bench workloads whose PMC summaries bench.py reads (roofline), one run_profiles.sh each.
#   profiles/profile_all.sh OUTDIR
set -euo pipefail
O=${1:-gpurun_out/prof}
bash profiles/run_profiles.sh "$O/decent_n10_N5" --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1
bash profiles/run_profiles.sh "$O/admm_n10_N10" --controller admm --n 10 --N 10 --platoons 1024 --steps 1 --warmup 1 --no-cpu
bash profiles/run_profiles.sh "$O/gadmm_n20_N10" --controller gadmm --n 20 --N 10 --platoons 2048 --steps 1 --warmup 0 --no-cpu
bash profiles/run_profiles.sh "$O/cent_n10_N5" --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu
echo all profiles done
