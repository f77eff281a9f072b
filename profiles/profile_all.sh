#!/usr/bin/env bash
# The bench workloads whose PMC summaries bench.py reads (roofline), one run_profiles.sh each.
# The tag's _P<platoons> is the launch size the bench's roofline pass uses: decent and cent time
# one handle over the whole batch; admm and gadmm time each of their 2 engines (S/2 platoons).
#   profiles/profile_all.sh OUTDIR [workload ...]   (default: all six)
set -euo pipefail
O=${1:-gpurun_out/prof}
shift || true
W=("$@")
[ ${#W[@]} -gt 0 ] || W=(decent_n10_N5_P16384 decent_n10_N5_P16384_s3 decent_n10_N5_l1_P16384 admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096)
for w in "${W[@]}"; do
  case $w in
    decent_n10_N5_P16384) bash profiles/run_profiles.sh "$O/$w" --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 ;;
    # the headline's own configuration: the default bench (three handles on three streams)
    decent_n10_N5_P16384_s3) bash profiles/run_profiles.sh "$O/$w" --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 3 --no-roofline-pass ;;
    decent_n10_N5_l1_P16384) bash profiles/run_profiles.sh "$O/$w" --cost l1 --platoons 16384 --steps 2 --warmup 1 --no-cpu --streams 1 ;;
    admm_n10_N10_P512) bash profiles/run_profiles.sh "$O/$w" --controller admm --n 10 --N 10 --platoons 512 --steps 1 --warmup 1 --no-cpu --streams 1 ;;
    gadmm_n20_N10_P2048) bash profiles/run_profiles.sh "$O/$w" --controller gadmm --n 20 --N 10 --platoons 2048 --steps 1 --warmup 0 --no-cpu --streams 1 ;;
    cent_n10_N5_P4096) bash profiles/run_profiles.sh "$O/$w" --controller cent --n 10 --N 5 --platoons 4096 --steps 1 --warmup 0 --no-cpu --streams 1 ;;
    # naive-ADMM min_1_norm (the wave interior point): the bench line's 64 platoons on 2 engines
    admm_n10_N10_l1_P32) bash profiles/run_profiles.sh "$O/$w" --controller admm --cost l1 --n 10 --N 10 --platoons 32 --steps 1 --warmup 0 --no-cpu --streams 1 ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
done
echo all profiles done
