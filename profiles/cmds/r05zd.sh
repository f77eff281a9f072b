# r05zd: hash-stamped PMC profiles of the C3, C4 and centralised workloads of the round's library
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 1100 bash profiles/profile_all.sh gpurun_out/r05zd admm_n10_N10_P512 gadmm_n20_N10_P2048 cent_n10_N5_P4096 > gpurun_out/r05zd_prof.log 2>&1 || exit 1
