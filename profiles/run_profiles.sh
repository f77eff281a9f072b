#!/usr/bin/env bash
# Profiling recipe used for profiles/ (run on the GPU box from the repo root).
#   profiles/run_profiles.sh OUT [bench args...]
#   1. kernel trace + stats of the bench command (per-kernel average durations)
#   2. separate PMC passes (one counter group each, kernel dispatch only, no tracing domains):
#      fetch / write : HBM bytes (FETCH_SIZE, WRITE_SIZE; each its own pass, TCC slots)
#      f64           : FP64 instruction mix + VALU / SALU / LDS instruction counts
#      occ           : occupancy and issue utilisation (waves, wave / busy cycles, VALU active and
#                      thread cycles = lane utilisation, issue and wait stalls) + GRBM_GUI_ACTIVE
# profiles/summarize.py OUT <round> <tag> condenses the passes into profiles/<round>_<tag>_summary.json
# (profiles/profile_all.sh runs the four bench workloads bench.py looks up by tag).
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift || true
if [ $# -gt 0 ]; then BENCH=(python3 bench.py "$@"); else BENCH=(python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1); fi
mkdir -p "$OUT"
echo "${BENCH[*]}" > "$OUT/cmd.txt"
# the stamp bench.py matches against the library it loads (HVP_LIB, else the in-tree build)
sha256sum "${HVP_LIB:-hybrid-vehicle-platoon_amd/lib/libhvpsolve.so}" | cut -d' ' -f1 > "$OUT/lib_sha256.txt"
echo "profiling: ${BENCH[*]}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- "${BENCH[@]}" > "$OUT/trace.log" 2>&1
echo trace done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$OUT/fetch" -o run -- "${BENCH[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$OUT/write" -o run -- "${BENCH[@]}" > "$OUT/write.log" 2>&1
echo hbm done
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT64 \
    -T -f csv -d "$OUT/f64" -o run -- "${BENCH[@]}" > "$OUT/f64.log" 2>&1
echo f64 done
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU \
    SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    -T -f csv -d "$OUT/occ" -o run -- "${BENCH[@]}" > "$OUT/occ.log" 2>&1
# memory instructions and L2 write-back transaction sizes (the byte budget of DESIGN.md section 4):
# vector memory instructions issued (incl. scratch), scalar loads, and the L2's write requests to
# the fabric in total and as whole 64-byte transactions (the rest are 32-byte partial lines)
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
    -T -f csv -d "$OUT/mem" -o run -- "${BENCH[@]}" > "$OUT/mem.log" 2>&1
echo profiles done
