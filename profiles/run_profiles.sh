#!/usr/bin/env bash
# Profiling recipe used for profiles/ (run on the GPU box from the repo root).
#   1. kernel trace + stats of the bench command (per-kernel average durations)
#   2. separate PMC passes (one counter group each, no tracing domains besides kernel dispatch):
#      HBM bytes (FETCH_SIZE, WRITE_SIZE) and the FP64 instruction mix of the QP kernel
set -euo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
BENCH=(python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/trace" -o run -- "${BENCH[@]}" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d "$OUT/fetch" -o run -- "${BENCH[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d "$OUT/write" -o run -- "${BENCH[@]}" > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 -T -f csv -d "$OUT/f64" -o run -- "${BENCH[@]}" > "$OUT/f64.log" 2>&1
# switching ADMM (configs[3]) kernel trace, its own workload directory
GADMM=(python3 bench.py --controller gadmm --n 20 --N 10 --platoons 2048 --steps 1 --warmup 0 --no-cpu)
mkdir -p "$OUT/gadmm"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$OUT/gadmm/trace" -o run -- "${GADMM[@]}" > "$OUT/gadmm/trace.log" 2>&1
echo profiles done
