# r04e: (1) kernel trace of the root-refill-only library (per-level refill times against r04b's
# traces of round 3's library and HEAD), (2) min_1_norm kernel traces: per-lane simplex vs the wave
# interior point, (3) the solve of test_long_horizon_leaf_fallback[sweep_n5_N10] that timed out in
# r04b, timed alone on round 3's library, the root-refill-only one and HEAD (kernel-serialised with
# the HIP launch log for HEAD, so the last launch names the kernel that does not finish)
set -o pipefail
export TMPDIR=/tmp
L=$PWD/hybrid-vehicle-platoon_amd/lib
HVP_LIB=$L/libhvpsolve_rr.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r04e_trace_rr -o run -- python3 bench.py --platoons 16384 --steps 5 --warmup 1 --no-cpu --streams 1 > gpurun_out/r04e_trace_rr.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r04e_trace_l1_simplex -o run -- python3 bench.py --cost l1 --platoons 16384 --steps 2 --warmup 1 --no-cpu --streams 1 > gpurun_out/r04e_trace_l1_simplex.log 2>&1 || exit 3
HVP_L1_SIMPLEX=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r04e_trace_l1_ipm -o run -- python3 bench.py --cost l1 --platoons 16384 --steps 2 --warmup 1 --no-cpu --streams 1 > gpurun_out/r04e_trace_l1_ipm.log 2>&1 || exit 4
HVP_LEAF_GI_CAP=2 HVP_LIB=$L/libhvpsolve_r03.so timeout -k 10 60 python -u profiles/cmds/diag_leafcap.py > gpurun_out/r04e_leafcap_r03.jsonl 2> gpurun_out/r04e_leafcap_r03.err || exit 5
HVP_LEAF_GI_CAP=2 HVP_LIB=$L/libhvpsolve_rr.so timeout -k 10 60 python -u profiles/cmds/diag_leafcap.py > gpurun_out/r04e_leafcap_rr.jsonl 2> gpurun_out/r04e_leafcap_rr.err || exit 6
HVP_LEAF_GI_CAP=2 AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=3 timeout -k 10 60 python -u profiles/cmds/diag_leafcap.py > gpurun_out/r04e_leafcap_new.jsonl 2> gpurun_out/r04e_leafcap_new.err || exit 7
