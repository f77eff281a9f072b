#!/bin/bash
# round 6: admm_l1_local_ct_N5 instance 5 (HVP_MAXITER on the device) under larger iteration caps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u profiles/diag_admm_l1.py admm_l1_local_ct_N5.npz 0 120 400 > gpurun_out/r06q.log 2>&1
