#!/bin/bash
# round 6: admm_l1_local_ct_N5 instance 5 alone through a debug build of the N = 5 unit that prints
# the interior point's residuals (HVP_L1ADMM_DEBUG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
HVP_LIB=$PWD/hybrid-vehicle-platoon_amd/lib/libhvpsolve_dbg.so timeout -k 10 120 python -u -c "
import sys, numpy as np
sys.path[:0] = ['hybrid-vehicle-platoon_amd', 'tests', 'oracle']
from golden_io import load
from test_admm_l1 import _cfg, _problem, _system
from hvp.solver import BatchSolver
fx = load('admm_l1_local_ct_N5.npz')
s = BatchSolver(_problem(5, float(fx['rho']), _cfg(fx)), [_system()])
i = 5
r = s.solve_admm(np.zeros(1, np.int32), fx['roles'][i:i+1], fx['params'][i:i+1])
print('status', r.status, 'exp region', fx['exp_region'][i], 'exp cost', fx['exp_cost'][i], 'role', fx['roles'][i])
" > gpurun_out/r06r.log 2>&1
