#!/usr/bin/env python3
"""Round 6 diagnostic: the naive-ADMM min_1_norm local problems of a fixture under several interior-
point iteration caps (hvp_problem.max_iter): which instances return HVP_MAXITER, and their costs
against the oracle's.   python profiles/diag_admm_l1.py [fixture] [max_iter ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from golden_io import load  # noqa: E402
from test_admm_l1 import _cfg, _problem, _system  # noqa: E402

from hvp.solver import BatchSolver  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "admm_l1_local_ct_N5.npz"
fx = load(name)
N = int(fx["N"])
for mi in [int(a) for a in sys.argv[2:]] or [0, 120, 400]:
    prob = _problem(N, float(fx["rho"]), _cfg(fx))
    prob.max_iter = mi
    s = BatchSolver(prob, [_system()])
    B = len(fx["roles"])
    r = s.solve_admm(np.zeros(B, np.int32), fx["roles"], fx["params"])
    rel = np.abs(r.cost - fx["exp_cost"]) / np.maximum(1.0, np.abs(fx["exp_cost"]))
    print(f"max_iter {mi}: status {r.status.tolist()} nodes {r.nodes.tolist()} iters {r.iters.tolist()}")
    print(f"   cost rel err {np.array2string(rel, precision=2)} region ok "
          f"{[bool(np.array_equal(r.region[i], fx['exp_region'][i])) for i in range(B)]}", flush=True)
