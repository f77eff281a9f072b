#!/usr/bin/env python3
"""Round 6 diagnostic: the min_1_norm branch and bound on the l1_variant_n3_N3 fixture under the
search's A/B switches (which component returns HVP_MAXITER)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
from golden_io import load, product_problem  # noqa: E402
from hvp import _abi  # noqa: E402
from hvp.solver import BatchSolver  # noqa: E402

fx = load(sys.argv[1] if len(sys.argv) > 1 else "l1_variant_n3_N3.npz")
prob, systems = product_problem(fx)
prob.method = _abi.METHOD_BNB
s = BatchSolver(prob, systems)
res = s.solve(fx["sys"], fx["roles"], fx["params"])
st = s.stats()
print(os.environ.get("TAG", ""), "status", res.status.tolist(), "exp", fx["exp_status"].tolist(), "nodes", res.nodes.tolist(),
      "cand", st.n_candidates, "cost", np.round(res.cost, 6).tolist(), "exp", np.round(fx["exp_cost"], 6).tolist(),
      "regions", res.region.tolist(), flush=True)
