"""Diagnostics run (not a test): a centralised min_1_norm search with the LP trace on stdout.
Args: debug level (HVP_CENT_DEBUG: 1 failing LPs, 4 iterations, 5 + rows), QP cap, and optionally
a golden fixture name and platoon index (default: oracle seed-0 platoon, n = 3, N = 5)."""
import os
import sys

os.environ["HVP_CENT_DEBUG"] = sys.argv[1] if len(sys.argv) > 1 else "5"
os.environ["HVP_CENT_SPLIT"] = "0"
here = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(here, "..", "..", d) for d in ("hybrid-vehicle-platoon_amd", "tests", "oracle")]
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
from hvp import tables  # noqa: E402
from hvp.cent import CentSolver, cent_problem  # noqa: E402
from hvp.models import PwaGearVehicle  # noqa: E402
from instances import leader_window  # noqa: E402

cap = int(sys.argv[2]) if len(sys.argv) > 2 else 1
veh = PwaGearVehicle(800)
st = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
if len(sys.argv) > 3:
    from golden_io import load

    fx = load(sys.argv[3])
    p = int(sys.argv[4])
    N, n = int(fx["N"]), int(fx["n"])
    x0, lead, li, lsp = fx["x0"][p], fx["leader_x"][p], int(fx["leader_index"][p]), bool(fx["lsp"][p])
    print("EXPECT", fx["exp_status"][p], fx["exp_cost"][p], fx["exp_nodes"][p], fx["exp_region"][p].tolist(), flush=True)
else:
    n, N = 3, 5
    x0, lead, li, lsp = O.env_initial_state(n, 0).astype(float).reshape(n, 2), leader_window(N), 0, False
s = CentSolver(cent_problem(N, quadratic_cost=False), [st])
r = s.solve(np.zeros((1, n), np.int32), np.asarray(x0).reshape(1, n, 2), lead, li, lsp, cap)
print("RESULT", r.status[0], r.cost[0], r.nodes[0], r.region[0].tolist(), flush=True)
