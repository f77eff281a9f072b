#!/usr/bin/env python3
"""Diagnostic: one centralised platoon (n, N, seed) on the GPU with HVP_CENT_DEBUG printf output."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
os.environ.setdefault("HVP_CENT_DEBUG", "1")
import oracle as O  # noqa: E402
from instances import leader_window  # noqa: E402
from hvp import tables  # noqa: E402
from hvp.cent import CentSolver, cent_problem  # noqa: E402
from hvp.models import PwaGearVehicle  # noqa: E402

n, N, seed = (int(a) for a in sys.argv[1:4])
veh = PwaGearVehicle(800)
st = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
s = CentSolver(cent_problem(N), [st])
x0 = O.env_initial_state(n, seed).astype(float).reshape(1, n, 2)
r = s.solve(np.zeros((1, n), np.int32), x0, leader_window(N), max_nodes=int(sys.argv[4]) if len(sys.argv) > 4 else 2000)
print("status", r.status, "nodes", r.nodes, "cost", r.cost, "regions", r.region[0].tolist(), flush=True)
