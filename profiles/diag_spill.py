"""Diagnostic (round 5): the level buckets' spill (hvp_lane.h bnb_put_children) at C2's shape.
For HVP_SPLIT_LEVELS = 1, 2, 4: the smallest node capacity at which no instance overflows
(bisection), and at a few capacities the overflowed instances and the spilled reservations.

    python profiles/diag_spill.py [platoons]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), ROOT]


def main():
    import torch

    import bench
    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    n, N = 10, 5
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    params, roles = bench.make_inputs(range(S), n, N)
    dev = torch.device("cuda", 0)
    tp, tr = torch.from_numpy(params).to(dev), torch.from_numpy(roles).to(dev)
    ts = torch.zeros(len(roles), dtype=torch.int32, device=dev)
    B = len(roles)
    veh = PwaGearVehicle(800)

    def solve(cap):  # a fresh handle per capacity (hvp_reserve only ever grows a workspace)
        s = BatchSolver(tables.problem(N), [tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))])
        s.reserve(B, cap)
        out = s.solve_device(ts, tr, tp)
        torch.cuda.synchronize()
        st = s.stats()
        return int((out["status"] == _abi.OVERFLOW).sum().item()), int(st.n_spilled), int(st.n_candidates)

    res = {}
    for split in (1, 2, 4):
        os.environ["HVP_SPLIT_LEVELS"] = str(split)
        lo, hi = B // 4, 16 * B
        while hi - lo > 16:
            mid = (lo + hi) // 2
            if solve(mid)[0]:
                lo = mid
            else:
                hi = mid
        res[split] = hi
        print(f"split {split}: smallest capacity without overflow {hi} (B = {B}); at it: {solve(hi)}", flush=True)
    for split in (2, 4):
        os.environ["HVP_SPLIT_LEVELS"] = str(split)
        for cap in (res[1], res[1] + 64 * split, (res[1] * 3) // 2):
            print(f"split {split} cap {cap}: (overflowed, spilled, QPs) {solve(cap)}", flush=True)


if __name__ == "__main__":
    main()
