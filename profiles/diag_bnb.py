#!/usr/bin/env python3
"""Diagnostic (GPU): branch-and-bound search statistics at one sweep point, device vs the
host build of the same algorithm (lib/libhvp_hostref.so).  Used to size the workspace and to
find where the device search diverges from the host's."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), ROOT]


def main():
    import torch

    import bench
    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    n, N, S = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    veh = PwaGearVehicle(800)
    sysv = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    params, roles = bench.make_inputs(range(S), n, N)
    B = len(roles)
    s = BatchSolver(tables.problem(N), [sysv])
    s.reserve(B, int(sys.argv[4]) * B if len(sys.argv) > 4 else 0)
    dev = torch.device("cuda", 0)
    out = s.solve_device(torch.zeros(B, dtype=torch.int32, device=dev), torch.from_numpy(roles).to(dev),
                         torch.from_numpy(params).to(dev))
    st = s.stats()
    status = out["status"].cpu().numpy()
    nodes = out["nodes"].cpu().numpy()
    L = ctypes.CDLL(_abi.HOSTREF_PATH)
    bufs = [np.zeros((B, N)), np.zeros((B, 2, N + 1)), np.zeros((B, N), np.int8), np.zeros(B), np.zeros(B, np.int32),
            np.zeros(B, np.int32), np.zeros(B, np.int32)]
    f = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    prob = tables.problem(N)
    S_ = (_abi.HvpSystem * 1)(sysv)
    L.hvp_hostref_solve_batch(ctypes.byref(prob), S_, B, f(np.zeros(B, np.int32)), f(roles),
                              f(np.ascontiguousarray(params)), *[f(b) for b in bufs], 16)
    reg = out["region"].cpu().numpy()
    same = (reg == bufs[2]).all(axis=1) & (status == bufs[4])
    res = {"n": n, "N": N, "B": B, "capacity": st.capacity, "qps": st.n_candidates,
           "failed_bounds": st.n_failed_bounds, "leaf_fallbacks": st.n_fallback,
           "status_dev": np.bincount(status, minlength=4).tolist(),
           "status_host": np.bincount(bufs[4], minlength=4).tolist(),
           "nodes_dev_mean": float(nodes.mean()), "nodes_dev_max": int(nodes.max()),
           "nodes_host_mean": float(bufs[5].mean()), "nodes_host_max": int(bufs[5].max()),
           "same_solution": int(same.sum()), "differ": np.flatnonzero(~same)[:20].tolist()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
