"""Diagnostic (round 5): how much active-set work a warm start of the naive-ADMM node QPs saves.

Records the local-problem parameter blocks of the oracle coordinator (configs[2]: n = 10,
N = 10, 20 ADMM iterations, 2 closed-loop steps; AdmmCoordinator, fleet_naive_admm.py:379-477),
then re-solves every iteration's batch of n local MIQPs with the host build of the product's
branch and bound (hvp_hostref_solve_admm_batch) under each hinge-state start mode
(hvp_hostref_set_admm_warm):
  0  every node QP from the constant-velocity hinge states (the product until round 5)
  1  a child from its parent's final hinge states (the root cold)
  2  as 1, and the root from the previous ADMM iteration's root states of the same vehicle
  3  every node QP from the record of the same node (depth, region code) of the previous ADMM
     iteration: its final hinge states and active set, forced in as equalities (what a warm start
     that carries the factors begins from; counted as one iteration)
  4  as 3 through the device's table: per (vehicle, depth) a direct-mapped table of S records
     (slot = hash of the region code); among one level's nodes sharing a slot the smallest code
     owns it, the others start cold
and prints QPs, active-set iterations and hinge rounds per MIQP, with the answers' agreement.

    python profiles/diag_admm_warm.py
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), ROOT]

import oracle as O  # noqa: E402
from instances import leader_window  # noqa: E402


def record(n=10, N=10, iters=20, steps=2, seed=0):
    calls = []
    orig = O.solve_admm_miqp

    def rec(sysd, cfg, N_, role, rho, params, maxit=200):
        calls.append((role, np.array(params, dtype=np.float64)))
        return orig(sysd, cfg, N_, role, rho, params, maxit)

    O.solve_admm_miqp = rec
    try:
        coord = O.AdmmCoordinator(O.gear_pwa_system(800.0), O.Cfg(), N, n)
        st = O.env_initial_state(n, seed).astype(float)
        for t in range(steps):
            coord.set_leader_x(leader_window(N, t))
            _, hist = coord.step(st, iters)
            st = np.concatenate([r.x[:, 1] for r in hist[-1]])
    finally:
        O.solve_admm_miqp = orig
    # calls are in (step, iteration, vehicle) order
    roles = np.array([c[0] for c in calls], np.int32).reshape(-1, n)
    params = np.stack([c[1] for c in calls]).reshape(roles.shape[0], n, -1)
    return roles, params


def main():
    from hvp import _abi, tables
    from hvp.admm import admm_problem
    from hvp.models import PwaGearVehicle

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), "lib/libhvp_hostref.so"],
                   check=True)
    lib = ctypes.CDLL(_abi.HOSTREF_PATH)
    N = 10
    roles, params = record(N=N)
    veh = PwaGearVehicle(800)
    S = (_abi.HvpSystem * 1)(tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh)))
    prob = admm_problem(N, 0.5)
    f = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    n = roles.shape[1]
    ref = None
    for mode, slots in ((0, 0), (1, 0), (2, 0), (3, 0), (4, 16), (4, 32), (4, 64), (4, 128), (4, 256), (4, 1024)):
        lib.hvp_hostref_set_admm_warm(mode)
        lib.hvp_hostref_set_admm_slots(slots)
        lib.hvp_hostref_reset_admm_warm()
        tot = np.zeros(3, np.int64)
        outs = []
        for it in range(roles.shape[0]):
            B = n
            u, x, reg = np.zeros((B, N)), np.zeros((B, 2, N + 1)), np.zeros((B, N), np.int8)
            cost, st, nodes, its = np.zeros(B), np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(B, np.int32)
            xf, xb = np.zeros((B, 2, N + 1)), np.zeros((B, 2, N + 1))
            rc = lib.hvp_hostref_solve_admm_batch(ctypes.byref(prob), S, B, f(np.zeros(B, np.int32)),
                                                  f(np.ascontiguousarray(roles[it])),
                                                  f(np.ascontiguousarray(params[it])), f(u), f(x), f(reg), f(cost),
                                                  f(st), f(nodes), f(its), f(xf), f(xb), 1)
            assert rc == 0
            tot[0] += nodes.sum()
            tot[1] += its.sum()
            outs.append((u.copy(), reg.copy(), cost.copy(), st.copy()))
        h = np.zeros(8, np.int64)
        lib.hvp_hostref_admm_warm_stats(f(h))
        m = roles.size
        print(f"mode {mode}{f' ({slots} slots per depth)' if slots else ''}: {m} MIQPs, QPs/MIQP {tot[0] / m:.1f}, active-set iterations/MIQP {tot[1] / m:.1f}, "
              f"hinge rounds/QP {h[1] / max(h[0], 1):.3f} (QPs {h[0]}, first round consistent {h[2] / max(h[0], 1):.3f}, "
              f"failed {h[3]})")
        if mode >= 3:
            print(f"   node records: lookups {h[4]}, hits {h[5] / max(h[4], 1):.3f}, "
                  f"warm starts dual-feasible {h[6] / max(h[5], 1):.3f} (without drops {h[7] / max(h[5], 1):.3f})")
        if ref is None:
            ref = outs
        else:
            du = max(np.abs(a[0] - b[0]).max() for a, b in zip(outs, ref))
            same_reg = all(np.array_equal(a[1], b[1]) for a, b in zip(outs, ref))
            bit = all(np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2]) for a, b in zip(outs, ref))
            print(f"   vs mode 0: regions equal {same_reg}, max |du| {du:.3g}, bit-identical {bit}")


if __name__ == "__main__":
    main()
