"""Host replay of configs[3] (switching ADMM, n = 20, N = 10, fixture gadmm_steps_n20_N10): the
oracle coordinator (oracle.py GAdmmCoordinator, restating fleet_g_admm.py:255-301) with its local
QPs solved by the product's lane algorithm built for the host (hvp_hostref_gadmm_solve) in one of
its modes:

    mode 0   the active-set method (the device's unforced path)
    mode 1   every local QP by the interior-point fallback (hvp_admm.h solve_admm_ipm)
    mode 2   HVP_LEAF_GI_CAP=2 as the device runs it: two active-set steps, then the fallback

Test infrastructure (tests/test_gadmm.py) and a diagnostic: per coordinator
call, whether the run equals the fixture (u, cost, sequences, rounds) and how many local QPs
failed.

    python tests/gadmm_replay.py [mode] [calls]
"""

from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import oracle as O  # noqa: E402
from golden_io import load  # noqa: E402
from instances import leader_window  # noqa: E402


def replay(mode: int, ncalls: int, verbose: bool = True) -> int:
    """Number of coordinator calls (of the first `ncalls`) that differ from the fixture."""
    from hvp import _abi, tables
    from hvp.gadmm import gadmm_problem
    from hvp.models import PwaGearVehicle

    lib = ctypes.CDLL(_abi.HOSTREF_PATH)
    fx = load("gadmm_steps_n20_N10.npz")
    n, N = int(fx["n"]), int(fx["N"])
    prob = gadmm_problem(N, float(fx["rho"]))
    veh = PwaGearVehicle(800)
    S = (_abi.HvpSystem * 1)(tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh)))
    f = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    stats = {"qps": 0, "fail": 0}

    def local(sysd, cfg, N_, role, back_copy, rho, params, sigma):
        u, x, xf, xb = np.zeros(N), np.zeros((2, N + 1)), np.zeros((2, N + 1)), np.zeros((2, N + 1))
        cost, st, edge = np.zeros(1), np.zeros(1, np.int32), np.zeros(1, np.uint32)
        rl = np.array([role | (64 if back_copy else 0)], np.int32)
        p = np.ascontiguousarray(np.asarray(params, np.float64))
        sq = np.ascontiguousarray(np.asarray(sigma).astype(np.int8))
        rc = lib.hvp_hostref_gadmm_solve(ctypes.byref(prob), S, 1, f(np.zeros(1, np.int32)), f(rl), f(p), f(sq),
                                         f(u), f(x), f(xf), f(xb), f(cost), f(st), f(edge))
        assert rc == 0
        stats["qps"] += 1
        stats["fail"] += int(st[0] != 0)
        return O.GAdmmQpResult(x, u, xf, xb, float(cost[0]), 0 if st[0] == 0 else 1, True, int(edge[0]))

    original = O.solve_gadmm_qp
    O.solve_gadmm_qp = local
    lib.hvp_hostref_set_admm_leaf_ipm(mode)
    try:
        co = O.GAdmmCoordinator([O.gear_pwa_system(800.0)] * n, O.Cfg(), N, admm_iters=int(fx["iters"]),
                                max_rounds=int(fx["max_rounds"]))
        steps = int(fx["steps"])
        bad = 0
        for c in range(min(ncalls, len(fx["states"]))):
            t = c % steps
            if t == 0:
                co.prev_u = None
            co.set_leader_traj(leader_window(N, t))
            stats.update(qps=0, fail=0)
            try:
                u, cost, runs = co.control(fx["states"][c])
            except RuntimeError as e:
                if verbose:
                    print(f"call {c}: {e}; local QPs {stats['qps']} failed {stats['fail']}", flush=True)
                bad += 1
                continue
            du = np.abs(u - fx["exp_u"][c]).max()
            dc = abs(cost - fx["exp_cost"][c]) / abs(fx["exp_cost"][c])
            rounds = [r[2]["rounds"] if r else -1 for r in runs]
            exp_rounds = [int(r) for r in fx["exp_rounds"][c][:len(rounds)]]
            seq_ok = all(r is None or np.array_equal(r[2]["sigma"], fx["exp_seq"][c][k]) for k, r in enumerate(runs))
            ok = du <= 1e-6 and dc <= 1e-8 and seq_ok and rounds == exp_rounds
            bad += not ok
            if verbose:
                print(f"call {c}: du {du:.2e} dcost {dc:.2e} sequences {'=' if seq_ok else '!='} rounds {rounds} "
                      f"(fixture {exp_rounds}) local QPs {stats['qps']} failed {stats['fail']} "
                      f"{'OK' if ok else 'DIFF'}", flush=True)
        return bad
    finally:
        O.solve_gadmm_qp = original
        lib.hvp_hostref_set_admm_leaf_ipm(0)


if __name__ == "__main__":
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sys.exit(1 if replay(mode, calls) else 0)
