#!/usr/bin/env python3
"""Diagnostic (run on the GPU box): the centralised MLD kernel against the live CPU oracle on a
few platoons, with per-platoon QP counts and kernel time.  Usage: diag_cent.py n N seeds"""

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hybrid-vehicle-platoon_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
from instances import leader_window  # noqa: E402


def main():
    n, N, S = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    oracle_check = len(sys.argv) <= 4 or sys.argv[4] != "nooracle"
    max_nodes = int(sys.argv[5]) if len(sys.argv) > 5 else 200000
    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    st = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    s = CentSolver(cent_problem(N), [st])
    x0 = np.stack([O.env_initial_state(n, p).astype(float).reshape(n, 2) for p in range(S)])
    t0 = time.perf_counter()
    res = s.solve(np.zeros((S, n), np.int32), x0, leader_window(N), max_nodes=max_nodes)
    dt = time.perf_counter() - t0
    stt = s.stats()
    print(f"device: {S} platoons n={n} N={N} in {dt:.3f}s (kernel {stt.last_ms:.1f} ms), QPs {stt.n_candidates}, "
          f"iters {stt.qp_iterations}, status {np.bincount(res.status, minlength=4).tolist()}", flush=True)
    q = np.percentile(res.nodes, [0, 50, 90, 99, 100])
    print(f"nodes per platoon: min {q[0]:.0f} p50 {q[1]:.0f} p90 {q[2]:.0f} p99 {q[3]:.0f} max {q[4]:.0f}; "
          f"mean iters/QP {res.iters.sum() / max(1, res.nodes.sum()):.1f}", flush=True)
    odd = np.flatnonzero(res.status != 0)
    if len(odd):
        print(f"non-optimal platoons (seed: status, nodes): "
              f"{[(int(p), int(res.status[p]), int(res.nodes[p])) for p in odd[:12]]}", flush=True)
    if not oracle_check:
        return
    bad = 0
    for p in range(S):
        line = f"  p={p} st={res.status[p]} cost={res.cost[p]:.9f} nodes={res.nodes[p]} iters={res.iters[p]}"
        if oracle_check:
            r = O.solve_cent([O.gear_pwa_system(800.0)] * n, O.Cfg(), N, x0[p].reshape(-1), leader_window(N))
            same = np.array_equal(r.sigma, res.region[p])
            dc = abs(r.cost - res.cost[p]) / max(1.0, abs(r.cost))
            du = np.abs(r.u - res.u[p]).max()
            line += f" | oracle cost={r.cost:.9f} nodes={r.n_qps} same_sigma={same} dcost={dc:.2e} du={du:.2e}"
            if not same:
                line += f"\n    dev {res.region[p].tolist()}\n    ora {r.sigma.tolist()}"
            bad += (not same) or dc > 1e-9 or r.n_qps != res.nodes[p]
        print(line, flush=True)
    print(f"mismatches: {bad}")


if __name__ == "__main__":
    main()
