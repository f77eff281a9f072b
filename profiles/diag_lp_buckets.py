#!/usr/bin/env python3
"""Round 6 diagnostic: do a min_1_norm node LP's simplex pivots follow its
parent's, as the QP path's active-set steps do (correlation 0.84, DESIGN.md section 4 "Level lists
in buckets")?  And what would bucketing the LP refill kernel's level lists by the parent's pivot count
buy?

The product's search and simplex compiled for the host (lib/libhvp_hostref.so, hvp_hostref.cpp
solve_one_bnb records every node LP's (parent pivots, own pivots)) over C2-size min_1_norm instances
(n = 10, N = 5, env.reset states).  Model of the refill kernel (k_lp_bound_refill): a wave takes 64
nodes of a level at a time and runs until its slowest LP is done, so a generation costs the maximum
of its 64 pivot counts; the nodes of a level are drawn (a) in list order -- modelled as a random
order -- or (b) from buckets split on the parent's pivot count (bucket 0 first), as LevelList does.

    python profiles/diag_lp_buckets.py [platoons]   -> profiles/r06_lp_parent_child.txt
"""

from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hybrid-vehicle-platoon_amd"))
sys.path.insert(0, ROOT)


def main() -> None:
    from bench import make_inputs
    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle

    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    n, N = 10, 5
    L = ctypes.CDLL(_abi.HOSTREF_PATH)
    veh = PwaGearVehicle(800)
    S = (_abi.HvpSystem * 1)(tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh)))
    prob = tables.problem(N, quadratic_cost=False, method=_abi.METHOD_BNB)
    L.hvp_hostref_set_l1_solver(1)
    hist = (ctypes.c_longlong * 1024)()
    L.hvp_hostref_lp_parent_child(hist)  # reset
    params, roles = make_inputs(range(0, P), n, N)
    B = len(roles)
    bufs = [np.zeros((B, N)), np.zeros((B, 2, N + 1)), np.zeros((B, N), np.int8), np.zeros(B),
            np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(B, np.int32)]
    f = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.hvp_hostref_solve_batch(ctypes.byref(prob), S, B, f(np.zeros(B, np.int32)), f(roles),
                              f(np.ascontiguousarray(params)), *[f(b) for b in bufs], 8)
    L.hvp_hostref_lp_parent_child(hist)
    H = np.array(hist[:], dtype=np.int64).reshape(32, 32)
    pp, cc = np.nonzero(H)
    w = H[pp, cc].astype(float)
    tot = w.sum()
    mp, mc = (w * pp).sum() / tot, (w * cc).sum() / tot
    cov = (w * (pp - mp) * (cc - mc)).sum() / tot
    corr = cov / np.sqrt((w * (pp - mp) ** 2).sum() / tot * (w * (cc - mc) ** 2).sum() / tot)
    pairs = np.repeat(np.stack([pp, cc], 1), H[pp, cc], axis=0)
    rng = np.random.default_rng(0)

    def gen_cost(order_children):
        m = len(order_children) // 64 * 64
        return order_children[:m].reshape(-1, 64).max(axis=1).sum(), order_children[:m].sum()

    base, busy = gen_cost(rng.permutation(pairs[:, 1]))
    lines = [f"# profiles/diag_lp_buckets.py: {P} platoons x {n} local MILPs (n = {n}, N = {N}, min_1_norm, "
             f"branch and bound, per-lane simplex), host build of the product's search",
             f"node LPs (levels 1..N): {int(tot)}; mean pivots: parent {mp:.2f}, child {mc:.2f}; "
             f"correlation parent -> child pivots: {corr:.3f}",
             f"generation model (64 nodes, cost = max pivots): random order {base} pivot-cycles "
             f"(lane utilisation {busy / (64.0 * base):.3f})"]
    for split in ([4], [6], [8], [4, 8], [3, 6, 10]):
        b = np.digitize(pairs[:, 0], split)
        cost = 0
        for q in range(len(split) + 1):
            cost += gen_cost(rng.permutation(pairs[b == q, 1]))[0]
        lines.append(f"  buckets split at parent pivots {split}: {cost} ({cost / base - 1:+.1%})")
    lines.append("child pivots by parent pivots (rows 0..15, mean / count):")
    for i in range(16):
        if H[i].sum():
            lines.append(f"  {i:2d}: {(H[i] * np.arange(32)).sum() / H[i].sum():5.2f}  {H[i].sum()}")
    out = "\n".join(lines)
    print(out)
    with open(os.path.join(ROOT, "profiles", "r06_lp_parent_child.txt"), "w") as fo:
        fo.write(out + "\n")


if __name__ == "__main__":
    main()
