"""The CPU oracle against independent solvers (no GPU).

* golden regression: the oracle reproduces the committed fixtures;
* fixed-sequence QPs against scipy's trust-constr on the oracle's own dense export;
* region-sequence enumeration against brute force: every one of the 7^N sequences checked for
  feasibility of the velocity constraints with HiGHS (scipy.optimize.linprog);
* the MIQP layer against HiGHS MILP (scipy.optimize.milp) on the reference's big-M MLD
  formulation with the L1 cost (min_1_norm): an independent exact MIP solver on the model the
  reference hands to Gurobi.
"""

from __future__ import annotations

import itertools

import numpy as np
import pytest

import oracle as O
from golden_io import fixture_names, load
from instances import decent_instances, leader_window, split_params


@pytest.mark.parametrize("name", [n for n in fixture_names() if n.startswith(("decent_n2", "variant_n4_N3"))])
def test_oracle_reproduces_golden(name):
    fx = load(name)
    N = int(fx["N"])
    cv = fx["cfg"]
    cfg = O.Cfg(Qx=tuple(cv[0:4]), Qu=cv[4], Qdu=cv[5], w=cv[6], a_acc=cv[7], a_dec=cv[8], ts=cv[9], d_safe=cv[10],
                tight=cv[11], d0=cv[12], t0=cv[13])
    systems = [O.gear_pwa_system(float(m)) for m in fx["masses"]]
    for i, (p, r, s) in enumerate(zip(fx["params"], fx["roles"], fx["sys"])):
        x0, xf, xb, xl = split_params(p, N)
        res = O.solve_miqp(systems[s], cfg, N, int(r), x0, xf, xb, xl)
        assert res.status == fx["exp_status"][i]
        assert list(res.sigma) == list(fx["exp_region"][i])
        assert abs(res.cost - fx["exp_cost"][i]) <= 1e-10 * max(1, abs(res.cost))
        assert res.n_candidates == fx["exp_nodes"][i]


def _instance(seed=0, n=4, N=5, i=1):
    params, roles = decent_instances(O.env_initial_state(n, seed), N, leader_window(N))
    return params[i], int(roles[i])


def test_certify_batch_reproduces_golden():
    """oracle_certify_batch (the full-size KKT check of the GPU answers) on the golden sequences:
    certified, the fixture's cost and u."""
    fx = load("decent_n10_N5.npz")
    systems = [O.gear_pwa_system(float(m)) for m in fx["masses"]]
    obj, cert, u = O.certify_batch(systems, O.Cfg(), int(fx["N"]), fx["sys"], fx["roles"], fx["params"],
                                   fx["exp_region"], nthreads=4)
    ok = fx["exp_status"] == 0
    assert cert[ok].all()
    # the IPM objective of a fresh solve agrees to ~1e-8 absolute (costs 1 .. 1e5)
    assert np.all(np.abs(obj[ok] - fx["exp_cost"][ok]) <= 1e-9 * np.abs(fx["exp_cost"][ok]) + 1e-7)
    assert np.abs(u[ok] - fx["exp_u"][ok]).max() <= 1e-6


@pytest.mark.parametrize("seed,veh", [(0, 0), (1, 1), (2, 3), (5, 2)])
def test_fixed_sequence_qp_vs_scipy(seed, veh):
    from scipy.optimize import LinearConstraint, minimize

    N = 5
    sysd = O.gear_pwa_system(800.0)
    p, role = _instance(seed, 4, N, veh)
    x0, xf, xb, xl = split_params(p, N)
    cands = O.candidates(sysd, O.Cfg(), N, x0)
    for sig in cands[:: max(1, len(cands) // 4)]:
        obj, conv, cert, z, _ = O.solve_qp(sysd, O.Cfg(), N, role, sig, x0, xf, xb, xl)
        assert conv and cert
        P, q, r0, A, b, G, h = O.export_qp(sysd, O.Cfg(), N, role, sig, x0, xf, xb, xl)
        f = lambda v: 0.5 * v @ P @ v + q @ v + r0  # noqa: E731
        res = minimize(f, z + 1e-3, jac=lambda v: P @ v + q, method="trust-constr",
                       constraints=[LinearConstraint(A, b, b), LinearConstraint(G, -np.inf, h)],
                       options=dict(maxiter=3000, gtol=1e-10, xtol=1e-12))
        assert res.constr_violation < 1e-6
        # the oracle is never worse than scipy and agrees to scipy's accuracy
        assert obj <= res.fun + 1e-6 * max(1, abs(obj))
        assert abs(obj - res.fun) <= 1e-5 * max(1, abs(obj))


@pytest.mark.parametrize("seed,v0", [(0, None), (3, None), (1, 9.3), (2, 22.95), (4, 32.4)])
def test_enumeration_matches_lp_feasibility(seed, v0):
    """Every sequence of {0..6}^3: pruned  <=>  its velocity constraints are LP-infeasible."""
    from scipy.optimize import linprog

    N = 3
    sysd = O.gear_pwa_system(800.0)
    p, role = _instance(seed, 3, N, 1)
    x0 = p[:2].copy()
    if v0 is not None:
        x0[1] = v0
    got = {tuple(s) for s in O.candidates(sysd, O.Cfg(), N, x0)}
    A11, B1, c1 = sysd["A"][:, 1, 1], sysd["B"][:, 1], sysd["c"][:, 1]
    lo = np.where(sysd["S"][:, 1, 1] < 0, -sysd["T"][:, 1], -np.inf)
    hi = np.where(sysd["S"][:, 0, 1] > 0, sysd["T"][:, 0], np.inf)
    for seq in itertools.product(range(7), repeat=N):
        if not (lo[seq[0]] <= x0[1] <= hi[seq[0]]):
            feas = False
        else:
            # variables v_1..v_N, u_0..u_{N-1}
            nv = 2 * N
            Aeq, beq, Aub, bub, bounds = [], [], [], [], []
            for k in range(N):
                r = seq[k]
                row = np.zeros(nv)
                row[k] = 1.0
                row[N + k] = -B1[r]
                if k:
                    row[k - 1] = -A11[r]
                    beq.append(c1[r])
                else:
                    beq.append(c1[r] + A11[r] * x0[1])
                Aeq.append(row)
                # accel rows
                row = np.zeros(nv)
                row[k] = 1.0
                if k:
                    row[k - 1] = -1.0
                    Aub.append(row); bub.append(2.5)
                    Aub.append(-row); bub.append(2.0)
                else:
                    Aub.append(row); bub.append(2.5 + x0[1])
                    Aub.append(-row); bub.append(2.0 - x0[1])
            for k in range(N):  # v_{k+1} bounds: box and region of step k+1
                l, h_ = 3.94, 45.84
                if k + 1 < N:
                    l, h_ = max(l, lo[seq[k + 1]]), min(h_, hi[seq[k + 1]])
                bounds.append((l, h_))
            bounds += [(-1.0, 1.0)] * N
            if any(b0 > b1 for b0, b1 in bounds):
                feas = False
            else:
                res = linprog(np.zeros(nv), A_ub=np.array(Aub), b_ub=bub, A_eq=np.array(Aeq), b_eq=beq,
                              bounds=bounds, method="highs")
                feas = res.status == 0
        assert feas == (seq in got), (seq, feas)


def _milp_l1(sysd, cfg, N, role, x0, xf, xb, xl):
    """The reference's MLD (dmpcpwa big-M) with min_1_norm, solved by HiGHS MILP."""
    from scipy.optimize import Bounds, LinearConstraint, milp

    s = 7
    # variable layout: x (2, N+1) | u (N) | delta (s, N) | z (2, s, N) | sf (N+1) | sb (N+1) | aux ...
    idx = {}
    nv = 0

    def add(name, count):
        nonlocal nv
        idx[name] = nv
        nv += count

    add("x", 2 * (N + 1)); add("u", N); add("d", s * N); add("z", 2 * s * N); add("sf", N + 1); add("sb", N + 1)
    terms = []  # (vector e over variables + const, weight) for |.|
    X = lambda i, k: idx["x"] + i * (N + 1) + k  # noqa: E731
    rows, lo_, hi_ = [], [], []

    def con(coefs, lb, ub):
        r = np.zeros(nv_max)
        for j, c in coefs:
            r[j] += c
        rows.append(r); lo_.append(lb); hi_.append(ub)

    # aux for the L1 terms
    naux = 0
    aux_terms = []
    for k in range(N + 1):
        if role & O.ROLE_TRACK_LEADER:
            aux_terms.append(([(X(0, k), 1.0)], -xl[0, k], cfg.Qx[0]))
            aux_terms.append(([(X(1, k), 1.0)], -xl[1, k], cfg.Qx[3]))
        if role & O.ROLE_TRACK_FRONT:
            aux_terms.append(([(X(0, k), 1.0), (X(1, k), cfg.t0)], cfg.d0 - xf[0, k], cfg.Qx[0]))
            aux_terms.append(([(X(1, k), 1.0)], -xf[1, k], cfg.Qx[3]))
        if role & O.ROLE_TRACK_BACK:
            aux_terms.append(([(X(0, k), -1.0)], xb[0, k] + cfg.t0 * xb[1, k] + cfg.d0, cfg.Qx[0]))
            aux_terms.append(([(X(1, k), -1.0)], xb[1, k], cfg.Qx[3]))
    for k in range(N):
        aux_terms.append(([(idx["u"] + k, 1.0)], 0.0, cfg.Qu))
    idx["aux"] = nv
    nv += len(aux_terms)
    nv_max = nv
    cost = np.zeros(nv)
    for a, (e, c0, wgt) in enumerate(aux_terms):
        j = idx["aux"] + a
        cost[j] = 1.0
        con([(v, wgt * cf) for v, cf in e] + [(j, -1.0)], -np.inf, -wgt * c0)   # Q e - y <= 0
        con([(v, -wgt * cf) for v, cf in e] + [(j, -1.0)], -np.inf, wgt * c0)   # -Q e - y <= 0
    for k in range(N + 1):
        cost[idx["sf"] + k] = cfg.w
        cost[idx["sb"] + k] = cfg.w
    # initial state
    con([(X(0, 0), 1.0)], x0[0], x0[0]); con([(X(1, 0), 1.0)], x0[1], x0[1])
    # big-M bounds over the box (p in [0, 1e4], v in [vmin, vmax] -- x0 inside)
    pb, vb, ub_ = (0.0, 1e4), (3.94, 45.84), (-1.0, 1.0)
    for k in range(N):
        con([(idx["d"] + r * N + k, 1.0) for r in range(s)], 1, 1)
        for r in range(s):
            dk = idx["d"] + r * N + k
            for row in range(2):
                Srow, T = sysd["S"][r][row], sysd["T"][r][row]
                if not Srow.any():
                    continue
                ex = Srow[0] * np.array(pb) + Srow[1] * np.array(vb)
                M = max(ex) - T
                # S x - T <= M (1 - d)
                con([(X(0, k), Srow[0]), (X(1, k), Srow[1]), (dk, M)], -np.inf, T + M)
            for i in range(2):
                zi = idx["z"] + (i * s + r) * N + k
                A, B, c = sysd["A"][r][i], sysd["B"][r][i], sysd["c"][r][i]
                vals = [A[0] * p + A[1] * v + B * u + c for p in pb for v in vb for u in ub_]
                lo_b, hi_b = min(vals), max(vals)
                aff = [(X(0, k), A[0]), (X(1, k), A[1]), (idx["u"] + k, B)]
                con([(zi, 1.0), (dk, -hi_b)], -np.inf, 0)
                con([(zi, 1.0), (dk, -lo_b)], 0, np.inf)
                con([(zi, 1.0)] + [(j, -cf) for j, cf in aff] + [(dk, -lo_b)], -np.inf, c - lo_b)
                con([(zi, 1.0)] + [(j, -cf) for j, cf in aff] + [(dk, -hi_b)], c - hi_b, np.inf)
        for i in range(2):
            con([(X(i, k + 1), 1.0)] + [(idx["z"] + (i * s + r) * N + k, -1.0) for r in range(s)], 0, 0)
        con([(X(1, k + 1), 1.0), (X(1, k), -1.0)], cfg.a_dec * cfg.ts + k * cfg.tight, cfg.a_acc * cfg.ts - k * cfg.tight)
    lb = np.full(nv, -np.inf)
    ub = np.full(nv, np.inf)
    for k in range(1, N + 1):
        lb[X(0, k)], ub[X(0, k)] = pb
        lb[X(1, k)], ub[X(1, k)] = vb
    lb[idx["u"]:idx["u"] + N], ub[idx["u"]:idx["u"] + N] = -1, 1
    lb[idx["d"]:idx["d"] + s * N], ub[idx["d"]:idx["d"] + s * N] = 0, 1
    for k in range(N + 1):
        lb[idx["sf"] + k] = 0
        lb[idx["sb"] + k] = 0
        ub[idx["sf"] + k] = np.inf if role & O.ROLE_SAFE_FRONT else 0
        ub[idx["sb"] + k] = np.inf if role & O.ROLE_SAFE_BACK else 0
        if role & O.ROLE_SAFE_FRONT:
            con([(X(0, k), 1.0), (idx["sf"] + k, -1.0)], -np.inf, xf[0, k] - cfg.d_safe)
        if role & O.ROLE_SAFE_BACK:
            con([(X(0, k), 1.0), (idx["sb"] + k, 1.0)], xb[0, k] + cfg.d_safe, np.inf)
    integrality = np.zeros(nv)
    integrality[idx["d"]:idx["d"] + s * N] = 1
    res = milp(cost, constraints=LinearConstraint(np.array(rows)[:, :nv], lo_, hi_), integrality=integrality,
               bounds=Bounds(lb, ub), options={"mip_rel_gap": 1e-9, "presolve": True})
    return res


@pytest.mark.slow
@pytest.mark.parametrize("seed,veh", [(0, 0), (0, 1), (1, 2), (2, 3), (3, 1)])
def test_miqp_l1_vs_highs_milp(seed, veh):
    N = 4
    sysd = O.gear_pwa_system(800.0)
    p, role = _instance(seed, 4, N, veh)
    x0, xf, xb, xl = split_params(p, N)
    ora = O.solve_miqp(sysd, O.Cfg(), N, role, x0, xf, xb, xl, quadratic=False)
    ref = _milp_l1(sysd, O.Cfg(), N, role, x0, xf, xb, xl)
    assert ora.status == 0 and ref.status == 0
    assert abs(ora.cost - ref.fun) <= 1e-6 * max(1.0, abs(ref.fun)), (ora.cost, ref.fun)


@pytest.mark.parametrize("n,N,seed", [(4, 5, 0), (4, 6, 1), (3, 7, 2), (10, 5, 3)])
def test_oracle_branch_and_bound_equals_enumeration(n, N, seed):
    """The oracle's branch and bound (used for the N = 10 / 15 sweep fixtures, where exhaustive
    enumeration needs ~1e4 .. 1e6 QPs per vehicle) returns exactly what its exhaustive
    enumeration returns: same sequence (tie rule included), same cost, same trajectory."""
    sysd = O.gear_pwa_system(800.0)
    params, roles = decent_instances(O.env_initial_state(n, seed), N, leader_window(N))
    for p, r in zip(params, roles):
        x0, xf, xb, xl = split_params(p, N)
        O.set_method(O.METHOD_ENUMERATE)
        a = O.solve_miqp(sysd, O.Cfg(), N, int(r), x0, xf, xb, xl)
        O.set_method(O.METHOD_BNB)
        try:
            b = O.solve_miqp(sysd, O.Cfg(), N, int(r), x0, xf, xb, xl)
        finally:
            O.set_method(O.METHOD_ENUMERATE)
        assert a.status == b.status == 0
        assert list(a.sigma) == list(b.sigma)
        assert abs(a.cost - b.cost) <= 1e-10 * max(1.0, abs(a.cost))
        assert np.abs(a.u - b.u).max() <= 1e-7
        assert b.n_candidates < a.n_candidates or N <= 5


def test_gear_model_restatement():
    """MpcGear on pwa_friction (mpcs/mpc_gear.py:30-114): one mode per (gear, friction region),
    band = gear window ∩ region, input gain B_r * Vehicle.b[j] on u_g.  Branch and bound and
    enumeration agree on it, and every optimal mode respects its gear's velocity window."""
    g = O.gear_friction_mld_system(800.0)
    assert list(g["gear"]) == [1, 2, 3, 4, 4, 5, 5, 6, 6]
    assert list(g["friction"]) == [0, 0, 0, 0, 1, 0, 1, 0, 1]
    assert np.allclose(g["B"][:, 1] * 800.0, [4057, 2945, 2116, 1607, 1607, 1166, 1166, 838, 838])
    N = 4
    params, roles = decent_instances(O.env_initial_state(3, 5), N, leader_window(N))
    vl = np.array([3.94, 5.43, 7.56, 9.96, 13.70, 19.10])
    vh = np.array([9.46, 13.04, 18.15, 23.90, 32.93, 45.84])
    for p, r in zip(params, roles):
        x0, xf, xb, xl = split_params(p, N)
        a = O.solve_miqp(g, O.Cfg(), N, int(r), x0, xf, xb, xl)
        O.set_method(O.METHOD_BNB)
        try:
            b = O.solve_miqp(g, O.Cfg(), N, int(r), x0, xf, xb, xl)
        finally:
            O.set_method(O.METHOD_ENUMERATE)
        assert a.status == b.status == 0
        assert list(a.sigma) == list(b.sigma)
        assert abs(a.cost - b.cost) <= 1e-10 * max(1.0, abs(a.cost))
        gears = g["gear"][a.sigma] - 1
        v = a.x[1, :N]
        assert np.all(v >= vl[gears] - 1e-7) and np.all(v <= vh[gears] + 1e-7)
        assert np.abs(a.u).max() <= 1 + 1e-9
