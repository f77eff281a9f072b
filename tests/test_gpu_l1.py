"""GPU parity of the min_1_norm cost (quadratic_cost=False, fleet_decent_mld.py:73-76).

The local MILP of LocalMpcMld / LocalMpcGear with the L1 norm, by either search:
  * enumeration (N <= 8): the device enumerates the velocity-feasible region sequences (k_enum),
    solves every fixed-sequence LP by the interior point of csrc/hvp_l1.h (k_qp_l1), prices it term
    by term (k_cost) and applies the same tie rule (k_select);
  * branch and bound (any N, the default beyond N = 8): node LPs relaxed after K steps, one per
    wavefront (k_l1_root / k_l1_bound), children by k_bnb_expand, the same tie rule (k_bnb_key).
Checked against the oracle's MILP optima (the oracle's L1 path is pinned to HiGHS milp on the
reference's big-M MLD, tests/test_oracle.py).  Bar: region sequences, gears and (enumeration)
sequence counts exact; cost 1e-9 relative; u 1e-6; x 1e-4 (positions ~3e3).  LPs proven
infeasible are excluded; an LP left unresolved makes its instance HVP_MAXITER.
"""

from __future__ import annotations

import numpy as np
import pytest

import oracle as O
from golden_io import expected_gears, l1_fixture_names, load, product_problem
from instances import decent_instances, leader_window, oracle_solve

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", l1_fixture_names())
def test_l1_enumeration_fixture_on_gpu(gpu_available, name):
    from hvp.solver import BatchSolver

    from hvp import _abi

    fx = load(name)
    if int(fx["N"]) > 8:
        pytest.skip("beyond exhaustive enumeration (HVP_MAX_N_ENUM): branch and bound only")
    prob, systems = product_problem(fx)
    assert prob.quadratic_cost == 0
    prob.method = _abi.METHOD_ENUMERATE
    s = BatchSolver(prob, systems)
    res = s.solve(fx["sys"], fx["roles"], fx["params"])
    assert np.array_equal(res.status, fx["exp_status"])
    if int(fx.get("method", 0)) == 0:  # enumeration on both sides: same sequence counts
        assert np.array_equal(res.nodes, fx["exp_nodes"])
    assert np.array_equal(res.region, fx["exp_region"])
    assert np.array_equal(res.gear, expected_gears(fx))
    ce = fx["exp_cost"]
    assert np.all(np.abs(res.cost - ce) <= 1e-9 * np.maximum(1, np.abs(ce)))
    assert np.abs(res.u - fx["exp_u"]).max() <= 1e-6
    assert np.abs(res.x - fx["exp_x"]).max() <= 1e-4


def _l1_cost(x, u, params, roles, N, cfg=O.Cfg()):
    """min_1_norm objective of trajectories (numpy restatement of fleet_decent_mld.py:107-169)."""
    K1 = N + 1
    xf = params[:, 2:2 + 2 * K1].reshape(-1, 2, K1)
    xb = params[:, 2 + 2 * K1:2 + 4 * K1].reshape(-1, 2, K1)
    xl = params[:, 2 + 4 * K1:].reshape(-1, 2, K1)
    p, v = x[:, 0, :], x[:, 1, :]
    has = lambda bit: ((roles & bit) != 0)[:, None]  # noqa: E731
    J = np.zeros(len(roles))
    J += (has(O.ROLE_TRACK_FRONT) * (cfg.Qx[0] * np.abs(p + cfg.d0 - xf[:, 0]) + cfg.Qx[3] * np.abs(v - xf[:, 1]))).sum(1)
    J += (has(O.ROLE_TRACK_BACK) * (cfg.Qx[0] * np.abs(xb[:, 0] + cfg.d0 - p) + cfg.Qx[3] * np.abs(xb[:, 1] - v))).sum(1)
    J += (has(O.ROLE_TRACK_LEADER) * (cfg.Qx[0] * np.abs(p - xl[:, 0]) + cfg.Qx[3] * np.abs(v - xl[:, 1]))).sum(1)
    J += (has(O.ROLE_SAFE_FRONT) * cfg.w * np.maximum(0, p - xf[:, 0] + cfg.d_safe)).sum(1)
    J += (has(O.ROLE_SAFE_BACK) * cfg.w * np.maximum(0, xb[:, 0] + cfg.d_safe - p)).sum(1)
    J += cfg.Qu * np.abs(u).sum(1)
    return J


def test_l1_platoon_batch(gpu_available):
    """4096 local MILPs (n = 10, N = 5, 410 platoon seeds): every answer feasible, its reported
    cost the min_1_norm objective of its own (x, u), deterministic, and a sample equal to the
    oracle's MILP optimum (sequence, cost, u)."""
    import torch

    from hvp import tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    n, N = 10, 5
    veh = PwaGearVehicle(800.0)
    s = BatchSolver(tables.problem(N, quadratic_cost=False), [tables.system_from_dict(veh.get_discrete_system(1),
                                                                                       tables.gears_of(veh))])
    P, R = [], []
    for seed in range(410):
        p, r = decent_instances(O.env_initial_state(n, seed), N, leader_window(N))
        P.append(p)
        R.append(r)
    params, roles = np.concatenate(P), np.concatenate(R)
    dev = torch.device("cuda", 0)
    tp, tr = torch.from_numpy(params).to(dev), torch.from_numpy(roles).to(dev)
    ts = torch.zeros(len(roles), dtype=torch.int32, device=dev)
    a = s.solve_device(ts, tr, tp)
    b = s.solve_device(ts, tr, tp)
    torch.cuda.synchronize()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    st = a["status"].cpu().numpy()
    assert (st == 0).all()
    u, x, reg = a["u"].cpu().numpy(), a["x"].cpu().numpy(), a["region"].cpu().numpy()
    cost = a["cost"].cpu().numpy()
    assert np.abs(u).max() <= 1 + 1e-9
    v = x[:, 1, :]
    assert v[:, 1:].min() >= 3.94 - 1e-9 and v[:, 1:].max() <= 45.84 + 1e-9
    dv = np.diff(v, axis=1)
    assert dv.min() >= -2 - 1e-9 and dv.max() <= 2.5 + 1e-9
    lim = np.array([-np.inf, 9.235, 12.855, 16.93, 22.92, 23.315, 32.47, np.inf])
    assert np.all(v[:, :N] >= lim[reg] - 1e-7) and np.all(v[:, :N] <= lim[reg + 1] + 1e-7)
    g = O.gear_pwa_system(800.0)
    assert np.abs(g["A"][reg, 1, 1] * v[:, :N] + g["B"][reg, 1] * u + g["c"][reg, 1] - v[:, 1:]).max() <= 1e-9
    assert np.all(np.abs(_l1_cost(x, u, params, roles, N) - cost) <= 1e-9 * np.maximum(1, np.abs(cost)))
    rng = np.random.default_rng(1)
    idx = rng.choice(len(roles), 40, replace=False)
    ref = oracle_solve(g, O.Cfg(), N, params[idx], roles[idx], quadratic=False)
    face = []
    for j, r in zip(idx, ref):
        assert list(reg[j]) == list(r.sigma), j
        assert abs(cost[j] - r.cost) <= 1e-9 * max(1.0, abs(r.cost)), j
        # where the LP optimum is a face, the simplex (hvp_lp.h) returns a vertex of it and the
        # oracle's interior point a point inside: both optimal.  The device's (x, u) is priced by
        # the ORACLE's own LP of that sequence (oracle_export_qp: its rows and objective, with the
        # slack / epigraph variables re-optimised for the fixed trajectory) at the oracle's optimum
        if np.abs(u[j] - r.u).max() > 1e-6:
            face.append(int(j))
            p = params[j]
            K = 2 * (N + 1)
            val = reprice_l1(g, O.Cfg(), N, int(roles[j]), reg[j], p[:2], p[2:2 + K].reshape(2, -1),
                             p[2 + K:2 + 2 * K].reshape(2, -1), p[2 + 2 * K:].reshape(2, -1), x[j], u[j])
            assert abs(val - r.cost) <= 1e-8 * max(1.0, abs(r.cost)), (j, val, r.cost)
    # the sample is fixed (40 of the 4100 instances, rng seed 1) and so is the vertex the simplex
    # returns: the face instances are pinned (MI355X r05b), so a change of the solver's vertex choice
    # shows up here
    assert face == L1_FACE_INSTANCES, face


# instances of test_l1_platoon_batch's fixed sample where the LP optimum is a face and the device's
# vertex differs from the oracle's interior point (the host build of the same simplex: none)
L1_FACE_INSTANCES: list = []


def reprice_l1(sysd, cfg, N, role, sigma, x0, xf, xb, xl, x, u):
    """The oracle's min_1_norm objective (oracle_export_qp: the full (x, u, s, aux) LP of the fixed
    sequence, fleet_decent_mld.py:73-208) at the trajectory (x, u): x_1..x_N and u fixed, the slack and
    epigraph variables minimised (scipy HiGHS); every equality and inequality row must hold."""
    from scipy.optimize import linprog

    P, q, r0, A, b, G, h = O.export_qp(sysd, cfg, N, role, sigma, x0, xf, xb, xl, quadratic=False)
    assert not P.any()
    nz = len(q)
    fixed = np.concatenate([np.asarray(x)[:, 1:].T.reshape(-1), np.asarray(u)])  # z = [x_1 .. x_N | u | ...]
    lo = np.full(nz, -np.inf)
    hi = np.full(nz, np.inf)
    lo[:3 * N] = hi[:3 * N] = fixed
    res = linprog(q, A_ub=G, b_ub=h, A_eq=A, b_eq=b, bounds=list(zip(lo, hi)),
                  method="highs")
    assert res.status == 0, res.message
    return float(res.fun + r0)


def test_l1_local_mpc_api(gpu_available):
    """The reference call surface: LocalMpcMld(quadratic_cost=False).solve_mpc after the setters."""
    from hvp.models import PwaGearVehicle
    from hvp.mpc import LocalMpcMld

    N = 5
    veh = PwaGearVehicle(800.0)
    mpc = LocalMpcMld(N, veh.get_discrete_system(1), quadratic_cost=False)
    x = O.env_initial_state(3, 7).reshape(-1)
    xf = O.constant_velocity_prediction(x[0], x[1], N)
    xb = O.constant_velocity_prediction(x[4], x[5], N)
    mpc.set_x_front(xf)
    mpc.set_x_back(xb)
    u0, info = mpc.solve_mpc(x[2:4].reshape(2, 1))
    r = O.solve_miqp(O.gear_pwa_system(800.0), O.Cfg(), N, O.role_bits(1, 3, 0, False), x[2:4], xf, xb,
                     np.zeros((2, N + 1)), quadratic=False)
    assert abs(info["cost"] - r.cost) <= 1e-9 * max(1.0, abs(r.cost))
    assert np.abs(info["u"].ravel() - r.u).max() <= 1e-6
    assert abs(float(u0[0, 0]) - r.u[0]) <= 1e-6


def test_l1_local_mpc_gear_evaluate(gpu_available):
    """LocalMpcGear (pwa_friction) with min_1_norm: solve_mpc against the oracle MILP, and
    evaluate_cost (mpcs/mpc_gear.py:137-170) of its own optimum returns the same cost; an
    infeasible (u, gear) returns 'inf'."""
    from hvp.models import PwaFrictionVehicle
    from hvp.mpc import LocalMpcGear

    N = 5
    veh = PwaFrictionVehicle(800.0)
    m = LocalMpcGear(N, veh.get_discrete_system(1), quadratic_cost=False)
    x = O.env_initial_state(3, 4).reshape(-1)
    xf = O.constant_velocity_prediction(x[0], x[1], N)
    xb = O.constant_velocity_prediction(x[4], x[5], N)
    m.set_x_front(xf)
    m.set_x_back(xb)
    _, info = m.solve_mpc(x[2:4].reshape(2, 1))
    r = O.solve_miqp(O.gear_friction_mld_system(800.0), O.Cfg(), N, O.role_bits(1, 3, 0, False), x[2:4], xf, xb,
                     np.zeros((2, N + 1)), quadratic=False)
    assert abs(info["cost"] - r.cost) <= 1e-9 * max(1.0, abs(r.cost))
    c = m.evaluate_cost(x[2:4].reshape(2, 1), info["u"][[0]], info["u"][[1]])
    assert abs(c - info["cost"]) <= 1e-9 * max(1.0, abs(info["cost"]))
    assert m.evaluate_cost(x[2:4].reshape(2, 1), np.ones((1, N)), np.ones((1, N))) == "inf"


@pytest.mark.parametrize("name", l1_fixture_names())
def test_l1_branch_and_bound_fixture_on_gpu(gpu_available, name):
    """Every min_1_norm fixture by branch and bound (N = 3..10): same answers as the oracle."""
    from hvp import _abi
    from hvp.solver import BatchSolver

    fx = load(name)
    prob, systems = product_problem(fx)
    prob.method = _abi.METHOD_BNB
    res = BatchSolver(prob, systems).solve(fx["sys"], fx["roles"], fx["params"])
    assert np.array_equal(res.status, fx["exp_status"])
    assert np.array_equal(res.region, fx["exp_region"])
    assert np.array_equal(res.gear, expected_gears(fx))
    ce = fx["exp_cost"]
    assert np.all(np.abs(res.cost - ce) <= 1e-9 * np.maximum(1, np.abs(ce)))
    assert np.abs(res.u - fx["exp_u"]).max() <= 1e-6
    assert np.abs(res.x - fx["exp_x"]).max() <= 1e-4
    if int(fx["N"]) >= 5 and int(fx.get("method", 0)) == 0:
        assert res.nodes.mean() < fx["exp_nodes"].mean()  # the search prunes


def test_l1_branch_and_bound_equals_enumeration_at_batch(gpu_available):
    """4100 local MILPs (n = 10, N = 5): branch and bound and enumeration return the same
    sequence, cost and trajectory for every instance (a size-independent property: both are
    exact with the same tie rule)."""
    import torch

    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    n, N = 10, 5
    veh = PwaGearVehicle(800.0)
    table = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    P, R = [], []
    for seed in range(1000, 1410):
        p, r = decent_instances(O.env_initial_state(n, seed), N, leader_window(N))
        P.append(p)
        R.append(r)
    params, roles = np.concatenate(P), np.concatenate(R)
    dev = torch.device("cuda", 0)
    tp, tr = torch.from_numpy(params).to(dev), torch.from_numpy(roles).to(dev)
    ts = torch.zeros(len(roles), dtype=torch.int32, device=dev)
    out = {}
    for m in (_abi.METHOD_ENUMERATE, _abi.METHOD_BNB):
        s = BatchSolver(tables.problem(N, quadratic_cost=False, method=m), [table])
        out[m] = {k: v.cpu().numpy() for k, v in s.solve_device(ts, tr, tp).items()}
    e, b = out[_abi.METHOD_ENUMERATE], out[_abi.METHOD_BNB]
    assert (e["status"] == 0).all() and (b["status"] == 0).all()
    assert np.array_equal(e["region"], b["region"])
    assert np.all(np.abs(e["cost"] - b["cost"]) <= 1e-9 * np.maximum(1, np.abs(e["cost"])))
    # the same leaf LP by the same solver in both searches: the same vertex
    assert np.abs(e["u"] - b["u"]).max() <= 1e-6
    assert b["nodes"].mean() < e["nodes"].mean()


def test_l1_refill_kernels_equal_grid_stride_kernels(gpu_available, monkeypatch):
    """4100 local MILPs (n = 10, N = 5): the node LPs through persistent waves (k_lp_bound_refill,
    the root level and its dive leaves included) against the grid-stride kernels (k_lp_root +
    k_lp_bound, HVP_LP_REFILL=0): the same LPs by the same simplex, so the same tree -- sequences,
    statuses, LP counts -- and the same optima."""
    import torch

    from hvp import tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    n, N = 10, 5
    veh = PwaGearVehicle(800.0)
    table = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    P, R = [], []
    for seed in range(2000, 2410):
        p, r = decent_instances(O.env_initial_state(n, seed), N, leader_window(N))
        P.append(p)
        R.append(r)
    params, roles = np.concatenate(P), np.concatenate(R)
    dev = torch.device("cuda", 0)
    tp, tr = torch.from_numpy(params).to(dev), torch.from_numpy(roles).to(dev)
    ts = torch.zeros(len(roles), dtype=torch.int32, device=dev)
    s = BatchSolver(tables.problem(N, quadratic_cost=False), [table])
    a = {k: v.cpu().numpy() for k, v in s.solve_device(ts, tr, tp).items()}
    monkeypatch.setenv("HVP_LP_REFILL", "0")
    b = {k: v.cpu().numpy() for k, v in s.solve_device(ts, tr, tp).items()}
    assert (a["status"] == 0).all()
    assert np.array_equal(a["status"], b["status"])
    assert np.array_equal(a["region"], b["region"])
    assert np.all(np.abs(a["cost"] - b["cost"]) <= 1e-12 * np.maximum(1, np.abs(b["cost"])))
    assert np.abs(a["u"] - b["u"]).max() <= 1e-9
    assert np.array_equal(a["nodes"], b["nodes"])


@pytest.mark.parametrize("N,method", [(5, 1), (5, 2), (10, 2)])
def test_l1_status_infeasible_and_unresolved(gpu_available, N, method):
    """Statuses of the min_1_norm search: a leader whose position box cannot be respected is
    HVP_INFEASIBLE (every LP proven infeasible by the exact hard-row test); with the interior
    point capped at 2 iterations no LP converges and the instance is HVP_MAXITER -- never a
    sequence reported optimal over an LP that was not solved."""
    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    veh = PwaGearVehicle(800.0)
    table = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    lead = np.stack([9950 + 40 * np.arange(N + 1), np.full(N + 1, 40.0)])
    xb = O.constant_velocity_prediction(9790, 30, N)
    bad = np.concatenate([[9870.0, 30.0], np.zeros(2 * (N + 1)), xb.ravel(), lead.ravel()])
    x = O.env_initial_state(3, 7).reshape(-1).astype(float)
    good, roles = decent_instances(x, N, leader_window(N))
    params = np.concatenate([bad[None], good])
    role = np.concatenate([[tables.role_bits(True, False, True)], roles]).astype(np.int32)
    sysi = np.zeros(len(role), np.int32)
    res = BatchSolver(tables.problem(N, quadratic_cost=False, method=method), [table]).solve(sysi, role, params)
    assert res.status[0] == _abi.INFEASIBLE and (res.status[1:] == _abi.OPTIMAL).all()
    capped = tables.problem(N, quadratic_cost=False, method=method, max_iter=2)
    res = BatchSolver(capped, [table]).solve(sysi, role, params)
    assert res.status[0] == _abi.INFEASIBLE and (res.status[1:] == _abi.MAXITER).all()
