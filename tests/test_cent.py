"""Centralised MLD (mpcs/cent_mld.py MpcMldCent, fleet_cent_mld.py): one MIQP per platoon.

CPU: the oracle's joint branch and bound equals its exhaustive joint enumeration; the oracle
reproduces the committed fixtures; the host-side API raises like the reference.
GPU (through hvp_cent_solve_batch): the committed fixtures -- region sequences and gears
bit-exact, cost within 1e-9 relative, u within 1e-6, x within 1e-4 (positions ~3e3), QP counts
equal to the oracle's (same exploration order; min_1_norm: not compared, exact LP bound ties make
the order noise-driven); exhaustive mode = branch and bound; at the configs[1] size (n = 10,
N = 5) determinism, the PWA dynamics of the chosen regions, and the drop-in MpcMldCent /
simulate surface, for both costs (cent_l1_*.npz: the min_1_norm MILP, cent_mld.py:58-61).
"""

from __future__ import annotations

import glob
import os

import numpy as np
import pytest

import oracle as O
from golden_io import GOLDEN, CfgParams, load
from instances import leader_window

CENT = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "cent_*.npz")))
FAST = [c for c in CENT if c.startswith(("cent_n2_", "cent_n4_", "cent_lsp", "cent_lead2", "cent_qdu", "cent_n10_N3",
                                         "cent_l1_n3_N5", "cent_l1_lead1", "cent_l1_gear", "cent_l1_qdu"))]


def _quadratic(fx) -> bool:
    """Fixtures of the min_1_norm controller carry quadratic = 0 (older files: the MIQP)."""
    return bool(int(fx["quadratic"])) if "quadratic" in fx else True


def _cfg(v) -> O.Cfg:
    v = np.asarray(v, dtype=float)
    return O.Cfg(Qx=tuple(v[0:4]), Qu=v[4], Qdu=v[5], w=v[6], a_acc=v[7], a_dec=v[8], ts=v[9], d_safe=v[10],
                 tight=v[11], d0=v[12], t0=v[13])


def _oracle_systems(fx, p):
    mk = O.gear_friction_mld_system if int(fx["model"]) == 1 else O.gear_pwa_system
    return [mk(float(m)) for m in fx["masses"][p]]


# ------------------------------------------------------------------ CPU: the oracle
@pytest.mark.parametrize("n,N,seed", [(2, 3, 0), (2, 4, 1), (3, 3, 2), (2, 5, 3)])
def test_oracle_bnb_equals_exhaustive(n, N, seed):
    systems = [O.gear_pwa_system(800.0)] * n
    x0 = O.env_initial_state(n, seed).astype(float)
    a = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N))
    b = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N), exhaustive=True)
    assert a.status == b.status == 0
    assert np.array_equal(a.sigma, b.sigma)
    assert abs(a.cost - b.cost) <= 1e-9 * abs(b.cost)
    assert a.n_qps <= b.n_qps


@pytest.mark.parametrize("n,N,seed,model", [(2, 3, 0, 0), (2, 4, 1, 0), (3, 3, 2, 0), (2, 3, 3, 1)])
def test_oracle_l1_bnb_equals_exhaustive(n, N, seed, model):
    """min_1_norm (cent_mld.py:58-61, a MILP): the joint branch and bound over LP relaxations
    equals the exhaustive joint enumeration of fixed-sequence LPs."""
    mk = O.gear_friction_mld_system if model else O.gear_pwa_system
    systems = [mk(800.0)] * n
    x0 = O.env_initial_state(n, seed).astype(float)
    a = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N), quadratic=False)
    b = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N), exhaustive=True, quadratic=False)
    assert a.status == b.status == 0
    assert np.array_equal(a.sigma, b.sigma)
    assert abs(a.cost - b.cost) <= 1e-9 * abs(b.cost)
    assert a.n_qps <= b.n_qps
    q = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N))
    assert q.status == 0 and abs(q.cost - a.cost) > 1e-6 * abs(a.cost)  # a different objective


@pytest.mark.parametrize("n,N,seed", [(2, 3, 0), (2, 4, 1), (3, 3, 2)])
def test_oracle_bnb_equals_exhaustive_gear_friction(n, N, seed):
    """The gear-friction model (MpcGearCent: b differs per gear inside a friction region, so the
    virtual-region relaxation is active): branch and bound = exhaustive joint enumeration."""
    systems = [O.gear_friction_mld_system(800.0)] * n
    x0 = O.env_initial_state(n, seed).astype(float)
    a = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N))
    b = O.solve_cent(systems, O.Cfg(), N, x0, leader_window(N), exhaustive=True)
    assert a.status == b.status == 0
    assert np.array_equal(a.sigma, b.sigma)
    assert abs(a.cost - b.cost) <= 1e-9 * abs(b.cost)
    assert a.n_qps <= b.n_qps


@pytest.mark.parametrize("name", ["cent_gear_n3_N4.npz", "cent_qdu_n4_N5.npz"])
def test_tail_relaxation_changes_only_the_search(name):
    """The tail relaxation (reachable intervals + virtual regions) against the
    plain relaxation (undecided steps without dynamics or input terms) on the gear-friction and
    Q_du fixtures: the same regions and cost, and never more QPs."""
    fx = load(name)
    N = int(fx["N"])
    cfg = _cfg(fx["cfg"])
    for p in range(len(fx["x0"])):
        args = (_oracle_systems(fx, p), cfg, N, fx["x0"][p].reshape(-1), fx["leader_x"][p], int(fx["leader_index"][p]),
                bool(fx["lsp"][p]))
        on = O.solve_cent(*args)
        O.set_cent_relax(False)
        try:
            off = O.solve_cent(*args)
        finally:
            O.set_cent_relax(True)
        assert on.status == off.status
        if on.status == 0:
            assert np.array_equal(on.sigma, off.sigma), p
            assert abs(on.cost - off.cost) <= 1e-9 * max(1.0, abs(off.cost)), p
            assert on.n_qps <= off.n_qps, (p, on.n_qps, off.n_qps)


@pytest.mark.parametrize("name", FAST)
def test_oracle_reproduces_cent_golden(name):
    fx = load(name)
    N = int(fx["N"])
    cfg = _cfg(fx["cfg"])
    for p in range(len(fx["x0"])):
        r = O.solve_cent(_oracle_systems(fx, p), cfg, N, fx["x0"][p].reshape(-1), fx["leader_x"][p],
                         int(fx["leader_index"][p]), bool(fx["lsp"][p]), quadratic=_quadratic(fx))
        assert r.status == fx["exp_status"][p]
        assert np.array_equal(r.sigma, fx["exp_region"][p])
        assert abs(r.cost - fx["exp_cost"][p]) <= 1e-10 * abs(fx["exp_cost"][p])
        assert r.n_qps == fx["exp_nodes"][p]


def test_cent_beats_decentralised_plan_cost():
    """Sanity of the formulation: the centralised optimum is no worse than the platoon cost of
    every vehicle holding its constant-velocity trajectory (a feasible point of the MIQP)."""
    n, N = 4, 5
    x0 = O.env_initial_state(n, 0).astype(float)
    r = O.solve_cent([O.gear_pwa_system(800.0)] * n, O.Cfg(), N, x0, leader_window(N))
    assert r.status == 0 and np.isfinite(r.cost)
    # the predicted trajectory obeys the first-state constraint and the horizon shape
    assert np.allclose(r.x[:, :, 0], x0.reshape(n, 2))
    assert r.u.shape == (n, N) and r.sigma.shape == (n, N)


def test_api_raises_like_the_reference():
    """mpcs/cent_mld.py:63-66 (checked before any device handle exists) and the problem block."""
    from hvp.cent import MpcMldCent, cent_problem
    from hvp.models import Platoon

    systems = Platoon(3, vehicle_type="pwa_gear").get_vehicle_system_dicts(1)
    with pytest.raises(NotImplementedError):
        MpcMldCent(3, 5, systems, leader_index=1, real_vehicle_as_reference=True)
    with pytest.raises(ValueError):
        MpcMldCent(4, 5, systems)
    p = cent_problem(5)
    assert int(p.formulation) == 3 and int(p.method) == 2
    assert int(cent_problem(5, exhaustive=True).method) == 1
    assert int(cent_problem(5, quadratic_cost=False).quadratic_cost) == 0


# ------------------------------------------------------------------ GPU
def _product(fx):
    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.models import PwaFrictionVehicle, PwaGearVehicle
    from hvp.params import ConstantTimePolicy

    cp = CfgParams(fx["cfg"])
    prob = cent_problem(int(fx["N"]), ConstantTimePolicy(cp.d0, cp.t0), quadratic_cost=_quadratic(fx),
                        accel_cnstr_tightening=cp.tight, params=cp)
    masses = np.unique(fx["masses"].reshape(-1))
    systems = []
    for m in masses:
        if int(fx["model"]) == 1:
            systems.append(tables.gear_system_from_dict(PwaFrictionVehicle(float(m)).get_discrete_system(float(cp.ts))))
        else:
            veh = PwaGearVehicle(float(m))
            systems.append(tables.system_from_dict(veh.get_discrete_system(float(cp.ts)), tables.gears_of(veh)))
    sys_idx = np.searchsorted(masses, fx["masses"]).astype(np.int32)
    s = CentSolver(prob, systems)
    s.tables = systems
    return s, sys_idx


def _l1_objective(fx, p, x, u) -> float:
    """min_1_norm objective of a platoon trajectory (numpy restatement of cent_mld.py:83-140 with
    the L1 norms, as hvp_oracle.c cent_objective prices a leaf): x (n, 2, N+1), u (n, N)."""
    c = _cfg(fx["cfg"])
    N = int(fx["N"])
    L, lsp, xl = int(fx["leader_index"][p]), bool(fx["lsp"][p]), fx["leader_x"][p]
    n = x.shape[0]
    J = 0.0
    for k in range(N + 1):
        for i in range(n):
            pp, v = x[i, 0, k], x[i, 1, k]
            if i == L:
                J += abs(c.Qx[0] * (pp - xl[0, k] + (c.t0 * v + c.d0 if lsp else 0.0))) + abs(c.Qx[3] * (v - xl[1, k]))
            if i >= 1:
                pm, vm = x[i - 1, 0, k], x[i - 1, 1, k]
                J += abs(c.Qx[0] * (pp + c.t0 * v + c.d0 - pm)) + abs(c.Qx[3] * (v - vm))
                J += c.w * max(0.0, pp - pm + c.d_safe)
            elif lsp and L == 0:
                J += c.w * max(0.0, pp - xl[0, k] + c.d_safe)
    J += np.abs(c.Qu * u).sum() + np.abs(c.Qdu * np.diff(u, axis=1)).sum()
    return J


def _check_alternative_optimum(fx, p, s, sys_idx, res, j, name):
    """A min_1_norm LP may have a face of optima (the oracle's interior point and the device's stop
    at different points of it): the device's (x, u) must then follow the PWA dynamics of the
    returned regions inside the boxes and price at the oracle's optimal cost."""
    N = int(fx["N"])
    for i in range(res.u.shape[1]):
        st = s.tables[int(sys_idx[p, i])]
        for k in range(N):
            r = int(res.region[j, i, k])
            v, vn = res.x[j, i, 1, k], res.x[j, i, 1, k + 1]
            assert st.vlo[r] - 1e-6 <= v <= st.vhi[r] + 1e-6, (name, p, i, k)
            assert abs(vn - (st.a[r] * v + st.b[r] * res.u[j, i, k] + st.c[r])) <= 1e-8, (name, p, i, k)
            assert abs(res.x[j, i, 0, k + 1] - (res.x[j, i, 0, k] + st.ts * v)) <= 1e-8, (name, p, i, k)
            assert st.umin - 1e-7 <= res.u[j, i, k] <= st.umax + 1e-7, (name, p, i, k)
    J = _l1_objective(fx, p, res.x[j], res.u[j])
    assert abs(J - fx["exp_cost"][p]) <= 1e-9 * abs(fx["exp_cost"][p]), (name, p, J, fx["exp_cost"][p])


@pytest.mark.gpu
@pytest.mark.parametrize("name", CENT)
def test_gpu_matches_cent_golden(gpu_available, name):
    fx = load(name)
    s, sys_idx = _product(fx)
    P = len(fx["x0"])
    for lead_idx, lsp in sorted({(int(a), int(b)) for a, b in zip(fx["leader_index"], fx["lsp"])}):
        sel = np.flatnonzero((fx["leader_index"] == lead_idx) & (fx["lsp"] == lsp))
        res = s.solve(sys_idx[sel], fx["x0"][sel], fx["leader_x"][sel], lead_idx, bool(lsp))
        for j, p in enumerate(sel):
            assert res.status[j] == fx["exp_status"][p], (name, p, res.status[j])
            if fx["exp_status"][p] != 0:
                continue
            assert np.array_equal(res.region[j], fx["exp_region"][p]), (name, p, res.region[j], fx["exp_region"][p],
                                                                        res.cost[j], fx["exp_cost"][p])
            assert np.array_equal(res.gear[j], fx["exp_gear"][p]), (name, p)
            assert abs(res.cost[j] - fx["exp_cost"][p]) <= 1e-9 * abs(fx["exp_cost"][p]), (name, p)
            if _quadratic(fx) or np.abs(res.u[j] - fx["exp_u"][p]).max() <= 1e-6:
                assert np.abs(res.u[j] - fx["exp_u"][p]).max() <= 1e-6, (name, p)
                assert np.abs(res.x[j] - fx["exp_x"][p]).max() <= 1e-4, (name, p)
            else:
                _check_alternative_optimum(fx, p, s, sys_idx, res, j, name)
            if _quadratic(fx):  # LP bounds tie exactly between sibling regions: the visiting order
                # (and so the LP count) of the min_1_norm search follows 1e-12 noise on both sides
                assert res.nodes[j] == fx["exp_nodes"][p], (name, p, res.nodes[j], fx["exp_nodes"][p])
    assert P == len(fx["exp_status"])


@pytest.mark.gpu
@pytest.mark.parametrize("name,split", [("cent_n6_N5.npz", 40), ("cent_n8_N5.npz", 25), ("cent_n3_N10.npz", 30),
                                        ("cent_gear_n3_N4.npz", 10), ("cent_task2_n5_N5.npz", 20),
                                        ("cent_l1_n3_N8.npz", 20), ("cent_l1_n4_N5.npz", 15)])
def test_gpu_split_search_matches_cent_golden(gpu_available, monkeypatch, name, split):
    """The split search (heavy platoons: open DFS frames exported as subtree tasks run by every
    wave, shared incumbent, tie rule over the merged leaves) forced on the fixtures by a tiny
    split budget: the same regions, gears, cost and trajectories as the oracle's sequential
    search (the QP counts differ: the order of exploration does)."""
    monkeypatch.setenv("HVP_CENT_SPLIT", str(split))
    monkeypatch.setenv("HVP_CENT_TASK_BUDGET", "32")
    fx = load(name)
    s, sys_idx = _product(fx)
    for lead_idx, lsp in sorted({(int(a), int(b)) for a, b in zip(fx["leader_index"], fx["lsp"])}):
        sel = np.flatnonzero((fx["leader_index"] == lead_idx) & (fx["lsp"] == lsp))
        res = s.solve(sys_idx[sel], fx["x0"][sel], fx["leader_x"][sel], lead_idx, bool(lsp))
        for j, p in enumerate(sel):
            assert res.status[j] == fx["exp_status"][p], (name, p, res.status[j])
            if fx["exp_status"][p] != 0:
                continue
            assert np.array_equal(res.region[j], fx["exp_region"][p]), (name, p, res.region[j], fx["exp_region"][p])
            assert np.array_equal(res.gear[j], fx["exp_gear"][p]), (name, p)
            assert abs(res.cost[j] - fx["exp_cost"][p]) <= 1e-9 * abs(fx["exp_cost"][p]), (name, p)
            if _quadratic(fx) or np.abs(res.u[j] - fx["exp_u"][p]).max() <= 1e-6:
                assert np.abs(res.u[j] - fx["exp_u"][p]).max() <= 1e-6, (name, p)
                assert np.abs(res.x[j] - fx["exp_x"][p]).max() <= 1e-4, (name, p)
            else:
                _check_alternative_optimum(fx, p, s, sys_idx, res, j, name)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cent_n6_N5.npz", "cent_n4_N5.npz"])
def test_gpu_small_task_budget_no_overflow(gpu_available, monkeypatch, name):
    """A tiny task budget (HVP_CENT_TASK_BUDGET=16, split past 10 QPs) makes many short tasks;
    merge() keeps only leaves inside the shared incumbent's tie window, so the platoon's tie list
    does not fill up (no HVP_OVERFLOW) and the answer is the oracle's."""
    from hvp import _abi

    monkeypatch.setenv("HVP_CENT_SPLIT", "10")
    monkeypatch.setenv("HVP_CENT_TASK_BUDGET", "16")
    fx = load(name)
    s, sys_idx = _product(fx)
    for lead_idx, lsp in sorted({(int(a), int(b)) for a, b in zip(fx["leader_index"], fx["lsp"])}):
        sel = np.flatnonzero((fx["leader_index"] == lead_idx) & (fx["lsp"] == lsp))
        res = s.solve(sys_idx[sel], fx["x0"][sel], fx["leader_x"][sel], lead_idx, bool(lsp))
        assert not (res.status == _abi.OVERFLOW).any(), res.status
        for j, p in enumerate(sel):
            assert res.status[j] == fx["exp_status"][p], (name, p, res.status[j])
            if fx["exp_status"][p] == 0:
                assert np.array_equal(res.region[j], fx["exp_region"][p]), (name, p)
                assert abs(res.cost[j] - fx["exp_cost"][p]) <= 1e-9 * abs(fx["exp_cost"][p]), (name, p)


@pytest.mark.gpu
def test_gpu_exhaustive_equals_bnb(gpu_available):
    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    sysd = [tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))]
    n, N = 2, 4
    x0 = np.stack([O.env_initial_state(n, s).astype(float).reshape(n, 2) for s in range(6)])
    sys_idx = np.zeros((6, n), np.int32)
    a = CentSolver(cent_problem(N), sysd).solve(sys_idx, x0, leader_window(N))
    b = CentSolver(cent_problem(N, exhaustive=True), sysd).solve(sys_idx, x0, leader_window(N))
    assert (a.status == 0).all() and (b.status == 0).all()
    assert np.array_equal(a.region, b.region)
    assert np.allclose(a.cost, b.cost, rtol=1e-9, atol=0)
    assert (a.nodes <= b.nodes).all()


@pytest.mark.gpu
def test_gpu_early_stop_keeps_the_search(gpu_available, monkeypatch):
    """The dual-bound early stop (hvp_cent.h solve, GI_CUT) only ends QPs the search prunes anyway:
    with and without it (HVP_CENT_CUT=0) the same regions, costs, trajectories and QP counts at
    configs[1]'s platoon size (n = 10, N = 5), and fewer active-set iterations with it."""
    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    st = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    n, N, P = 10, 5, 24
    x0 = np.stack([O.env_initial_state(n, 300 + p).astype(float).reshape(n, 2) for p in range(P)])
    a = CentSolver(cent_problem(N), [st]).solve(np.zeros((P, n), np.int32), x0, leader_window(N))
    monkeypatch.setenv("HVP_CENT_CUT", "0")
    b = CentSolver(cent_problem(N), [st]).solve(np.zeros((P, n), np.int32), x0, leader_window(N))
    assert (a.status == 0).all() and (b.status == 0).all(), (a.status, b.status)
    for k in ("region", "gear"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    # a search past 1000 QPs splits into tasks sharing one incumbent: its QP count follows their timing
    seq = (a.nodes <= 1000) & (b.nodes <= 1000)
    assert seq.sum() >= P // 2 and np.array_equal(a.nodes[seq], b.nodes[seq])
    assert np.allclose(a.cost, b.cost, rtol=1e-12, atol=0)
    assert np.abs(a.u - b.u).max() <= 1e-9 and np.abs(a.x - b.x).max() <= 1e-9
    assert a.iters.sum() < b.iters.sum(), (a.iters.sum(), b.iters.sum())


@pytest.mark.gpu
def test_gpu_c2_size_properties(gpu_available):
    """configs[1] platoon size (n = 10, N = 5): every platoon optimal, deterministic, and the
    returned trajectory follows the PWA dynamics of the returned regions inside the boxes."""
    import torch

    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    st = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    n, N, P = 10, 5, 8
    s = CentSolver(cent_problem(N), [st])
    x0 = np.stack([O.env_initial_state(n, 100 + p).astype(float).reshape(n, 2) for p in range(P)])
    a = s.solve(np.zeros((P, n), np.int32), x0, leader_window(N))
    b = s.solve(np.zeros((P, n), np.int32), x0, leader_window(N))
    assert (a.status == 0).all(), a.status
    for k in ("region", "u", "x", "cost", "nodes"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    for p in range(P):
        for i in range(n):
            for k in range(N):
                r = int(a.region[p, i, k])
                v, vn = a.x[p, i, 1, k], a.x[p, i, 1, k + 1]
                assert st.vlo[r] - 1e-6 <= v <= st.vhi[r] + 1e-6
                assert abs(vn - (st.a[r] * v + st.b[r] * a.u[p, i, k] + st.c[r])) <= 1e-8
                assert abs(a.x[p, i, 0, k + 1] - (a.x[p, i, 0, k] + st.ts * v)) <= 1e-8
                assert st.umin - 1e-7 <= a.u[p, i, k] <= st.umax + 1e-7
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_mpc_cent_drop_in_and_simulate(gpu_available):
    from hvp.cent import MpcMldCent, TrackingCentralizedAgent, simulate
    from hvp.models import Platoon
    from hvp.params import Sim

    n, N = 3, 4
    platoon = Platoon(n, vehicle_type="pwa_gear")
    mpc = MpcMldCent(n, N, platoon.get_vehicle_system_dicts(1))
    mpc.set_leader_traj(leader_window(N))
    state = O.env_initial_state(n, 0).astype(float).reshape(2 * n, 1)
    u, info = mpc.solve_mpc(state)
    assert u.shape == (n, 1) and info["x"].shape == (2 * n, N + 1) and info["u"].shape == (n, N)
    assert info["bin_vars"] == 7 * n * N and info["nodes"] > 0 and np.isfinite(info["cost"])
    r = O.solve_cent([O.gear_pwa_system(800.0)] * n, O.Cfg(), N, state.reshape(-1), leader_window(N))
    assert abs(info["cost"] - r.cost) <= 1e-9 * abs(r.cost)

    class Short(Sim):
        n, N, ep_len = 3, 4, 6
        id = "test_cent"

    sim = Short()
    X, U, R, agent, env = simulate(sim, seed=1)
    assert isinstance(agent, TrackingCentralizedAgent)
    assert X.shape[0] == sim.ep_len + 1 and U.shape[0] == sim.ep_len
    assert np.all(agent.node_counts > 0)


@pytest.mark.gpu
def test_gpu_mpc_cent_l1_drop_in_and_simulate(gpu_available):
    """MpcMldCent(quadratic_cost=False) (cent_mld.py:58-61): the min_1_norm MILP of one platoon
    equals the oracle's, and the fleet_cent_mld.py loop runs on it."""
    from hvp.cent import MpcMldCent, simulate
    from hvp.models import Platoon
    from hvp.params import Sim

    n, N = 3, 5
    platoon = Platoon(n, vehicle_type="pwa_gear")
    mpc = MpcMldCent(n, N, platoon.get_vehicle_system_dicts(1), quadratic_cost=False)
    mpc.set_leader_traj(leader_window(N))
    for seed in range(3):
        state = O.env_initial_state(n, seed).astype(float).reshape(2 * n, 1)
        u, info = mpc.solve_mpc(state)
        r = O.solve_cent([O.gear_pwa_system(800.0)] * n, O.Cfg(), N, state.reshape(-1), leader_window(N),
                         quadratic=False)
        assert r.status == 0 and info["status"] == 0
        assert np.array_equal(mpc.regions_pred, r.sigma), seed
        assert abs(info["cost"] - r.cost) <= 1e-9 * abs(r.cost)
        assert np.abs(info["u"] - r.u).max() <= 1e-6
        assert np.abs(info["x"] - r.x.reshape(2 * n, N + 1)).max() <= 1e-4

    class Short(Sim):
        n, N, ep_len = 3, 4, 6
        quadratic_cost = False
        id = "test_cent_l1"

    sim = Short()
    X, U, R, agent, env = simulate(sim, seed=2)
    assert X.shape[0] == sim.ep_len + 1 and U.shape[0] == sim.ep_len
    assert np.all(agent.node_counts > 0) and np.all(np.isfinite(R))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["cent_n6_N5.npz", "cent_n8_N5.npz", "cent_l1_n4_N5.npz"])
def test_gpu_full_task_list_declines_the_split(gpu_available, monkeypatch, name):
    """the split-task list used to overflow (HVP_OVERFLOW) when heavy searches exported
    more open frames than it holds.  Exports now reserve their slots at once or not at all: with a
    4-task list and a split every 10 QPs most exports are declined and those searches go on in their
    own wave -- no HVP_OVERFLOW, the oracle's answers."""
    from hvp import _abi

    monkeypatch.setenv("HVP_CENT_SPLIT", "10")
    monkeypatch.setenv("HVP_CENT_TASK_BUDGET", "16")
    monkeypatch.setenv("HVP_CENT_TASK_CAP", "4")
    fx = load(name)
    s, sys_idx = _product(fx)
    for lead_idx, lsp in sorted({(int(a), int(b)) for a, b in zip(fx["leader_index"], fx["lsp"])}):
        sel = np.flatnonzero((fx["leader_index"] == lead_idx) & (fx["lsp"] == lsp))
        res = s.solve(sys_idx[sel], fx["x0"][sel], fx["leader_x"][sel], lead_idx, bool(lsp))
        assert not (res.status == _abi.OVERFLOW).any(), res.status
        for j, p in enumerate(sel):
            assert res.status[j] == fx["exp_status"][p], (name, p, res.status[j])
            if fx["exp_status"][p] == 0:
                assert np.array_equal(res.region[j], fx["exp_region"][p]), (name, p)
                assert abs(res.cost[j] - fx["exp_cost"][p]) <= 1e-9 * abs(fx["exp_cost"][p]), (name, p)
