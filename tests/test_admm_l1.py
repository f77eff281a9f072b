"""Naive ADMM with min_1_norm (LocalMpcADMM(quadratic_cost=False), fleet_naive_admm.py:74-77).

The local problem keeps the neighbour copies as decision variables with their quadratic ADMM terms
y'(c - z) + rho/2 |c - z|^2 (:172-198) next to L1 tracking / input terms -- a QP with epigraph
variables.  Expected values: the oracle in the full (x, u, s, copies) space (hvp_oracle.c
oracle_solve_admm_miqp, role bit 17), branch and bound, every QP KKT-certified
(tests/golden/make_golden.py admm_l1_fixtures).  Parity unpinned against Gurobi (absent).

CPU: the oracle's fixtures reproduce, and the copies it returns are the exact minimisers of their
own terms given the vehicle's trajectory (a check independent of the oracle's QP solver).
GPU (marked): the device's wave interior point with the copies as variables (csrc/hvp_lane.h
L1AdmmWave) through the C ABI, against the fixtures and the oracle coordinator.
"""

from __future__ import annotations

import os

import numpy as np
import pytest

import oracle as O
from golden_io import load

HERE = os.path.dirname(os.path.abspath(__file__))


def _system():
    from hvp import tables
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    return tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))


def _cfg(fx) -> O.Cfg:
    v = np.asarray(fx["cfg"], dtype=float)
    return O.Cfg(Qx=tuple(v[:4]), Qu=v[4], Qdu=v[5], w=v[6], a_acc=v[7], a_dec=v[8], ts=v[9], d_safe=v[10],
                 tight=v[11], d0=v[12], t0=v[13])


def _problem(N, rho, cfg: O.Cfg):
    from hvp.admm import admm_problem
    from hvp.params import ConstantSpacingPolicy, ConstantTimePolicy

    sp = ConstantTimePolicy(cfg.d0, cfg.t0) if cfg.t0 else ConstantSpacingPolicy(cfg.d0)
    return admm_problem(N, rho, sp, quadratic_cost=False)


LOCAL = ["admm_l1_local_N5.npz", "admm_l1_local_N10.npz", "admm_l1_local_ct_N5.npz"]


@pytest.mark.parametrize("name", LOCAL)
def test_oracle_reproduces_its_fixtures(name):
    """The oracle's min_1_norm ADMM local MIQPs re-solved: same statuses, regions and costs (a
    change of the checker shows up here, on the CPU, before any GPU comparison)."""
    fx = load(name)
    N, cfg = int(fx["N"]), _cfg(fx)
    sysd = O.gear_pwa_system(800.0)
    idx = range(len(fx["roles"])) if N <= 5 else range(0, len(fx["roles"]), 4)  # N = 10: the leaders (fast)
    for i in idx:
        r = O.solve_admm_miqp(sysd, cfg, N, int(fx["roles"][i]), float(fx["rho"]), fx["params"][i], quadratic=False)
        assert r.status == fx["exp_status"][i]
        assert np.array_equal(r.sigma, fx["exp_region"][i])
        assert abs(r.cost - fx["exp_cost"][i]) <= 1e-9 * max(1.0, abs(fx["exp_cost"][i]))
    assert fx["exp_cert"].all()  # every fixture answer KKT-certified


@pytest.mark.parametrize("name", LOCAL)
def test_copies_minimise_their_own_terms(name):
    """Given the vehicle's trajectory, each copy of the min_1_norm local problem minimises its own
    terms: for the front copy (p, v separable) Q_pp |p + t0 v + d0 - c_p| + w max(0, p - c_p + d_safe)
    + y_p (c_p - z_p) + rho/2 (c_p - z_p)^2 and Q_vv |v - c_v| + y_v (c_v - z_v) + rho/2 (c_v - z_v)^2
    (fleet_naive_admm.py:110-121, 172-198, 205-226) -- checked by a bounded scalar minimisation."""
    from scipy.optimize import minimize_scalar

    fx = load(name)
    N, cfg, rho = int(fx["N"]), _cfg(fx), float(fx["rho"])
    K1 = N + 1
    for i, role in enumerate(fx["roles"]):
        if not (role & O.ROLE_SAFE_FRONT) or fx["exp_status"][i] != 0:
            continue
        p = fx["params"][i]
        yf, zf = p[2:2 + 2 * K1].reshape(2, K1), p[2 + 2 * K1:2 + 4 * K1].reshape(2, K1)
        tr = bool(role & O.ROLE_TRACK_FRONT)
        for k in range(K1):
            pk, vk = fx["exp_x"][i][0, k], fx["exp_x"][i][1, k]

            def fp(c):
                return ((cfg.Qx[0] * abs(pk + cfg.t0 * vk + cfg.d0 - c) if tr else 0.0)
                        + cfg.w * max(0.0, pk - c + cfg.d_safe) + yf[0, k] * (c - zf[0, k])
                        + 0.5 * rho * (c - zf[0, k]) ** 2)

            def fv(c):
                return ((cfg.Qx[3] * abs(vk - c) if tr else 0.0) + yf[1, k] * (c - zf[1, k])
                        + 0.5 * rho * (c - zf[1, k]) ** 2)

            for f, got in ((fp, fx["exp_xf"][i][0, k]), (fv, fx["exp_xf"][i][1, k])):
                lo, hi = min(got, pk, zf[0, k], zf[1, k], vk) - 1e5, max(got, pk, zf[0, k], zf[1, k], vk) + 1e5
                best = minimize_scalar(f, bounds=(lo, hi), method="bounded", options={"xatol": 1e-11}).x
                # equal objective values (a flat stretch allows several minimisers) and a close point
                assert f(got) <= f(best) + 1e-6 * max(1.0, abs(f(best))), (name, i, k)
                assert abs(best - got) <= 1e-3 * max(1.0, abs(got)), (name, i, k)


def _check(fx, u, x, region, cost, status, xf, xb):
    ok = fx["exp_status"] == 0
    assert np.array_equal(status, fx["exp_status"])
    assert np.array_equal(region[ok], fx["exp_region"][ok])
    ce = fx["exp_cost"][ok]
    assert np.all(np.abs(cost[ok] - ce) <= 1e-9 * np.maximum(1.0, np.abs(ce))), np.abs(cost[ok] - ce).max()
    assert np.abs(u[ok] - fx["exp_u"][ok]).max() <= 1e-6
    assert np.abs(x[ok] - fx["exp_x"][ok]).max() <= 1e-4
    assert np.abs(xf[ok] - fx["exp_xf"][ok]).max() <= 1e-4
    assert np.abs(xb[ok] - fx["exp_xb"][ok]).max() <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("name", LOCAL)
def test_admm_l1_local_problem_on_gpu(gpu_available, name):
    """The device's min_1_norm ADMM local MIQPs (branch and bound over node QPs, the copies as
    variables of the wave interior point) equal the oracle's: statuses and regions exact, costs to
    1e-9 relative, u to 1e-6, x and the copies to 1e-4."""
    from hvp.solver import BatchSolver

    fx = load(name)
    N = int(fx["N"])
    s = BatchSolver(_problem(N, float(fx["rho"]), _cfg(fx)), [_system()])
    B = len(fx["roles"])
    res = s.solve_admm(np.zeros(B, np.int32), fx["roles"], fx["params"])
    _check(fx, res.u, res.x, res.region, res.cost, res.status, res.x_front, res.x_back)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["admm_l1_steps_n4_N5.npz", "admm_l1_steps_n10_N10.npz"])
def test_admm_l1_coordinator_steps_match_oracle(gpu_available, name):
    """Closed-loop time steps of the min_1_norm naive-ADMM coordinator: the device engine (batched
    local solves + hvp_admm_update, y carried across steps) reproduces the oracle coordinator's
    regions, controls and trajectories of the last ADMM iteration of every step -- 3 steps x 4
    iterations at n = 4, N = 5, and configs[2]'s size (n = 10, N = 10, 20 iterations, 2 steps)."""
    import torch

    from hvp.admm import AdmmEngine
    from instances import leader_window

    if not os.path.exists(os.path.join(HERE, "golden", name)):
        pytest.skip(f"{name} not generated (make_golden.py admm_l1 n10)")
    fx = load(name)
    n, N, iters = int(fx["n"]), int(fx["N"]), int(fx["iters"])
    roles = [O.role_bits(i, n) for i in range(n)]
    eng = AdmmEngine(_problem(N, float(fx["rho"]), O.Cfg()), [_system()], np.zeros(n, np.int32), roles, n, 1)
    for t in range(len(fx["states"])):
        eng.set_leader(leader_window(N, t))
        o = eng.step(fx["states"][t][None], iters)
        torch.cuda.synchronize()
        assert (o["status"] == 0).all()
        if fx["exp_region"].ndim == 4:  # every iteration's regions (n = 4 fixture)
            assert np.array_equal(o["region"].cpu().numpy(), fx["exp_region"][t][-1]), t
        assert np.abs(o["u"].cpu().numpy() - fx["exp_u"][t][-1]).max() <= 1e-6, t
        assert np.abs(o["x"].cpu().numpy() - fx["exp_x"][t][-1]).max() <= 1e-4, t


@pytest.mark.gpu
def test_local_mpc_admm_l1_solve_mpc_surface(gpu_available):
    """LocalMpcADMM(quadratic_cost=False).solve_mpc -- the reference's per-agent call surface
    (fleet_naive_admm.py:24-258) -- returns the oracle's first control and the copies."""
    from hvp.admm import LocalMpcADMM
    from hvp.models import PwaGearVehicle

    fx = load("admm_l1_local_N5.npz")
    N, K1 = int(fx["N"]), int(fx["N"]) + 1
    i = 5  # seed 1, vehicle 1: front and back copies
    role = int(fx["roles"][i])
    assert role & O.ROLE_SAFE_FRONT and role & O.ROLE_SAFE_BACK
    mpc = LocalMpcADMM(N, PwaGearVehicle(800).get_discrete_system(1), float(fx["rho"]), quadratic_cost=False,
                       is_front=False, is_leader=False, is_trailer=False)
    p = fx["params"][i]
    mpc.set_front_vars(p[2:2 + 2 * K1].reshape(2, K1), p[2 + 2 * K1:2 + 4 * K1].reshape(2, K1))
    mpc.set_back_vars(p[2 + 4 * K1:2 + 6 * K1].reshape(2, K1), p[2 + 6 * K1:2 + 8 * K1].reshape(2, K1))
    u0, info = mpc.solve_mpc(p[:2])
    assert abs(float(u0[0, 0]) - fx["exp_u"][i][0]) <= 1e-6
    assert abs(info["cost"] - fx["exp_cost"][i]) <= 1e-9 * abs(fx["exp_cost"][i])
    assert np.abs(mpc.x_front.X - fx["exp_xf"][i]).max() <= 1e-4
    assert np.abs(mpc.x_back.X - fx["exp_xb"][i]).max() <= 1e-4
