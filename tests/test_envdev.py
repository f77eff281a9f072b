"""The plant step (env.py PlatoonEnv.step, models.py step_platoon): the oracle restatement
against the host env (CPU), and the device step hvp_env_step_batch against the oracle (GPU):
state within 1e-9 relative (explicit Euler in float64; FMA contraction on the device), stage cost
within 1e-12 relative, violation flags and failure status identical."""

from __future__ import annotations

import numpy as np
import pytest

import oracle as O


def _platoons(P, n, seed=0):
    rng = np.random.default_rng(seed)
    X = np.stack([O.env_initial_state(n, s).astype(float) for s in range(P)])
    U = rng.uniform(-1, 1, (P, n))
    Up = rng.uniform(-1, 1, (P, n))
    M = rng.uniform(700, 1000, (P, n))
    L = np.stack([[3000.0 + 20.0 * s, 20.0] for s in range(P)])
    return X, U, Up, M, L


@pytest.mark.parametrize("quadratic", [True, False])
def test_oracle_step_matches_host_env(quadratic):
    from hvp.env import PlatoonEnv
    from hvp.models import Platoon
    from hvp.params import ConstantVelocityLeaderTrajectory

    n = 6
    pl = Platoon(n, vehicle_type="pwa_gear")
    env = PlatoonEnv(n=n, platoon=pl, ep_len=20, leader_trajectory=ConstantVelocityLeaderTrajectory(3000, 20, 70, 1),
                     quadratic_cost=quadratic)
    x, _ = env.reset(seed=5)
    rng = np.random.default_rng(1)
    prev = None
    for t in range(5):
        u = rng.uniform(-1, 1, (n, 1))
        xo, c, viol, ok = O.env_step(x, u, [800.0] * n, env.leader_x[:, t], u_prev=prev if prev is not None else u,
                                     quadratic=quadratic)
        x, r, *_ = env.step(u)
        assert ok and np.array_equal(xo, np.asarray(x, float).reshape(-1))
        assert abs(c - r) <= 1e-12 * abs(r) and viol == env.viol_counter[-1][t]
        prev = u


class _OtherWeights:
    """Controller weights that differ from PlatoonEnv's (env.py:16-18): the env must keep its own."""

    from hvp.params import Params as _P

    Q_x = np.diag([2.0, 0.5])
    Q_u = 3 * np.eye(1)
    Q_du = 0.7 * np.eye(1)
    w, a_acc, a_dec, ts, d_safe = _P.w, _P.a_acc, _P.a_dec, _P.ts, _P.d_safe


@pytest.mark.gpu
@pytest.mark.parametrize("rvar,weights,quadratic", [(False, False, True), (True, False, True), (False, True, True),
                                                    (False, False, False), (True, True, False)])
def test_device_step_matches_oracle(gpu_available, rvar, weights, quadratic):
    import torch

    from hvp import tables
    from hvp.envdev import DeviceEnv
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    P, n = 64, 10
    X, U, Up, M, L = _platoons(P, n)
    veh = PwaGearVehicle(800)
    prob = tables.problem(5, quadratic_cost=quadratic, params=_OtherWeights if weights else tables.Params)
    s = BatchSolver(prob, [tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))])
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    env = DeviceEnv(s, t(M), real_vehicle_as_reference=rvar)
    tx = t(X)
    gears = np.random.default_rng(2).integers(1, 7, (P, n)).astype(np.int8) if rvar else None
    out = env.step(tx, t(U), t(L), u_prev=t(Up), gear=None if gears is None else t(gears))
    torch.cuda.synchronize()
    xd = tx.cpu().numpy()
    for p in range(P):
        xo, c, viol, ok = O.env_step(X[p], U[p], M[p], L[p], u_prev=Up[p], gears=None if gears is None else gears[p],
                                     real_vehicle_as_reference=rvar, quadratic=quadratic)
        assert int(out["status"][p]) == (0 if ok else 1), p
        assert int(out["viol"][p]) == viol, p
        assert abs(float(out["cost"][p]) - c) <= 1e-12 * max(1.0, abs(c)), p
        if ok:
            assert np.allclose(xd[p], xo, rtol=1e-9, atol=1e-9), (p, np.abs(xd[p] - xo).max())


@pytest.mark.parametrize("estimator", ["none", "two_point", "sat"])
@pytest.mark.parametrize("N", [5, 6, 10])
def test_host_params_match_oracle_observe_states(estimator, N):
    """The product's batched observe_states (hvp.batched) against the oracle's per-vehicle
    restatement of fleet_decent_mld.py:348-455, the three velocity estimators."""
    from hvp.batched import decent_params_from_states

    P, n = 8, 6
    X, _, _, _, _ = _platoons(P, n)
    Xp = X + np.random.default_rng(5).uniform(-2, 2, X.shape)
    lead = np.stack([np.stack([3000.0 + 20.0 * (np.arange(N + 1) + p), np.full(N + 1, 20.0)]) for p in range(P)])
    for li, rvar in ((0, False), (0, True), (2, False)):
        hp, hr = decent_params_from_states(X, N, lead, leader_index=li, prev_states=Xp, velocity_estimator=estimator,
                                           real_vehicle_as_reference=rvar)
        hp, hr = hp.reshape(P, n, -1), hr.reshape(P, n)
        for p in range(P):
            op, orl = O.observe_states(X[p], Xp[p], N, lead[p], leader_index=li, real_vehicle_as_reference=rvar,
                                       velocity_estimator=estimator)
            assert np.array_equal(hr[p], orl)
            np.testing.assert_allclose(hp[p], op, rtol=1e-15, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("estimator", ["none", "two_point", "sat"])
def test_device_params_match_host(gpu_available, estimator):
    import torch

    from hvp import tables
    from hvp.batched import decent_params_from_states
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    P, n, N = 16, 10, 5
    X, _, _, _, _ = _platoons(P, n)
    Xp = X + np.random.default_rng(3).uniform(-2, 2, X.shape)
    lead = np.stack([np.stack([3000.0 + 20.0 * (np.arange(N + 1) + p), np.full(N + 1, 20.0)]) for p in range(P)])
    veh = PwaGearVehicle(800)
    s = BatchSolver(tables.problem(N), [tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    params, roles = s.decent_params_device(t(X), t(lead), x_prev=t(Xp), estimator=estimator, leader_index=2)
    hp, hr = decent_params_from_states(X, N, lead, leader_index=2, prev_states=Xp, velocity_estimator=estimator)
    assert np.array_equal(roles.cpu().numpy(), hr)
    assert np.array_equal(params.cpu().numpy(), hp)
    # and against the oracle's restatement of observe_states (fleet_decent_mld.py:348-455)
    dp, dr = params.cpu().numpy().reshape(P, n, -1), roles.cpu().numpy().reshape(P, n)
    for p in range(P):
        op, orl = O.observe_states(X[p], Xp[p], N, lead[p], leader_index=2, velocity_estimator=estimator)
        assert np.array_equal(dr[p], orl)
        np.testing.assert_allclose(dp[p], op, rtol=1e-15, atol=1e-12)


@pytest.mark.gpu
def test_device_closed_loop_matches_host_loop(gpu_available):
    """Three closed-loop steps fully on the device (params -> solve -> plant step) against the
    host coordinator + env (hvp.decent.TrackingDecentMldCoordinator, hvp.env.PlatoonEnv)."""
    import torch

    from hvp import tables
    from hvp.decent import TrackingDecentMldCoordinator
    from hvp.env import PlatoonEnv
    from hvp.envdev import DeviceEnv
    from hvp.models import Platoon
    from hvp.mpc import LocalMpcMld
    from hvp.params import ConstantVelocityLeaderTrajectory

    n, N, steps = 4, 5, 3
    lt = ConstantVelocityLeaderTrajectory(3000, 20, 60, 1)
    lx = lt.get_leader_trajectory()
    pl = Platoon(n, vehicle_type="pwa_gear")
    systems = pl.get_vehicle_system_dicts(1)
    gears = [tables.gears_of(v) for v in pl.get_vehicles()]
    mpcs = [LocalMpcMld(N, systems[i], is_front=i == 0, is_leader=i == 0, is_trailer=i == n - 1, gears=gears[i])
            for i in range(n)]
    coord = TrackingDecentMldCoordinator(mpcs, ep_len=steps, N=N, leader_x=lx, ts=1.0)
    env = PlatoonEnv(n=n, platoon=pl, ep_len=steps, leader_trajectory=lt)
    x, _ = env.reset(seed=7)
    coord.on_episode_start(env, 0, x)
    host_x, host_r = [], []
    for t in range(steps):
        u, _ = coord.get_control(x)
        x, r, *_ = env.step(u)
        coord.on_timestep_end(env, 0, t + 1)
        host_x.append(np.asarray(x, float).reshape(-1))
        host_r.append(r)
    # device loop
    s = coord._solver
    dev = torch.device("cuda", 0)
    tx = torch.from_numpy(np.asarray(env.reset(seed=7)[0], float).reshape(1, -1)).to(dev)
    denv = DeviceEnv(s, torch.full((1, n), 800.0, dtype=torch.float64, device=dev))
    sys_idx = torch.arange(n, dtype=torch.int32, device=dev)
    prev_u = None
    for t in range(steps):
        win = torch.from_numpy(np.ascontiguousarray(lx[:, t:t + N + 1])[None]).to(dev)
        params, roles = s.decent_params_device(tx, win)
        out = s.solve_device(sys_idx, roles, params)
        u = out["u"][:, 0].reshape(1, n).contiguous()
        st = denv.step(tx, u, torch.from_numpy(lx[:, t].copy()[None]).to(dev), u_prev=prev_u)
        prev_u = u
        torch.cuda.synchronize()
        assert int(st["status"][0]) == 0
        assert np.allclose(tx.cpu().numpy().reshape(-1), host_x[t], rtol=1e-9, atol=1e-8), t
        assert abs(float(st["cost"][0]) - host_r[t]) <= 1e-8 * abs(host_r[t]), t
