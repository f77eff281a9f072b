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


def test_oracle_step_matches_host_env():
    from hvp.env import PlatoonEnv
    from hvp.models import Platoon
    from hvp.params import ConstantVelocityLeaderTrajectory

    n = 6
    pl = Platoon(n, vehicle_type="pwa_gear")
    env = PlatoonEnv(n=n, platoon=pl, ep_len=20, leader_trajectory=ConstantVelocityLeaderTrajectory(3000, 20, 70, 1))
    x, _ = env.reset(seed=5)
    rng = np.random.default_rng(1)
    prev = None
    for t in range(5):
        u = rng.uniform(-1, 1, (n, 1))
        xo, c, viol, ok = O.env_step(x, u, [800.0] * n, env.leader_x[:, t], u_prev=prev if prev is not None else u)
        x, r, *_ = env.step(u)
        assert ok and np.array_equal(xo, np.asarray(x, float).reshape(-1))
        assert abs(c - r) <= 1e-12 * abs(r) and viol == env.viol_counter[-1][t]
        prev = u


@pytest.mark.gpu
@pytest.mark.parametrize("rvar", [False, True])
def test_device_step_matches_oracle(gpu_available, rvar):
    import torch

    from hvp import tables
    from hvp.envdev import DeviceEnv
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    P, n = 64, 10
    X, U, Up, M, L = _platoons(P, n)
    veh = PwaGearVehicle(800)
    s = BatchSolver(tables.problem(5), [tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))])
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
                                     real_vehicle_as_reference=rvar)
        assert int(out["status"][p]) == (0 if ok else 1), p
        assert int(out["viol"][p]) == viol, p
        assert abs(float(out["cost"][p]) - c) <= 1e-12 * max(1.0, abs(c)), p
        if ok:
            assert np.allclose(xd[p], xo, rtol=1e-9, atol=1e-9), (p, np.abs(xd[p] - xo).max())
