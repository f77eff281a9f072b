"""Test-input builders (independent of the product package: oracle restatements only)."""

from __future__ import annotations

import numpy as np

import oracle as O


def leader_window(N: int, t: int = 0, p0: float = 3000.0, v: float = 20.0) -> np.ndarray:
    """Constant-velocity leader (misc/leader_trajectory.py:17-30) window [t, t+N]."""
    k = np.arange(t, t + N + 1)
    return np.stack([p0 + v * k, np.full(N + 1, v)])


def decent_instances(state: np.ndarray, N: int, lead: np.ndarray, leader_index: int = 0,
                     real_vehicle_as_reference: bool = False):
    """(params, roles) of the n local MPCs of fleet_decent_mld.py for one platoon state,
    with constant-velocity neighbour predictions (fleet_decent_mld.py:348-428)."""
    x = np.asarray(state, dtype=float).reshape(-1)
    n = len(x) // 2
    P, R = [], []
    zero = np.zeros((2, N + 1))
    for i in range(n):
        xf = O.constant_velocity_prediction(x[2 * i - 2], x[2 * i - 1], N) if i > 0 else zero
        xb = O.constant_velocity_prediction(x[2 * i + 2], x[2 * i + 3], N) if i < n - 1 else zero
        xl = lead if i == leader_index else zero
        P.append(np.concatenate([x[2 * i:2 * i + 2], xf.ravel(), xb.ravel(), xl.ravel()]))
        R.append(O.role_bits(i, n, leader_index, real_vehicle_as_reference))
    return np.array(P), np.array(R, dtype=np.int32)


def split_params(p: np.ndarray, N: int):
    K = 2 * (N + 1)
    return p[:2], p[2:2 + K].reshape(2, N + 1), p[2 + K:2 + 2 * K].reshape(2, N + 1), p[2 + 2 * K:].reshape(2, N + 1)


def oracle_solve(sysd, cfg, N, params, roles, quadratic=True):
    out = []
    for p, r in zip(params, roles):
        x0, xf, xb, xl = split_params(p, N)
        out.append(O.solve_miqp(sysd, cfg, N, int(r), x0, xf, xb, xl, quadratic=quadratic))
    return out
