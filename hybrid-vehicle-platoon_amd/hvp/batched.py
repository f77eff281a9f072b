"""Vectorised instance builders for many platoons at once (the batched form of
``TrackingDecentMldCoordinator.observe_states``, fleet_decent_mld.py:348-455).

``decent_params_from_states`` turns S platoon states (S, 2n) into the S*n local-MPC parameter
blocks of include/hvp.h (x0, x_front, x_back, leader_x) and role flags, with the neighbour
predictions of the chosen velocity estimator.
"""

from __future__ import annotations

import numpy as np

from . import _abi
from .tables import role_bits


def extrapolate(p, v, N: int, ts: float = 1.0, dv=None, sat: bool = False) -> np.ndarray:
    """(..., 2, N+1) predictions from position p and velocity v (arrays of equal shape).

    dv None: constant velocity (fleet_decent_mld.py:421-428); dv given: two-point estimator
    adding dv per step (:430-440), or for only floor(N/2) steps when sat (:442-455).
    """
    p = np.asarray(p, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    out = np.zeros(p.shape + (2, N + 1))
    out[..., 0, 0] = p
    out[..., 1, 0] = v
    for k in range(N):
        out[..., 0, k + 1] = out[..., 0, k] + ts * out[..., 1, k]
        inc = 0.0 if dv is None or (sat and k >= N // 2) else dv
        out[..., 1, k + 1] = out[..., 1, k] + inc
    return out


def decent_params_from_states(states: np.ndarray, N: int, leader_window: np.ndarray, leader_index: int = 0,
                              real_vehicle_as_reference: bool = False, ts: float = 1.0,
                              prev_states: np.ndarray | None = None, velocity_estimator: str = "none"):
    """params (S*n, stride) float64 and roles (S*n,) int32 for S platoons of n vehicles.

    leader_window: (2, N+1) shared by all platoons, or (S, 2, N+1).
    """
    X = np.asarray(states, dtype=np.float64)
    if X.ndim == 1:
        X = X[None]
    S, n2 = X.shape
    n = n2 // 2
    pos, vel = X[:, 0::2], X[:, 1::2]
    dv = None
    sat = velocity_estimator == "sat"
    if velocity_estimator in ("two_point", "sat"):
        Xp = X if prev_states is None else np.asarray(prev_states, dtype=np.float64).reshape(S, n2)
        dv = vel - Xp[:, 1::2]
    pred = extrapolate(pos, vel, N, ts, dv, sat)  # (S, n, 2, N+1)
    stride = _abi.params_stride(N)
    K = 2 * (N + 1)
    P = np.zeros((S, n, stride))
    P[:, :, 0] = pos
    P[:, :, 1] = vel
    # front prediction of vehicle i is vehicle i-1's, back prediction is vehicle i+1's
    P[:, 1:, 2:2 + K] = pred[:, :-1].reshape(S, n - 1, K)
    P[:, :-1, 2 + K:2 + 2 * K] = pred[:, 1:].reshape(S, n - 1, K)
    lw = np.asarray(leader_window, dtype=np.float64)
    P[:, leader_index, 2 + 2 * K:] = lw.reshape(-1, K) if lw.ndim == 3 else lw.reshape(K)
    roles = np.array([role_bits(i == 0, i == n - 1, i == leader_index, real_vehicle_as_reference) for i in range(n)],
                     dtype=np.int32)
    return P.reshape(S * n, stride), np.tile(roles, S)
