"""Controller constants, simulation configs, spacing policies and leader trajectories.

Restates ``misc/common_controller_params.py:14-76``, ``misc/spacing_policy.py:14-37`` and
``misc/leader_trajectory.py:17-97`` of the reference.  These are the constants that enter
every local QP (weights, limits, spacing, the leader window).
"""

from __future__ import annotations

from typing import Literal

import numpy as np


# ---------------------------------------------------------------- spacing policies
class SpacingPolicy:
    """Desired inter-vehicle offset spacing(x) (misc/spacing_policy.py:4-11)."""

    #: spacing(x) = A_sp @ x + b_sp ; the solver uses (d0, t0) with
    #: A_sp = [[0, -t0], [0, 0]], b_sp = [-d0, 0]
    d0: float = 0.0
    t0: float = 0.0

    def spacing(self, x: np.ndarray) -> np.ndarray:
        x = np.asarray(x, dtype=float).reshape(2, 1)
        return np.array([[-self.d0 - self.t0 * x[1, 0]], [0.0]])


class ConstantSpacingPolicy(SpacingPolicy):
    """spacing = [-d0, 0] (misc/spacing_policy.py:14-22)."""

    def __init__(self, d0: float) -> None:
        self.d0 = float(d0)
        self.t0 = 0.0
        self.d = np.array([[-self.d0], [0.0]])

    def spacing(self, x: np.ndarray) -> np.ndarray:
        return self.d


class ConstantTimePolicy(SpacingPolicy):
    """spacing = [[0, -t0], [0, 0]] x + [-d0, 0] (misc/spacing_policy.py:25-37)."""

    def __init__(self, d0: float, t0: float) -> None:
        self.d0 = float(d0)
        self.t0 = float(t0)
        self.A = np.array([[0.0, -self.t0], [0.0, 0.0]])
        self.b = np.array([[-self.d0], [0.0]])


# ---------------------------------------------------------------- leader trajectories
class LeaderTrajectory:
    def __init__(self, trajectory_len: int, ts: float) -> None:
        self.trajectory_len = trajectory_len
        self.ts = ts

    def get_leader_trajectory(self) -> np.ndarray:
        raise NotImplementedError


class ConstantVelocityLeaderTrajectory(LeaderTrajectory):
    """(misc/leader_trajectory.py:17-30)."""

    def __init__(self, p: float, v: float, trajectory_len: int, ts: float) -> None:
        super().__init__(trajectory_len, ts)
        self.p0, self.v = p, v

    def get_leader_trajectory(self) -> np.ndarray:
        L = self.trajectory_len
        x = np.zeros((2, L))
        x[1, :] = self.v
        x[0, 0] = self.p0
        # sequential accumulation keeps the reference loop's rounding bit for bit
        for k in range(L - 1):
            x[0, k + 1] = x[0, k] + self.ts * self.v
        return x


class StopAndGoLeaderTrajectory(LeaderTrajectory):
    """Slow to vl for steps in [c0, c1), then vf (or vh) (misc/leader_trajectory.py:33-69)."""

    def __init__(self, p, vh, vl, v_change_steps, trajectory_len, ts, vf=None) -> None:
        super().__init__(trajectory_len, ts)
        if len(v_change_steps) != 2:
            raise ValueError(f"v_change_steps should have 2 items, received {len(v_change_steps)}")
        self.p0, self.vh, self.vl, self.vf = p, vh, vl, vf
        self.v_change_steps = v_change_steps

    def get_leader_trajectory(self) -> np.ndarray:
        L = self.trajectory_len
        c0, c1 = self.v_change_steps
        v_after = self.vh if self.vf is None else self.vf
        x = np.zeros((2, L))
        x[:, 0] = (self.p0, self.vh)
        v = self.vh
        for k in range(L - 1):
            x[0, k + 1] = x[0, k] + self.ts * v  # position uses the speed held during step k
            if c0 <= k < c1:
                v = self.vl
            elif k >= c1:
                v = v_after
            x[1, k + 1] = v if k >= c0 else x[1, k]
        return x


class VolatileTrajectory(LeaderTrajectory):
    """Piecewise human-like speed profile (misc/leader_trajectory.py:72-97)."""

    def __init__(self, p: float, trajectory_len: int, ts: float) -> None:
        super().__init__(trajectory_len, ts)
        self.p0 = p

    def get_leader_trajectory(self) -> np.ndarray:
        L = self.trajectory_len
        speeds = np.empty(L - 1)
        speeds[:20] = 30
        speeds[20:30] = 20
        speeds[30:50] = 20 + np.arange(1, 21)
        speeds[50:70] = 10
        speeds[70:] = 20
        x = np.zeros((2, L))
        x[:, 0] = (self.p0, 30)
        for k in range(L - 1):
            x[0, k + 1] = x[0, k] + self.ts * speeds[k]
            x[1, k + 1] = speeds[k]
        return x


# ---------------------------------------------------------------- parameters
class Params:
    """Weights and limits of every local MPC (common_controller_params.py:14-23)."""

    Q_x = np.diag([1.0, 0.1])
    Q_u = 1 * np.eye(1)
    q_du = 0
    Q_du = q_du * np.eye(1)
    w = 1e4
    ts = 1
    a_acc = 2.5
    a_dec = -2
    d_safe = 25


class Sim:
    """Default simulation config (common_controller_params.py:26-40)."""

    open_loop = False
    real_vehicle_as_reference = False
    vehicle_model_type: Literal["nonlinear", "pwa_friction", "pwa_gear"] = "pwa_gear"
    start_from_platoon: bool = False
    quadratic_cost: bool = True
    n = 3
    N = 6
    ep_len = N if open_loop else 150
    spacing_policy = ConstantSpacingPolicy(50)
    leader_trajectory = ConstantVelocityLeaderTrajectory(p=3000, v=20, trajectory_len=ep_len + 50, ts=Params.ts)
    masses = None
    id = f"default_n_{n}_N_{N}"


class Sim_n_task_1(Sim):
    def __init__(self, n: int) -> None:
        self.n = n
        self.id = f"task_1_n_{n}_N_{self.N}"
        self.spacing_policy = ConstantSpacingPolicy(50)
        self.leader_trajectory = ConstantVelocityLeaderTrajectory(
            p=3100, v=20, trajectory_len=self.ep_len + 50, ts=Params.ts
        )


class Sim_n_task_2(Sim):
    def __init__(self, n: int, seed: int, leader_index: int | None = None, N: int = 6) -> None:
        self.n, self.N = n, N
        self.id = f"task_2_n_{n}_N_{N}" + ("" if Params.q_du == 0 else f"_q_{Params.q_du}")
        if leader_index is not None:
            self.id += f"_lead_{leader_index}"
        self.spacing_policy = ConstantTimePolicy(10, 3)
        self.leader_trajectory = StopAndGoLeaderTrajectory(
            p=3000, vh=20, vl=10, vf=30, v_change_steps=[30, 50],
            trajectory_len=self.ep_len + 50, ts=Params.ts,
        )
        np.random.seed(seed)
        self.masses = np.random.uniform(700, 1000, n).tolist()
