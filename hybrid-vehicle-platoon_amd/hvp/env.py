"""Platoon plant / environment -- the *caller* of the hot path, restated without gymnasium.

Follows the reference's ``env.py:12-219`` (``PlatoonEnv``): random initial platoon
(``reset``, env.py:70-116, including the int64 state array that truncates the sampled
positions and velocities, env.py:79/99-100), stage cost and safe-distance violations
(``get_stage_cost``, env.py:126-180) and the step through the nonlinear model with
10 Euler sub-steps (``step``, env.py:182-212 -> models.py:236-257).

Only the gymnasium base class and the ``TimeLimit``/``MonitorEpisodes`` wrappers
(mpcrl, not installed here) are dropped; :class:`EpisodeMonitor` records the same
observations / actions / rewards lists that ``simulate()`` reads back.
"""

from __future__ import annotations

from typing import Any

import numpy as np

from .models import Platoon
from .params import ConstantSpacingPolicy, ConstantVelocityLeaderTrajectory, LeaderTrajectory, SpacingPolicy


def derive_env_seed(seed: int | None, episode: int = 0) -> int | None:
    """Seed the agent's ``evaluate`` hands to ``env.reset``.

    mpcrl's ``Agent.evaluate`` draws the per-episode env seeds from
    ``np.random.SeedSequence(seed).generate_state(episodes)`` (the reference hard-codes the
    episode-0 value for seed 0, 2968811710, at model_validation.py:76).
    """
    if seed is None:
        return None
    return int(np.random.SeedSequence(seed).generate_state(episode + 1)[episode])


def initial_platoon_state(n: int, seed: int | None) -> np.ndarray:
    """x0 of ``PlatoonEnv.reset`` with ``start_from_platoon=False`` (env.py:79-101).

    100 velocities 30*U+5 are drawn first, then 99 position decrements 100*U+60 from 3000;
    the n largest positions are assigned in order and every value is truncated to int64.
    """
    rs_state = np.random.get_state()
    try:
        np.random.seed(seed)
        vel = 30 * np.random.random(100) + 5
        steps = 100 * np.random.random(99)
    finally:
        np.random.set_state(rs_state)
    pos = np.empty(100)
    pos[0] = 3000.0
    for i in range(1, 100):
        pos[i] = -steps[i - 1] + pos[i - 1] - 60  # same operation order as env.py:92-94
    x = np.zeros((2 * n, 1), dtype=np.int64)
    x[0::2, 0] = np.sort(pos)[::-1][:n].astype(np.int64)
    x[1::2, 0] = vel[:n].astype(np.int64)
    return x


class PlatoonEnv:
    """n nonlinear hybrid vehicles tracking a leader trajectory."""

    Q_x = np.diag([1.0, 0.1])
    Q_u = 1 * np.eye(1)
    Q_du = 0 * np.eye(1)
    nx_l = Platoon.nx_l
    nu_l = Platoon.nu_l

    def __init__(
        self,
        n: int,
        platoon: Platoon,
        ep_len: int,
        leader_index: int = 0,
        ts: float = 1,
        leader_trajectory: LeaderTrajectory | None = None,
        spacing_policy: SpacingPolicy | None = None,
        d_safe: float = 25,
        start_from_platoon: bool = False,
        quadratic_cost: bool = True,
        real_vehicle_as_reference: bool = False,
        verbose: bool = False,
    ) -> None:
        if leader_index != 0 and real_vehicle_as_reference:
            raise NotImplementedError("Not implemented for real vehicle with leader not 0.")
        self.n, self.platoon, self.ep_len, self.ts = n, platoon, ep_len, ts
        self.leader_index = leader_index
        self.leader_trajectory = leader_trajectory or ConstantVelocityLeaderTrajectory(
            p=3000, v=20, trajectory_len=150, ts=1
        )
        self.spacing_policy = spacing_policy or ConstantSpacingPolicy(50)
        self.d_safe = d_safe
        self.start_from_platoon = start_from_platoon
        self.real_vehicle_as_reference = real_vehicle_as_reference
        self.quadratic_cost = quadratic_cost
        self.verbose = verbose
        self.step_counter = 0
        self.viol_counter: list[np.ndarray] = []
        self.previous_action: np.ndarray | None = None
        self.previous_state: np.ndarray | None = None
        self.x: np.ndarray | None = None

    # -------------------------------------------------------------- reset / step
    def reset(self, *, seed: int | None = None, options: dict[str, Any] | None = None):
        self.leader_x = self.leader_trajectory.get_leader_trajectory()
        if not self.start_from_platoon:
            self.x = initial_platoon_state(self.n, seed)
        else:
            x = np.zeros((2 * self.n, 1), dtype=np.int64)
            lead = self.leader_x[:, [0]]
            off = 1 if self.real_vehicle_as_reference else 0
            for i in range(self.n):
                x[2 * i : 2 * i + 2, :] = lead + (i + off) * self.spacing_policy.spacing(lead)
            self.x = x
        self.step_counter = 0
        self.previous_action = None
        self.previous_state = None
        self.viol_counter.append(np.zeros(self.ep_len))
        return self.x, {}

    def _cost(self, e: np.ndarray, Q: np.ndarray):
        """quad_cost / lin_cost (env.py:118-124): x'Qx is a (1, 1) array as in the reference, so
        the stage cost -- and the rewards the results files store -- keep its shape
        (results_analysis/perf_n.py reads sum(R)[0, 0])."""
        if self.quadratic_cost:
            return e.T @ Q @ e
        return np.linalg.norm(Q @ e, ord=1)

    def get_stage_cost(self, state: np.ndarray, action: np.ndarray):
        if self.previous_action is None:
            self.previous_action = action
        xs = np.split(np.asarray(state, dtype=float), self.n, axis=0)
        us = np.split(action, self.n, axis=0)
        ups = np.split(self.previous_action, self.n, axis=0)
        ref = self.leader_x[:, [self.step_counter]]
        sp = self.spacing_policy
        if self.real_vehicle_as_reference:
            cost = self._cost(xs[0] - ref - sp.spacing(xs[0]), self.Q_x)
        else:
            cost = self._cost(xs[self.leader_index] - ref, self.Q_x)
        cost += sum(self._cost(xs[i] - xs[i - 1] - sp.spacing(xs[i]), self.Q_x) for i in range(1, self.n))
        cost += sum(self._cost(us[i], self.Q_u) for i in range(self.n))
        cost += sum(self._cost(us[i] - ups[i], self.Q_du) for i in range(self.n))
        too_close = any(xs[i][0, 0] - xs[i + 1][0, 0] < self.d_safe for i in range(self.n - 1))
        if self.real_vehicle_as_reference and self.leader_x[0, self.step_counter] - xs[0][0, 0] < self.d_safe:
            self.viol_counter[-1][self.step_counter] = 100
        elif too_close:
            self.viol_counter[-1][self.step_counter] = 100
        self.previous_action = action
        self.previous_state = state
        return cost

    def step(self, action: np.ndarray):
        action = np.asarray(action)
        if action.shape not in ((self.n * self.nu_l, 1), (2 * self.n * self.nu_l, 1)):
            raise ValueError(f"Expected action of size {(self.n, 1)} or {(2 * self.n, 1)}. Got {action.shape}")
        if action.shape[0] == 2 * self.n:
            u, j = action[: self.n, :], action[self.n :, :]
        else:
            u = action
            j = np.array(
                [[self.platoon.get_gear_from_vehicle_velocity(i, float(self.x[2 * i + 1, 0]))] for i in range(self.n)]
            )
        r = self.get_stage_cost(self.x, u)
        self.x = self.platoon.step_platoon(self.x, u, j, self.ts)
        self.step_counter += 1
        if self.verbose:
            print(f"step {self.step_counter}")
        return self.x, r, False, False, {}

    def get_state(self) -> np.ndarray:
        return self.x

    def get_previous_state(self) -> np.ndarray:
        return self.previous_state if self.previous_state is not None else self.x


class EpisodeMonitor:
    """The slice of ``MonitorEpisodes``/``TimeLimit`` that ``simulate()`` relies on."""

    def __init__(self, env: PlatoonEnv, max_episode_steps: int) -> None:
        self.env = env
        self.max_episode_steps = max_episode_steps
        self.observations: list[np.ndarray] = []
        self.actions: list[np.ndarray] = []
        self.rewards: list[np.ndarray] = []
        self._obs: list = []
        self._act: list = []
        self._rew: list = []

    @property
    def unwrapped(self) -> PlatoonEnv:
        return self.env

    def __getattr__(self, name):
        return getattr(self.env, name)

    def reset(self, *, seed=None, options=None):
        x, info = self.env.reset(seed=seed, options=options)
        self._obs, self._act, self._rew = [np.asarray(x, dtype=float).copy()], [], []
        return x, info

    def step(self, action):
        x, r, term, trunc, info = self.env.step(action)
        self._obs.append(np.asarray(x, dtype=float).copy())
        self._act.append(np.asarray(action, dtype=float).copy())
        self._rew.append(r)
        trunc = trunc or self.env.step_counter >= self.max_episode_steps
        if term or trunc:
            self.observations.append(np.stack(self._obs))
            self.actions.append(np.stack(self._act))
            self.rewards.append(np.asarray(self._rew))
        return x, r, term, trunc, info
