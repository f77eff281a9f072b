"""Agent layer: the slice of dmpcpwa ``MldAgent`` / mpcrl ``Agent`` the reference's drivers use.

Evidence of the surface (all in the reference): ``get_control(state) -> (u, info)``
(fleet_decent_mld.py:316), ``run_time`` / ``node_count`` (:336-337), ``num_bin_vars``
(fleet_cent_mld.py:96), ``get_predicted_state(shifted)`` (fleet_naive_admm.py:394-402),
``get_predicted_cost`` (fleet_event_based.py:512) and ``evaluate(env, episodes, seed)``
driving the ``on_episode_start`` / ``on_timestep_end`` hooks (fleet_decent_mld.py:329-346, 530).
"""

from __future__ import annotations

import numpy as np

from .env import derive_env_seed


class MldAgent:
    def __init__(self, mpc) -> None:
        self.mpc = mpc
        self.run_time = 0.0
        self.node_count = 0
        self.num_bin_vars = getattr(mpc, "num_bin_vars", 0)
        self.x_pred: np.ndarray | None = None
        self.u_pred: np.ndarray | None = None
        self.cost_pred: float | None = None

    # ------------------------------------------------------------ control
    def record(self, info: dict) -> None:
        self.run_time = info["run_time"]
        self.node_count = info["nodes"]
        self.num_bin_vars = info["bin_vars"]
        self.x_pred = info["x"]
        self.u_pred = info["u"]
        self.cost_pred = info["cost"]

    def get_control(self, state: np.ndarray, raises: bool = True):
        u, info = self.mpc.solve_mpc(state, raises=raises)
        self.record(info)
        return u, info

    def get_predicted_state(self, shifted: bool = False) -> np.ndarray | None:
        if self.x_pred is None:
            return None
        if not shifted:
            return self.x_pred
        return np.hstack((self.x_pred[:, 1:], self.x_pred[:, [-1]]))

    def get_predicted_cost(self) -> float | None:
        return self.cost_pred

    # ------------------------------------------------------------ episode loop (mpcrl Agent.evaluate)
    def on_episode_start(self, env, episode: int, state) -> None:
        pass

    def on_timestep_end(self, env, episode: int, timestep: int) -> None:
        pass

    def evaluate(self, env, episodes: int, seed: int | None = None, raises: bool = True, open_loop: bool = False):
        returns = np.zeros(episodes)
        for ep in range(episodes):
            state, _ = env.reset(seed=derive_env_seed(seed, ep))
            self.on_episode_start(env, ep, state)
            t = 0
            done = False
            while not done:
                action, _ = self.get_control(state)
                state, r, term, trunc, _ = env.step(action)
                returns[ep] += float(np.asarray(r).sum())
                done = term or trunc
                t += 1
                self.on_timestep_end(env, ep, t)
        return returns
