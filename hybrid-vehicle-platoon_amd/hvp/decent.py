"""Decentralised MLD controller: coordinator + ``simulate`` (fleet_decent_mld.py:285-559).

``TrackingDecentMldCoordinator`` keeps the reference's interface and bookkeeping
(``get_control``, ``on_episode_start``, ``on_timestep_end``, ``observe_states`` with the three
velocity estimators, ``solve_times`` / ``node_counts``) but solves the n local MIQPs of a step
in ONE ``hvp_solve_batch`` call instead of n serial Gurobi solves (fleet_decent_mld.py:316) --
they are independent given the measured state.  ``run_time`` of every agent is that call's
time: the agents run in parallel, which is what the reference models with max over agents
(:334-338).
"""

from __future__ import annotations

import pickle
import time
from typing import Literal

import numpy as np

from . import _abi
from .agent import MldAgent
from .batched import extrapolate
from .env import EpisodeMonitor, PlatoonEnv
from .models import Platoon, Vehicle
from .mpc import LocalMpcGear, LocalMpcMld
from .params import Params, Sim
from .solver import BatchSolver
from .tables import gears_of


class TrackingDecentMldCoordinator(MldAgent):
    def __init__(self, local_mpcs: list, ep_len: int, N: int, leader_x: np.ndarray, ts: float,
                 leader_index: int = 0, velocity_estimator: Literal["none", "two_point", "sat"] = "none") -> None:
        super().__init__(local_mpcs[0])
        self.n = len(local_mpcs)
        self.ep_len = ep_len
        self.ts = ts
        self.N = N
        self.leader_x = leader_x
        self.leader_index = leader_index
        self.velocity_estimator = velocity_estimator
        self.nx_l = Vehicle.nx_l
        self.nu_l = Vehicle.nu_l
        self.agents = [MldAgent(m) for m in local_mpcs]
        self.solve_times = np.zeros((ep_len, 1))
        self.node_counts = np.zeros((ep_len, 1))
        # one handle for the whole platoon: every vehicle's table, the shared controller constants
        prob = local_mpcs[0].problem
        for m in local_mpcs[1:]:
            if bytes(m.problem) != bytes(prob):
                raise ValueError("local MPCs must share the controller constants")
        self._solver = BatchSolver(prob, [m.table for m in local_mpcs])
        self._sys = np.arange(self.n, dtype=np.int32)
        self._roles = np.array([m.role for m in local_mpcs], dtype=np.int32)

    # ------------------------------------------------------------ control (batched)
    def get_control(self, state: np.ndarray, raises: bool = True):
        x = np.asarray(state, dtype=np.float64).reshape(self.n, self.nx_l)
        params = np.stack([a.mpc.params_for(x[i]) for i, a in enumerate(self.agents)])
        t0 = time.perf_counter()
        res = self._solver.solve(self._sys, self._roles, params)
        dt = time.perf_counter() - t0
        u = []
        for i, a in enumerate(self.agents):
            ui, info = a.mpc.absorb(res, i, dt, raises, x[i])
            a.record(info)
            u.append(ui)
        if u[0].shape[0] > self.nu_l:  # gear MPCs: continuous controls first, then the gears (:318-324)
            return np.vstack((np.vstack([ui[: self.nu_l] for ui in u]), np.vstack([ui[self.nu_l:] for ui in u]))), {}
        return np.vstack(u), {}

    # ------------------------------------------------------------ hooks
    def on_timestep_end(self, env, episode: int, timestep: int) -> None:
        self.agents[self.leader_index].mpc.set_leader_x(self.leader_x[:, timestep:timestep + self.N + 1])
        self.observe_states(env, timestep)
        self.solve_times[env.step_counter - 1, :] = max(a.run_time for a in self.agents)
        self.node_counts[env.step_counter - 1, :] = max(a.node_count for a in self.agents)

    def on_episode_start(self, env, episode: int, state) -> None:
        self.agents[self.leader_index].mpc.set_leader_x(self.leader_x[:, 0:self.N + 1])
        self.observe_states(env, timestep=0)

    def observe_states(self, env, timestep) -> None:
        """Neighbour predictions from the measured state (fleet_decent_mld.py:348-419)."""
        x = np.asarray(env.x, dtype=np.float64).reshape(-1)
        # the reference tests the truthiness of the estimator string, so 'none' also reads the
        # previous state (fleet_decent_mld.py:349-350); only two_point / sat use it
        xp = np.asarray(env.get_previous_state(), dtype=np.float64).reshape(-1)
        for i in range(self.n):
            def pred(j):
                p, v = x[2 * j], x[2 * j + 1]
                if self.velocity_estimator in ("two_point", "sat"):
                    return extrapolate(p, v, self.N, self.ts, v - xp[2 * j + 1], self.velocity_estimator == "sat")
                return self.extrapolate_position_constant_vel(p, v)
            if i > 0:
                self.agents[i].mpc.set_x_front(pred(i - 1))
            if i < self.n - 1:
                self.agents[i].mpc.set_x_back(pred(i + 1))

    def extrapolate_position_constant_vel(self, initial_pos: float, initial_vel: float) -> np.ndarray:
        return extrapolate(initial_pos, initial_vel, self.N, self.ts)

    def extrapolate_position_two_point_estimator(self, initial_pos, initial_vel, previous_vel) -> np.ndarray:
        return extrapolate(initial_pos, initial_vel, self.N, self.ts, initial_vel - previous_vel)

    def extrapolate_position_two_point_estimator_saturated(self, initial_pos, initial_vel, previous_vel):
        return extrapolate(initial_pos, initial_vel, self.N, self.ts, initial_vel - previous_vel, sat=True)


def simulate(sim: Sim, save: bool = False, plot: bool = False, seed: int = 2, thread_limit: int | None = None,
             velocity_estimator: Literal["none", "two_point", "sat"] = "none", leader_index: int = 0,
             verbose: bool = False):
    """Closed-loop run of the decentralised controller (fleet_decent_mld.py:458-559)."""
    n, N, ep_len, ts = sim.n, sim.N, sim.ep_len, Params.ts
    leader_x = sim.leader_trajectory.get_leader_trajectory()
    platoon = Platoon(n, vehicle_type=sim.vehicle_model_type, masses=sim.masses)
    if sim.vehicle_model_type not in ("pwa_gear", "pwa_friction"):
        raise NotImplementedError("the GPU path implements the pwa_gear (LocalMpcMld) and pwa_friction "
                                  "(LocalMpcGear) models; the nonlinear model is out of scope (DESIGN.md)")
    systems = platoon.get_vehicle_system_dicts(ts)
    env = EpisodeMonitor(
        PlatoonEnv(n=n, platoon=platoon, leader_trajectory=sim.leader_trajectory, spacing_policy=sim.spacing_policy,
                   start_from_platoon=sim.start_from_platoon, real_vehicle_as_reference=sim.real_vehicle_as_reference,
                   ep_len=ep_len, leader_index=leader_index, verbose=verbose),
        max_episode_steps=ep_len,
    )
    vehicles = platoon.get_vehicles()
    def local(i):
        kw = dict(is_front=i == 0, is_leader=i == leader_index, is_trailer=i == n - 1, thread_limit=thread_limit,
                  real_vehicle_as_reference=sim.real_vehicle_as_reference)
        if sim.vehicle_model_type == "pwa_friction":  # fleet_decent_mld.py:532-533
            return LocalMpcGear(N, systems[i], sim.spacing_policy, **kw)
        return LocalMpcMld(N, systems[i], sim.spacing_policy, gears=gears_of(vehicles[i]), **kw)

    mpcs = [local(i) for i in range(n)]
    agent = TrackingDecentMldCoordinator(mpcs, ep_len=ep_len, N=N, leader_x=leader_x, ts=ts,
                                         velocity_estimator=velocity_estimator, leader_index=leader_index)
    agent.evaluate(env=env, episodes=1, seed=seed)
    X = env.observations[0].squeeze()
    U = env.actions[0].squeeze()
    R = env.rewards[0]
    if verbose:
        print(f"Return = {sum(R.squeeze())}")
        print(f"Violations = {env.unwrapped.viol_counter}")
        print(f"Run_times_sum: {sum(agent.solve_times)}")
    if save:
        with open(f"decent_vest_{velocity_estimator}_{sim.id}_seed_{seed}.pkl", "wb") as f:
            for obj in (X, U, R, agent.solve_times, agent.node_counts, env.unwrapped.viol_counter[0], leader_x):
                pickle.dump(obj, f)
    return X, U, R, agent, env
