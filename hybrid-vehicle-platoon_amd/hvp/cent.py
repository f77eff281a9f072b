"""Centralised MLD controller (mpcs/cent_mld.py, fleet_cent_mld.py) on the GPU.

* :class:`CentSolver` owns one ``HVP_FORM_CENT`` handle and solves P independent platoon MIQPs
  per ``hvp_cent_solve_batch`` call (one wavefront per platoon runs the whole branch and bound,
  csrc/hvp_cent_bnb.h).  ``solve_device`` takes torch tensors already on the GPU (the bench
  path); ``solve`` numpy arrays.
* :class:`MpcMldCent` <- mpcs/cent_mld.py:9-182: constructor arguments, ``set_leader_traj``
  (:179-182) and ``solve_mpc(state, raises) -> (u (n, 1), info)`` with the info keys of the
  MpcMld family (``x`` (2n, N+1) stacked per vehicle, ``u`` (n, N), ``cost``, ``run_time``,
  ``nodes``, ``bin_vars`` = 7 n N).
* :class:`MpcGearCent` <- fleet_cent_mld.py:25-52: the pwa_friction model with gear binaries,
  ``solve_mpc -> [u_g0 (n); gear0 (n)]`` and ``info["u"] = vstack(u_g, gears)`` (mpc_gear.py:116-135).
* :class:`TrackingCentralizedAgent` <- fleet_cent_mld.py:80-101 and :func:`simulate` <- :104-213.
"""

from __future__ import annotations

import ctypes
import pickle
import time
from dataclasses import dataclass

import numpy as np

from . import _abi, tables
from .agent import MldAgent
from .env import EpisodeMonitor, PlatoonEnv
from .models import Platoon, Vehicle
from .params import ConstantSpacingPolicy, Params, Sim, SpacingPolicy

DEFAULT_MAX_NODES = 2_000_000  # batched solves (bench.py names it in its metric)
# The per-platoon drop-in (MpcMldCent.solve_mpc) searches to the optimum like the reference's
# Gurobi call: the heaviest C2-size platoon found (seed 426) needs 27.8M QPs (84 s alone on one
# MI355X, profiles/r04l_cent_heavy_426_cap30M.jsonl); past this cap the call raises as the
# reference does on a non-optimal status.  Worst case at the default: ~3 QPs per 10 us on one
# MI355X for a platoon that splits over the whole chip, i.e. about 3 minutes for one call that
# exhausts 64M QPs; MpcMldCent(max_nodes=...) bounds it per controller.
DROPIN_MAX_NODES = 64_000_000


def cent_problem(N: int, spacing_policy: SpacingPolicy | None = None, quadratic_cost: bool = True,
                 accel_cnstr_tightening: float = 0.0, params=Params, exhaustive: bool = False) -> _abi.HvpProblem:
    """hvp_problem of MpcMldCent.setup_cost_and_constraints (mpcs/cent_mld.py:48-177)."""
    p = tables.problem(N, spacing_policy, quadratic_cost, accel_cnstr_tightening, params=params,
                       method=_abi.METHOD_ENUMERATE if exhaustive else _abi.METHOD_BNB)
    p.formulation = _abi.FORM_CENT
    return p


@dataclass
class CentResult:
    u: np.ndarray       # (P, n, N)
    x: np.ndarray       # (P, n, 2, N+1)
    region: np.ndarray  # (P, n, N)  -1 without a solution
    gear: np.ndarray    # (P, n, N)
    cost: np.ndarray    # (P,)
    status: np.ndarray  # (P,)
    nodes: np.ndarray   # (P,) QPs solved (bounds, leaves, the final re-solve)
    iters: np.ndarray   # (P,) active-set iterations


class CentSolver:
    """One HVP_FORM_CENT handle: the controller constants and the vehicles' PWA tables."""

    def __init__(self, problem: _abi.HvpProblem, systems: list[_abi.HvpSystem], device: int = 0) -> None:
        if int(problem.formulation) != _abi.FORM_CENT:
            raise ValueError("CentSolver needs an HVP_FORM_CENT problem (cent_problem)")
        self._lib = _abi.load()
        self.N = int(problem.N)
        self.problem = problem
        self.n_systems = len(systems)
        arr = (_abi.HvpSystem * len(systems))(*systems)
        h = ctypes.c_void_p()
        _abi.check(self._lib.hvp_create(ctypes.byref(h), ctypes.byref(problem), arr, len(systems), device), "hvp_create")
        self._h = h
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.hvp_destroy(self._h)
            self._h = None

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def stats(self) -> _abi.HvpStats:
        s = _abi.HvpStats()
        _abi.check(self._lib.hvp_get_stats(self._h, ctypes.byref(s)), "hvp_get_stats")
        return s

    def alloc_outputs(self, P: int, n: int, device=None) -> dict:
        import torch

        dev = device or torch.device("cuda", self.device)
        N = self.N
        return {
            "u": torch.empty((P, n, N), dtype=torch.float64, device=dev),
            "x": torch.empty((P, n, 2, N + 1), dtype=torch.float64, device=dev),
            "region": torch.empty((P, n, N), dtype=torch.int8, device=dev),
            "gear": torch.empty((P, n, N), dtype=torch.int8, device=dev),
            "cost": torch.empty((P,), dtype=torch.float64, device=dev),
            "status": torch.empty((P,), dtype=torch.int32, device=dev),
            "nodes": torch.empty((P,), dtype=torch.int32, device=dev),
            "iters": torch.empty((P,), dtype=torch.int32, device=dev),
        }

    def solve_device(self, sys_idx, x0, leader_x, leader_index: int = 0, real_vehicle_as_reference: bool = False,
                     max_nodes: int = DEFAULT_MAX_NODES, out: dict | None = None, stream=None) -> dict:
        """sys_idx (P, n) int32, x0 (P, n, 2) float64, leader_x (P, 2, N+1) float64, all contiguous
        CUDA tensors; asynchronous on ``stream`` (default: the current torch stream)."""
        import torch

        if sys_idx.dim() != 2:
            raise ValueError("sys_idx must be (P, n)")
        P, n = int(sys_idx.shape[0]), int(sys_idx.shape[1])
        for name, t, dt, shape in (("sys_idx", sys_idx, torch.int32, (P, n)), ("x0", x0, torch.float64, (P, n, 2)),
                                   ("leader_x", leader_x, torch.float64, (P, 2, self.N + 1))):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous() or tuple(t.shape) != shape:
                raise ValueError(f"{name} must be a contiguous CUDA {shape} tensor of dtype {dt}")
        out = out or self.alloc_outputs(P, n, x0.device)
        if stream is None:
            stream = torch.cuda.current_stream(x0.device)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = self._lib.hvp_cent_solve_batch(
            self._h, P, n, int(leader_index), 1 if real_vehicle_as_reference else 0, ptr(sys_idx), ptr(x0),
            ptr(leader_x), int(max_nodes), ptr(out["u"]), ptr(out["x"]), ptr(out["region"]), ptr(out["gear"]),
            ptr(out["cost"]), ptr(out["status"]), ptr(out["nodes"]), ptr(out["iters"]),
            ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_cent_solve_batch")
        return out

    def solve(self, sys_idx, x0, leader_x, leader_index: int = 0, real_vehicle_as_reference: bool = False,
              max_nodes: int = DEFAULT_MAX_NODES) -> CentResult:
        """Host-array form (synchronous): sys_idx (P, n), x0 (P, n, 2) or (P, 2n), leader_x
        (P, 2, N+1) or (2, N+1) shared by all platoons."""
        import torch

        sys_idx = np.asarray(sys_idx, dtype=np.int32)
        if sys_idx.ndim == 1:
            sys_idx = sys_idx[None]
        P, n = sys_idx.shape
        if P and (sys_idx.min() < 0 or sys_idx.max() >= self.n_systems):
            raise ValueError("system index out of range")
        x0 = np.asarray(x0, dtype=np.float64).reshape(P, n, 2)
        lx = np.asarray(leader_x, dtype=np.float64)
        lx = np.array(np.broadcast_to(lx.reshape(-1, 2, self.N + 1), (P, 2, self.N + 1)))
        dev = torch.device("cuda", self.device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        out = self.solve_device(t(sys_idx), t(x0), t(lx), leader_index, real_vehicle_as_reference, max_nodes)
        torch.cuda.synchronize(dev)
        h = {k: v.cpu().numpy() for k, v in out.items()}
        return CentResult(**h)


class MpcMldCent:
    """A centralized MPC controller for the platoon using the mixed-integer MLD approach
    (mpcs/cent_mld.py:9-182), solved on the GPU."""

    Q_x = Params.Q_x
    Q_u = Params.Q_u
    Q_du = Params.Q_du
    w = Params.w
    a_acc = Params.a_acc
    a_dec = Params.a_dec
    ts = Params.ts
    d_safe = Params.d_safe

    def __init__(self, n: int, N: int, pwa_systems: list[dict], spacing_policy: SpacingPolicy = ConstantSpacingPolicy(50),
                 leader_index: int = 0, quadratic_cost: bool = True, thread_limit: int | None = None,
                 accel_cnstr_tightening: float = 0.0, real_vehicle_as_reference: bool = False, gears=None,
                 max_nodes: int = DROPIN_MAX_NODES) -> None:
        """The reference's constructor arguments (mpcs/cent_mld.py:11-47), plus ``max_nodes``: the QPs
        one solve_mpc call may search before it reports a non-optimal status (see DROPIN_MAX_NODES)."""
        if max_nodes < 1:
            raise ValueError("max_nodes must be >= 1")
        self.n, self.N = n, N
        self.thread_limit = thread_limit  # no CPU thread pool: kept for signature compatibility
        if len(pwa_systems) != n:
            raise ValueError(f"expected {n} vehicle systems, got {len(pwa_systems)}")
        self.tables = self._tables(pwa_systems, gears)
        self.num_bin_vars = sum(len(s["S"]) for s in pwa_systems) * N
        self.setup_cost_and_constraints(None, spacing_policy, leader_index, quadratic_cost, accel_cnstr_tightening,
                                        real_vehicle_as_reference)
        self.leader_traj = np.zeros((2, N + 1))
        self.max_nodes = int(max_nodes)
        self.x_pred: np.ndarray | None = None
        self.u_pred: np.ndarray | None = None
        self.regions_pred: np.ndarray | None = None
        self.gears_pred: np.ndarray | None = None

    def _tables(self, pwa_systems, gears):
        return [tables.system_from_dict(s, None if gears is None else gears[i]) for i, s in enumerate(pwa_systems)]

    def setup_cost_and_constraints(self, u, spacing_policy=ConstantSpacingPolicy(50), leader_index: int = 0,
                                   quadratic_cost: bool = True, accel_cnstr_tightening: float = 0.0,
                                   real_vehicle_as_reference: bool = False) -> None:
        """mpcs/cent_mld.py:48-177: the cost / constraint constants become the handle's problem
        (quadratic_cost=False: the min_1_norm objective, epigraph variables per vehicle and step,
        solved as LPs by csrc/hvp_cent_l1.h)."""
        if leader_index != 0 and real_vehicle_as_reference:
            raise NotImplementedError("Not implemented for real vehicle with leader not 0.")
        self.leader_index = int(leader_index)
        self.real_vehicle_as_reference = bool(real_vehicle_as_reference)
        self.spacing_policy = spacing_policy
        self.problem = cent_problem(self.N, spacing_policy, quadratic_cost, accel_cnstr_tightening, params=type(self))
        self._solver = CentSolver(self.problem, self.tables)
        self._sys = np.arange(self.n, dtype=np.int32)[None]

    def set_leader_traj(self, leader_traj) -> None:
        a = np.asarray(leader_traj, dtype=np.float64)
        if a.shape != (2, self.N + 1):
            raise ValueError(f"expected a (2, {self.N + 1}) leader trajectory, got {a.shape}")
        self.leader_traj = a.copy()

    def solve_mpc(self, state, raises: bool = True):
        x0 = np.asarray(state, dtype=np.float64).reshape(1, self.n, 2)
        t0 = time.perf_counter()
        res = self._solver.solve(self._sys, x0, self.leader_traj[None], self.leader_index,
                                 self.real_vehicle_as_reference, self.max_nodes)
        return self.absorb(res, 0, time.perf_counter() - t0, raises, state)

    def absorb(self, res: CentResult, p: int, run_time: float, raises: bool, state=None):
        ok = int(res.status[p]) == _abi.OPTIMAL
        n, N = self.n, self.N
        if not ok:
            if raises:
                raise RuntimeError(f"MPC for state {np.asarray(state).reshape(-1)} returned "
                                   f"{_abi.STATUS_NAMES.get(int(res.status[p]))}")
            x, u, cost = np.zeros((2 * n, N + 1)), np.zeros((n, N)), float("inf")
        else:
            x = res.x[p].reshape(2 * n, N + 1).copy()
            u = res.u[p].copy()
            cost = float(res.cost[p])
        self.x_pred, self.u_pred = x, u
        self.regions_pred = res.region[p].copy()
        self.gears_pred = res.gear[p].astype(float)
        info = {"x": x, "u": u, "cost": cost, "run_time": run_time, "nodes": int(res.nodes[p]),
                "bin_vars": self.num_bin_vars, "status": int(res.status[p])}
        return u[:, [0]], info


class MpcGearCent(MpcMldCent):
    """fleet_cent_mld.py:25-52: the centralised MPC on the pwa_friction model with gear binaries
    (MpcGear.setup_gears on the stacked controls, mpcs/mpc_gear.py:30-114).  As in
    :class:`hvp.mpc.MpcGear` every vehicle's table holds one mode per (gear, friction region);
    the control box moves onto u_g and the cost is on u_g."""

    def _tables(self, pwa_systems, gears):
        return [tables.gear_system_from_dict(s) for s in pwa_systems]

    def __init__(self, n: int, N: int, systems: list[dict], spacing_policy: SpacingPolicy = ConstantSpacingPolicy(50),
                 leader_index: int = 0, quadratic_cost: bool = True, thread_limit: int | None = None,
                 accel_cnstr_tightening: float = 0.0, real_vehicle_as_reference: bool = False,
                 max_nodes: int = DROPIN_MAX_NODES) -> None:
        super().__init__(n, N, systems, spacing_policy, leader_index, quadratic_cost, thread_limit,
                         accel_cnstr_tightening, real_vehicle_as_reference, max_nodes=max_nodes)
        # delta (PWA regions) + sigma (gears) per vehicle and step
        self.num_bin_vars = sum(len(s["S"]) + len(Vehicle.b) for s in systems) * N

    def absorb(self, res: CentResult, p: int, run_time: float, raises: bool, state=None):
        """[u_g0; gear0] with info["u"] = vstack(u_g, gears) (mpc_gear.py:116-135)."""
        ok = int(res.status[p]) == _abi.OPTIMAL
        if not ok and raises:
            raise RuntimeWarning(f"gear mpc for state {np.asarray(state).reshape(-1)} is infeasible.")
        _, info = MpcMldCent.absorb(self, res, p, run_time, False, state)
        if ok:
            u_g = res.u[p].copy()
            gears = res.gear[p].astype(float)
        else:
            u_g = np.zeros((self.n, self.N))
            gears = 6 * np.ones((self.n, self.N))  # default: all gears 6 (:129-131)
        info["u"] = np.vstack((u_g, gears))
        self.gears_pred = gears
        return np.vstack((u_g[:, [0]], gears[:, [0]])), info


class TrackingCentralizedAgent(MldAgent):
    """fleet_cent_mld.py:80-101."""

    def __init__(self, mpc: MpcMldCent, ep_len: int, N: int, leader_x: np.ndarray) -> None:
        self.ep_len = ep_len
        self.N = N
        self.leader_x = leader_x
        self.solve_times = np.zeros((ep_len, 1))
        self.node_counts = np.zeros((ep_len, 1))
        self.bin_var_counts = np.zeros((ep_len, 1))
        super().__init__(mpc)

    def on_timestep_end(self, env, episode: int, timestep: int) -> None:
        # time step starts from 1, so this sets the cost for the next time step
        self.mpc.set_leader_traj(self.leader_x[:, timestep:timestep + self.N + 1])
        self.solve_times[env.step_counter - 1, :] = self.run_time
        self.node_counts[env.step_counter - 1, :] = self.node_count
        self.bin_var_counts[env.step_counter - 1, :] = self.num_bin_vars
        return super().on_timestep_end(env, episode, timestep)

    def on_episode_start(self, env, episode: int, state) -> None:
        self.mpc.set_leader_traj(self.leader_x[:, 0:self.N + 1])
        return super().on_episode_start(env, episode, state)


def simulate(sim: Sim, save: bool = False, plot: bool = False, seed: int = 1, thread_limit: int | None = None,
             leader_index: int = 0):
    """Closed-loop run of the centralised controller (fleet_cent_mld.py:104-213)."""
    n, N, ep_len, ts = sim.n, sim.N, sim.ep_len, Params.ts
    leader_x = sim.leader_trajectory.get_leader_trajectory()
    platoon = Platoon(n, vehicle_type=sim.vehicle_model_type, masses=sim.masses)
    systems = platoon.get_vehicle_system_dicts(ts)
    env = EpisodeMonitor(
        PlatoonEnv(n=n, platoon=platoon, leader_trajectory=sim.leader_trajectory, spacing_policy=sim.spacing_policy,
                   start_from_platoon=sim.start_from_platoon, real_vehicle_as_reference=sim.real_vehicle_as_reference,
                   ep_len=ep_len, leader_index=leader_index, quadratic_cost=sim.quadratic_cost),
        max_episode_steps=ep_len,
    )
    kw = dict(spacing_policy=sim.spacing_policy, leader_index=leader_index, thread_limit=thread_limit,
              real_vehicle_as_reference=sim.real_vehicle_as_reference, quadratic_cost=sim.quadratic_cost)
    if sim.vehicle_model_type == "pwa_gear":
        mpc = MpcMldCent(n, N, systems, gears=[tables.gears_of(v) for v in platoon.get_vehicles()], **kw)
    elif sim.vehicle_model_type == "pwa_friction":
        mpc = MpcGearCent(n, N, systems, **kw)
    elif sim.vehicle_model_type == "nonlinear":
        raise NotImplementedError("MpcNonlinearGearCent (nonlinear vehicle model) is out of scope (DESIGN.md)")
    else:
        raise ValueError(f"{sim.vehicle_model_type} is not a valid vehicle model type.")
    agent = TrackingCentralizedAgent(mpc, ep_len, N, leader_x)
    agent.evaluate(env=env, episodes=1, seed=seed, open_loop=sim.open_loop)
    X = env.observations[0].squeeze()
    U = env.actions[0].squeeze()
    R = env.rewards[0]
    if save:
        with open(f"cent_{sim.id}_seed_{seed}.pkl", "wb") as f:
            for obj in (X, U, R, agent.solve_times, agent.node_counts, env.unwrapped.viol_counter[0], leader_x):
                pickle.dump(obj, f)
    return X, U, R, agent, env
