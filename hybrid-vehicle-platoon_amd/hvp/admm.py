"""Naive-ADMM platoon controller (fleet_naive_admm.py) on the GPU.

* :class:`LocalMpcADMM` <- fleet_naive_admm.py:24-258: the local MIQP with neighbour COPIES as
  decision variables (``set_front_vars(y, z)``, ``set_back_vars(y, z)``, ``set_leader_x``;
  after a solve ``x.X``, ``u.X``, ``x_front.X``, ``x_back.X`` as the coordinator reads them).
* :class:`LocalMpcGear` <- :261-288: the same local problem on the pwa_friction model with gear
  binaries (MpcGear.setup_gears); the table enumerates (gear, friction region) modes as
  :class:`hvp.mpc.MpcGear` does, and ``solve_mpc`` returns [u_g0; gear0].
* :class:`AdmmEngine` -- the batched device form of ``ADMMCoordinator.get_control``
  (:379-468) for P platoons of n vehicles: per ADMM iteration ONE ``hvp_solve_admm_batch``
  over all P*n local MIQPs (they only couple through z, y of the previous iteration), then ONE
  ``hvp_admm_update`` launch (z-update, y-update and the next parameter blocks).  Everything
  stays in HBM between iterations.
* :class:`ADMMCoordinator` <- :306-577, the reference's agent surface on top of the engine
  (one platoon), and :func:`simulate` <- :580-692.

The local problem is solved exactly (branch and bound over the region sequences, copies
eliminated in closed form: csrc/hvp_admm.h); the coordinator is the reference's fixed-iteration
ADMM (``admm_iters``, rho = 0.5, y never reset across time steps).
"""

from __future__ import annotations

import ctypes
import pickle
import time

import numpy as np

from . import _abi, tables
from .agent import MldAgent
from .env import EpisodeMonitor, PlatoonEnv
from .models import Platoon, Vehicle
from .params import ConstantSpacingPolicy, Params, Sim, SpacingPolicy
from .solver import BatchSolver


class _Var:
    """The ``.X`` of a Gurobi MVar the reference coordinator reads."""

    def __init__(self, X=None) -> None:
        self.X = X


def admm_problem(N: int, rho: float, spacing_policy: SpacingPolicy | None = None, quadratic_cost: bool = True,
                 accel_cnstr_tightening: float = 0.0, params=Params) -> _abi.HvpProblem:
    p = tables.problem(N, spacing_policy, quadratic_cost, accel_cnstr_tightening, params=params,
                       method=_abi.METHOD_BNB)
    p.formulation = _abi.FORM_ADMM
    p.rho = float(rho)
    return p


class LocalMpcADMM:
    """A local MPC of the ADMM scheme (fleet_naive_admm.py:24-258), GPU-backed."""

    Q_x = Params.Q_x
    Q_u = Params.Q_u
    Q_du = Params.Q_du
    w = Params.w
    a_acc = Params.a_acc
    a_dec = Params.a_dec
    ts = Params.ts
    d_safe = Params.d_safe

    def __init__(self, N: int, pwa_system: dict, rho: float, spacing_policy: SpacingPolicy = ConstantSpacingPolicy(50),
                 quadratic_cost: bool = True, is_front: bool = False, is_leader: bool = False,
                 is_trailer: bool = False, thread_limit: int | None = None, accel_cnstr_tightening: float = 0.0,
                 gears=None) -> None:
        # quadratic_cost=False (min_1_norm, :74-77): L1 tracking / input terms next to the quadratic
        # ADMM terms of the copies, solved by the device's wave interior point with the copies as
        # variables (csrc/hvp_lane.h L1AdmmWave)
        self.quadratic_cost = quadratic_cost
        self.N = N
        self.rho = rho
        self.system = pwa_system
        self.thread_limit = thread_limit
        self.is_front, self.is_leader, self.is_trailer = is_front, is_leader, is_trailer
        self.table = tables.system_from_dict(pwa_system, gears)
        self.num_bin_vars = len(pwa_system["S"]) * N
        self.role = tables.role_bits(is_front, is_trailer, is_leader)
        self.problem = admm_problem(N, rho, spacing_policy, quadratic_cost, accel_cnstr_tightening, params=type(self))
        K = 2 * (N + 1)
        self._K = K
        self._params = np.zeros(_abi.params_stride(N, _abi.FORM_ADMM))
        self.x, self.u = _Var(), _Var()
        self.x_front = _Var() if not is_front else None
        self.x_back = _Var() if not is_trailer else None
        self._solver: BatchSolver | None = None

    # ------------------------------------------------------------ parameter blocks (:239-258)
    def _set(self, block: int, a) -> None:
        a = np.asarray(a, dtype=np.float64)
        if a.shape != (2, self.N + 1):
            raise ValueError(f"expected a (2, {self.N + 1}) array, got {a.shape}")
        self._params[2 + block * self._K:2 + (block + 1) * self._K] = a.reshape(-1)

    def set_front_vars(self, y_front, z_front) -> None:
        self._set(0, y_front)
        self._set(1, z_front)

    def set_back_vars(self, y_back, z_back) -> None:
        self._set(2, y_back)
        self._set(3, z_back)

    def set_leader_x(self, leader_x) -> None:
        self._set(4, leader_x)

    def params_for(self, state) -> np.ndarray:
        p = self._params.copy()
        p[:2] = np.asarray(state, dtype=np.float64).reshape(-1)[:2]
        return p

    # ------------------------------------------------------------ solve
    def solve_mpc(self, state, raises: bool = True):
        if self._solver is None:
            self._solver = BatchSolver(self.problem, [self.table])
        t0 = time.perf_counter()
        res = self._solver.solve_admm(np.zeros(1, np.int32), np.array([self.role], np.int32),
                                      self.params_for(state)[None])
        return self.absorb(res, 0, time.perf_counter() - t0, raises, state)

    def absorb(self, res, i: int, run_time: float, raises: bool, state=None):
        ok = int(res.status[i]) == _abi.OPTIMAL
        if not ok and raises:
            raise RuntimeError(f"ADMM local MPC for state {state} returned {_abi.STATUS_NAMES.get(int(res.status[i]))}")
        N = self.N
        x = res.x[i].copy() if ok else np.zeros((2, N + 1))
        u = res.u[i].reshape(1, -1).copy() if ok else np.zeros((1, N))
        self.x.X, self.u.X = x, u
        if self.x_front is not None:
            self.x_front.X = res.x_front[i].copy()
        if self.x_back is not None:
            self.x_back.X = res.x_back[i].copy()
        cost = float(res.cost[i]) if ok else float("inf")
        info = {"x": x, "u": u, "cost": cost, "run_time": run_time, "nodes": int(res.nodes[i]),
                "bin_vars": self.num_bin_vars, "status": int(res.status[i])}
        return u[:, [0]], info


class LocalMpcGear(LocalMpcADMM):
    """fleet_naive_admm.py:261-288: LocalMpcADMM's cost and copies on the gear MPC
    (mpcs/mpc_gear.py:30-114): the decision variable is the throttle u_g, bounded by the system's
    F u_g <= G, and every step picks a (gear, friction region) mode.  ``solve_mpc`` returns
    [u_g0; gear0] and info["u"] = vstack(u_g, gears), as MpcGear.solve_mpc does (:116-135)."""

    def __init__(self, N: int, system: dict, rho: float, spacing_policy: SpacingPolicy = ConstantSpacingPolicy(50),
                 quadratic_cost: bool = True, is_front: bool = False, is_leader: bool = False,
                 is_trailer: bool = False, thread_limit: int | None = None,
                 accel_cnstr_tightening: float = 0.0) -> None:
        from .mpc import MpcGear

        super().__init__(N, system, rho, spacing_policy, quadratic_cost, is_front, is_leader, is_trailer,
                         thread_limit, accel_cnstr_tightening)
        self.table = tables.gear_system_from_dict(system)
        MpcGear.setup_gears(self, N, system["F"], system["G"])  # the u_g box on self.table
        self.num_bin_vars = (len(system["S"]) + len(Vehicle.b)) * N
        self.gears_pred = None

    def absorb(self, res, i: int, run_time: float, raises: bool, state=None):
        _, info = super().absorb(res, i, run_time, raises, state)
        ok = info["status"] == _abi.OPTIMAL
        u_g = info["u"]
        gears = res.gear[i].reshape(1, -1).astype(float) if ok else 6 * np.ones((1, self.N))
        info["u"] = np.vstack((u_g, gears))
        self.gears_pred = gears
        return np.vstack((u_g[:, [0]], gears[:, [0]])), info


class AdmmEngine:
    """ADMMCoordinator.get_control for P platoons of n vehicles, entirely on the device."""

    def __init__(self, problem: _abi.HvpProblem, systems: list, sys_idx, roles, n: int, P: int, device: int = 0,
                 leader_index: int = 0, warm_incumbent: bool | None = None) -> None:
        import torch

        self.N = N = int(problem.N)
        self.n, self.P = n, P
        self.B = B = n * P
        self.leader_index = leader_index
        self.solver = BatchSolver(problem, systems, device=device)
        self.solver.reserve(B)
        self.dev = torch.device("cuda", device)
        E = 2 * (N + 1)
        z = lambda *s: torch.zeros(s, dtype=torch.float64, device=self.dev)  # noqa: E731
        self.stride = _abi.params_stride(N, _abi.FORM_ADMM)
        self.params = z(B, self.stride)
        self.y_front, self.y_back = z(B, 2, N + 1), z(B, 2, N + 1)
        self.sys = torch.as_tensor(np.asarray(sys_idx, np.int32).reshape(-1)).to(self.dev)
        self.roles = torch.as_tensor(np.asarray(roles, np.int32).reshape(-1)).to(self.dev)
        self.out = self.solver.alloc_outputs(B, self.dev)
        self.out["x_front"], self.out["x_back"] = z(B, 2, N + 1), z(B, 2, N + 1)
        # every ADMM solve tries the sequence the previous iteration chose (its region output) as
        # a second initial incumbent; -1 = no previous solution yet
        # (default: from N > 8, where the trees are deep enough for the extra leaf QP to pay off)
        self.out["region"].fill_(-1)
        if warm_incumbent if warm_incumbent is not None else N > 8:
            self.solver.set_region_hint(self.out["region"])
        self.z = z(B, 2, N + 1)
        self.x_prev = None  # last step's final local trajectories (warm start)
        self.E = E

    def set_leader(self, leader_x) -> None:
        """leader_x: (2, N+1) shared or (P, 2, N+1) per platoon (set_leader_x, :558-565)."""
        import torch

        lx = torch.as_tensor(np.asarray(leader_x, dtype=np.float64)).to(self.dev).reshape(-1, self.E)
        rows = torch.arange(self.P, device=self.dev) * self.n + self.leader_index
        self.params[rows, 2 + 4 * self.E:] = lx

    def set_leader_device(self, leader_x) -> None:
        """set_leader from a (P, 2, N+1) CUDA tensor (no host round trip)."""
        import torch

        rows = torch.arange(self.P, device=self.dev) * self.n + self.leader_index
        self.params[rows, 2 + 4 * self.E:] = leader_x.reshape(self.P, self.E)

    def step(self, states, admm_iters: int, stream=None, on_solve=None) -> dict:
        """One platoon time step (:379-468): warm start, admm_iters x (local solves + update).
        states: (P, 2n) tensor/array of the measured platoon states.  Returns the output dict of
        the last iteration's local solves (u, x, x_front, x_back, status, ...).  A local search
        that outgrows the workspace (HVP_OVERFLOW, rare) is re-solved alone inside its iteration
        (one host read of the status per iteration)."""
        import torch

        n, E, N = self.n, self.E, self.N
        st = torch.as_tensor(states, dtype=torch.float64).to(self.dev).reshape(self.P * n, 2)
        self.params[:, :2] = st
        # warm start (:392-402): z of the copies <- the neighbours' shifted predictions of the
        # previous step, y keeps its running value (never reset)
        if self.x_prev is not None:
            xp = self.x_prev.reshape(self.P, n, 2, N + 1)
            sh = torch.cat([xp[..., 1:], xp[..., -1:]], dim=-1)
            prm = self.params.reshape(self.P, n, self.stride)
            prm[:, 1:, 2:2 + E] = self.y_front.reshape(self.P, n, E)[:, 1:]
            prm[:, 1:, 2 + E:2 + 2 * E] = sh[:, :-1].reshape(self.P, n - 1, E)
            prm[:, :-1, 2 + 2 * E:2 + 3 * E] = self.y_back.reshape(self.P, n, E)[:, :-1]
            prm[:, :-1, 2 + 3 * E:2 + 4 * E] = sh[:, 1:].reshape(self.P, n - 1, E)
        o = self.out
        stream = stream or torch.cuda.current_stream(self.dev)
        for _ in range(admm_iters):
            self.solver.solve_admm_device(self.sys, self.roles, self.params, o, stream, retry_overflow=True)
            if on_solve is not None:
                on_solve(self.solver)
            self.solver.admm_update(self.P, n, o["x"], o["x_front"], o["x_back"], self.y_front, self.y_back,
                                    self.params, self.z, stream)
        self.x_prev = o["x"].clone()
        return o


class ADMMCoordinator(MldAgent):
    """fleet_naive_admm.py:306-577: fixed-iteration ADMM over the n local MIQPs."""

    def __init__(self, leader_index: int, local_mpcs: list, admm_iters: int, ep_len: int, N: int,
                 leader_x: np.ndarray, ts: float, rho: float) -> None:
        super().__init__(local_mpcs[0])
        self.n = len(local_mpcs)
        self.leader_index = leader_index
        self.agents = [MldAgent(m) for m in local_mpcs]
        self.leader_x = leader_x
        self.nx_l, self.nu_l = Vehicle.nx_l, Vehicle.nu_l
        self.ep_len, self.ts, self.N = ep_len, ts, N
        self.admm_iters = admm_iters
        self.rho = rho
        self.solve_times = np.zeros((ep_len, 1))
        self.node_counts = np.zeros((ep_len, 1))
        self.temp_solve_time = 0.0
        self.temp_node_count = 0
        prob = local_mpcs[0].problem
        for m in local_mpcs[1:]:
            if bytes(m.problem) != bytes(prob):
                raise ValueError("local MPCs must share the controller constants")
        self.engine = AdmmEngine(prob, [m.table for m in local_mpcs], np.arange(self.n), [m.role for m in local_mpcs],
                                 self.n, 1, leader_index=leader_index)

    @property
    def y_front_list(self):
        return list(self.engine.y_front.cpu().numpy())

    @property
    def y_back_list(self):
        return list(self.engine.y_back.cpu().numpy())

    @property
    def z_list(self):
        return list(self.engine.z.cpu().numpy())

    def get_control(self, state, raises: bool = True):
        import torch

        eng = self.engine
        t0 = time.perf_counter()
        o = eng.step(np.asarray(state, dtype=np.float64).reshape(1, -1), self.admm_iters)
        torch.cuda.synchronize(eng.dev)
        dt = time.perf_counter() - t0
        res = {k: v.cpu().numpy() for k, v in o.items()}
        if raises and not (res["status"] == _abi.OPTIMAL).all():
            bad = int(np.flatnonzero(res["status"] != _abi.OPTIMAL)[0])
            raise RuntimeError(f"ADMM local MPC {bad} returned {_abi.STATUS_NAMES.get(int(res['status'][bad]))}")
        u = []
        for i, a in enumerate(self.agents):
            m = a.mpc
            m.x.X, m.u.X = res["x"][i], res["u"][i].reshape(1, -1)
            if m.x_front is not None:
                m.x_front.X = res["x_front"][i]
            if m.x_back is not None:
                m.x_back.X = res["x_back"][i]
            a.record({"x": res["x"][i], "u": res["u"][i].reshape(1, -1), "cost": float(res["cost"][i]),
                      "run_time": dt / self.admm_iters, "nodes": int(res["nodes"][i]), "bin_vars": m.num_bin_vars})
            if isinstance(m, LocalMpcGear):
                m.gears_pred = res["gear"][i].reshape(1, -1).astype(float)
                u.append(np.array([[res["u"][i][0]], [m.gears_pred[0, 0]]]))
            else:
                u.append(res["u"][i][:1].reshape(1, 1))
        # solve-time bookkeeping (:470-477): per iteration the slowest agent; the n agents of an
        # iteration run in one batched launch
        self.temp_solve_time += dt
        self.temp_node_count = max(self.temp_node_count, int(res["nodes"].max()))
        if u[0].shape[0] > self.nu_l:  # gear MPCs: continuous controls first, then the gears (:557-566)
            return np.vstack([np.vstack([a[:self.nu_l] for a in u]), np.vstack([a[self.nu_l:] for a in u])]), {}
        return np.vstack(u), {}

    def on_timestep_end(self, env, episode: int, timestep: int) -> None:
        self.engine.set_leader(self.leader_x[:, timestep:timestep + self.N + 1])
        self.solve_times[env.step_counter - 1, :] = self.temp_solve_time
        self.node_counts[env.step_counter - 1, :] = self.temp_node_count
        self.temp_solve_time = 0.0
        self.temp_node_count = 0

    def on_episode_start(self, env, episode: int, state) -> None:
        self.engine.set_leader(self.leader_x[:, 0:self.N + 1])


def simulate(sim: Sim, admm_iters: int = 20, save: bool = False, plot: bool = False, seed: int = 1,
             thread_limit: int | None = None, leader_index: int = 0, verbose: bool = False):
    """Closed-loop run of the naive-ADMM controller (fleet_naive_admm.py:580-692)."""
    n, N, ep_len, ts = sim.n, sim.N, sim.ep_len, Params.ts
    leader_x = sim.leader_trajectory.get_leader_trajectory()
    if sim.vehicle_model_type not in ("pwa_gear", "pwa_friction"):  # :630-637
        raise NotImplementedError("the GPU ADMM path implements the pwa_gear (LocalMpcADMM) and pwa_friction "
                                  "(LocalMpcGear) models; the nonlinear model is out of scope (DESIGN.md)")
    platoon = Platoon(n, vehicle_type=sim.vehicle_model_type, masses=sim.masses)
    systems = platoon.get_vehicle_system_dicts(ts)
    env = EpisodeMonitor(
        PlatoonEnv(n=n, platoon=platoon, leader_trajectory=sim.leader_trajectory, spacing_policy=sim.spacing_policy,
                   start_from_platoon=sim.start_from_platoon, real_vehicle_as_reference=sim.real_vehicle_as_reference,
                   ep_len=ep_len, leader_index=leader_index, verbose=verbose),
        max_episode_steps=ep_len,
    )
    vehicles = platoon.get_vehicles()
    def local(i):
        kw = dict(rho=0.5, spacing_policy=sim.spacing_policy, is_front=i == 0, is_leader=i == leader_index,
                  is_trailer=i == n - 1, thread_limit=thread_limit)
        if sim.vehicle_model_type == "pwa_friction":
            return LocalMpcGear(N, systems[i], **kw)
        return LocalMpcADMM(N, systems[i], gears=tables.gears_of(vehicles[i]), **kw)

    mpcs = [local(i) for i in range(n)]
    agent = ADMMCoordinator(leader_index=leader_index, local_mpcs=mpcs, admm_iters=admm_iters, rho=0.5,
                            ep_len=ep_len, N=N, leader_x=leader_x, ts=ts)
    agent.evaluate(env=env, episodes=1, seed=seed)
    X = env.observations[0].squeeze()
    U = env.actions[0].squeeze()
    R = env.rewards[0]
    if save:
        with open(f"admm_{admm_iters}_{sim.id}_seed_{seed}.pkl", "wb") as f:
            for obj in (X, U, R, agent.solve_times, agent.node_counts, env.unwrapped.viol_counter[0], leader_x):
                pickle.dump(obj, f)
    return X, U, R, agent, env
