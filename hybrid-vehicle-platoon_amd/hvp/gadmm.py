"""Switching-ADMM platoon controller (fleet_g_admm.py) on the GPU.

* :class:`LocalMpc` <- fleet_g_admm.py:22-205: the local convex QP of one vehicle for a given
  switching sequence (MpcSwitching [EXT]) with its own state and its neighbour copies in the
  augmented Lagrangian (MpcAdmm [EXT]); GPU-backed through ``hvp_gadmm_solve``.
* :class:`GAdmmEngine` -- the batched device form of ``TrackingGAdmmCoordinator.g_admm_control``
  (:255-301 over GAdmmCoordinator [EXT]) for P platoons: per warm start one rollout launch, then
  rounds of ``admm_iters`` x (local-QP launch + consensus launch) and one switching launch per
  round; the host synchronises once per round (are any platoons still switching?).
* Vehicle sharding: a process may hold only the vehicles [lo, lo + m) of
  every platoon.  After every local-QP launch a :class:`HaloExchange` swaps the boundary
  vehicles' trajectories / copies with the neighbouring ranks (RCCL point-to-point over xGMI:
  the chain couples rank r only to r - 1 and r + 1), before the consensus launch.
* :class:`TrackingGAdmmCoordinator` <- :208-301 and :func:`simulate` <- :304-439, the reference's
  agent surface on top of the engine (one platoon).

The switching rule of dmpcpwa's GAdmmCoordinator cannot be inspected here (not installed); the
rule restated and implemented on both sides (here and in oracle/oracle.py GAdmmCoordinator)
is documented in DESIGN.md "Switching ADMM": after each ADMM run every vehicle moves the region
of step k across a velocity edge of its region whose row is active with a positive multiplier,
and the run repeats until no sequence changes (at most ``max_rounds``).
"""

from __future__ import annotations

import contextlib
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

RHO = 0.5  # LocalMpc.rho (fleet_g_admm.py:33)


def gadmm_problem(N: int, rho: float = RHO, spacing_policy: SpacingPolicy | None = None,
                  params=Params) -> _abi.HvpProblem:
    """hvp_problem of fleet_g_admm.LocalMpc: Params' weights, accel rows without tightening."""
    p = tables.problem(N, spacing_policy, True, 0.0, params=params, method=_abi.METHOD_BNB)
    p.formulation = _abi.FORM_GADMM
    p.rho = float(rho)
    return p


def gadmm_role(i: int, n: int) -> int:
    """Role of vehicle i of the chain (fleet_g_admm.py:341-389): vehicle 0 leads (x_ref
    tracking, :112-135), the others track and keep their distance to the front copy (:98-109,
    :136-158); every vehicle but the last holds a copy of the one behind (G[i] contains i + 1)."""
    r = _abi.ROLE_TRACK_LEADER if i == 0 else (_abi.ROLE_SAFE_FRONT | _abi.ROLE_TRACK_FRONT)
    if i < n - 1:
        r |= _abi.ROLE_BACK_COPY
    return r


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of vehicles of `rank` (the first n % world ranks get one more)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, base + (1 if rank < extra else 0)


class HaloExchange:
    """Boundary exchange of the vehicle-sharded switching ADMM (one call per ADMM iteration).

    The consensus step of vehicle i reads z_{i-1}, z_i, z_{i+1}, i.e. the trajectories x of
    i-1..i+1, the back copies of i-2..i-1 and the front copies of i+1..i+2.  For the block
    [lo, hi) that is, from the left neighbour: x_{lo-1}, xb_{lo-1}, xb_{lo-2}; from the right:
    x_hi, xf_hi, xf_{hi+1} -- 3 (P, 2, N+1) blocks per side, sent as one buffer with RCCL
    send / recv (``torch.distributed.batch_isend_irecv``).  Needs m >= 2 on every rank."""

    def __init__(self, P: int, n: int, N: int, rank: int, world: int, group=None) -> None:
        self.P, self.n, self.N, self.rank, self.world, self.group = P, n, N, rank, world, group
        self.lo, self.m = shard_range(n, rank, world)
        if world > 1 and n < 2 * world:
            raise ValueError(f"vehicle sharding needs >= 2 vehicles per rank (n={n}, world={world})")
        self.hi = self.lo + self.m
        self.bytes_per_call = 0

    def _idx(self, dev, vehicles):
        import torch

        v = torch.as_tensor(vehicles, dtype=torch.long, device=dev)
        return (torch.arange(self.P, device=dev, dtype=torch.long)[:, None] * self.n + v[None, :]).reshape(-1)

    def __call__(self, x, xf, xb) -> None:
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return
        dev = x.device
        P, E = self.P, 2 * (self.N + 1)
        flat = [t.view(P * self.n, E) for t in (x, xf, xb)]
        ops, recv = [], {}
        lo, hi = self.lo, self.hi
        if self.rank > 0:  # to / from the left neighbour
            send = torch.cat([flat[0][self._idx(dev, [lo])], flat[1][self._idx(dev, [lo])],
                              flat[1][self._idx(dev, [lo + 1])]])
            recv["left"] = torch.empty_like(send)
            ops += [dist.P2POp(dist.isend, send.contiguous(), self.rank - 1, self.group),
                    dist.P2POp(dist.irecv, recv["left"], self.rank - 1, self.group)]
            self.bytes_per_call = send.numel() * 8
        if self.rank < self.world - 1:  # to / from the right neighbour
            send = torch.cat([flat[0][self._idx(dev, [hi - 1])], flat[2][self._idx(dev, [hi - 1])],
                              flat[2][self._idx(dev, [hi - 2])]])
            recv["right"] = torch.empty_like(send)
            ops += [dist.P2POp(dist.isend, send.contiguous(), self.rank + 1, self.group),
                    dist.P2POp(dist.irecv, recv["right"], self.rank + 1, self.group)]
            self.bytes_per_call = send.numel() * 8
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        if "left" in recv:  # x_{lo-1}, xb_{lo-1}, xb_{lo-2}
            a, b, c = recv["left"].view(3, P, E)
            flat[0][self._idx(dev, [lo - 1])] = a
            flat[2][self._idx(dev, [lo - 1])] = b
            if lo >= 2:
                flat[2][self._idx(dev, [lo - 2])] = c
        if "right" in recv:  # x_hi, xf_hi, xf_{hi+1}
            a, b, c = recv["right"].view(3, P, E)
            flat[0][self._idx(dev, [hi])] = a
            flat[1][self._idx(dev, [hi])] = b
            if hi + 1 < self.n:
                flat[1][self._idx(dev, [hi + 1])] = c

    def reduce_flags(self, state) -> None:
        """Round end: failures and sequence changes of a platoon on any rank apply everywhere."""
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return
        f = torch.stack([(state & _abi.GADMM_FAILED) != 0, (state & _abi.GADMM_CHANGED) != 0]).to(torch.int32)
        dist.all_reduce(f, op=dist.ReduceOp.MAX, group=self.group)
        state |= f[0] * _abi.GADMM_FAILED + f[1] * _abi.GADMM_CHANGED
        state &= ~(f[0] * _abi.GADMM_LIVE)

    def reduce_cost(self, cost) -> None:
        import torch.distributed as dist

        if self.world > 1:
            dist.all_reduce(cost, op=dist.ReduceOp.SUM, group=self.group)


class GAdmmEngine:
    """TrackingGAdmmCoordinator.g_admm_control for P platoons of n vehicles on the device.

    systems: the n vehicles' hvp_system tables (vehicle i uses systems[i]); a sharded engine
    holds the vehicles [lo, lo + m) (``exchange`` is its :class:`HaloExchange`)."""

    def __init__(self, problem: _abi.HvpProblem, systems: list, n: int, P: int, device: int = 0,
                 admm_iters: int = 100, max_rounds: int = 10, exchange: HaloExchange | None = None) -> None:
        import torch

        if problem.formulation != _abi.FORM_GADMM:
            raise ValueError("GAdmmEngine needs an HVP_FORM_GADMM problem (gadmm_problem)")
        self.N = N = int(problem.N)
        self.n, self.P = n, P
        self.exchange = exchange
        self.lo, self.m = (exchange.lo, exchange.m) if exchange is not None else (0, n)
        self.B = B = P * self.m
        self.admm_iters, self.max_rounds = admm_iters, max_rounds
        self.solver = BatchSolver(problem, systems, device=device)
        self._lib, self._h = self.solver._lib, self.solver._h
        self.dev = torch.device("cuda", device)
        E = 2 * (N + 1)
        self.E = E
        f64 = dict(dtype=torch.float64, device=self.dev)
        veh = np.arange(self.lo, self.lo + self.m)
        self.sys = torch.as_tensor(np.tile(veh, P).astype(np.int32), device=self.dev)
        self.roles = torch.as_tensor(np.tile([gadmm_role(int(i), n) for i in veh], P).astype(np.int32),
                                     device=self.dev)
        self.stride = _abi.params_stride(N, _abi.FORM_GADMM)
        self.params = torch.zeros((B, self.stride), **f64)
        self.seq = torch.zeros((B, N), dtype=torch.int8, device=self.dev)
        self.state = torch.zeros(P, dtype=torch.int32, device=self.dev)
        self.x = torch.zeros((P * n, 2, N + 1), **f64)
        self.xf = torch.zeros_like(self.x)
        self.xb = torch.zeros_like(self.x)
        self.u = torch.zeros((B, N), **f64)
        self.u_ws = torch.zeros((B, N), **f64)
        self.cost = torch.zeros(B, **f64)
        self.status = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.edge = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.iters = torch.zeros(B, dtype=torch.int32, device=self.dev)
        self.prev_u = None  # (B, N): last successful warm start's controls
        self.last = {}

    # ------------------------------------------------------------------ C ABI calls
    def _p(self, t):
        return ctypes.c_void_p(t.data_ptr() if t is not None else 0)

    def _stream(self, stream):
        import torch

        return ctypes.c_void_p((stream or torch.cuda.current_stream(self.dev)).cuda_stream)

    def rollout(self, mode: int, stream=None) -> None:
        p = self._p
        _abi.check(self._lib.hvp_gadmm_rollout(self._h, self.P, self.n, self.lo, self.m, p(self.sys), p(self.params),
                                               int(mode), p(self.prev_u), p(self.x), p(self.seq), p(self.u_ws),
                                               p(self.state), self._stream(stream)), "hvp_gadmm_rollout")

    def solve(self, stream=None) -> None:
        p = self._p
        _abi.check(self._lib.hvp_gadmm_solve(self._h, self.P, self.n, self.lo, self.m, p(self.sys), p(self.roles),
                                             p(self.params), p(self.seq), p(self.state), p(self.u), p(self.x),
                                             p(self.xf), p(self.xb), p(self.cost), p(self.status), p(self.edge),
                                             p(self.iters), self._stream(stream)), "hvp_gadmm_solve")

    def update(self, init: bool = False, stream=None) -> None:
        p = self._p
        _abi.check(self._lib.hvp_gadmm_update(self._h, self.P, self.n, self.lo, self.m, p(self.x), p(self.xf),
                                              p(self.xb), p(self.params), p(self.state), int(init),
                                              self._stream(stream)), "hvp_gadmm_update")

    def switch(self, stream=None) -> None:
        p = self._p
        _abi.check(self._lib.hvp_gadmm_switch(self._h, self.P, self.n, self.lo, self.m, p(self.sys), p(self.edge),
                                              p(self.seq), p(self.state), self._stream(stream)), "hvp_gadmm_switch")

    # ------------------------------------------------------------------ coordinator
    def set_leader(self, leader_x) -> None:
        """x_ref_k parameters of the leader (TrackingGAdmmCoordinator.set_leader_traj, :251-253):
        (2, N+1) shared or (P, 2, N+1) per platoon."""
        import torch

        if self.lo != 0:
            return  # the leader (vehicle 0) is held by another rank
        lx = torch.as_tensor(np.asarray(leader_x, dtype=np.float64), device=self.dev).reshape(-1, self.E)
        rows = torch.arange(self.P, device=self.dev) * self.m
        self.params[rows, 2 + 4 * self.E:2 + 5 * self.E] = lx

    def _exchange(self) -> None:
        if self.exchange is not None:
            self.exchange(self.x, self.xf, self.xb)

    def _on(self, stream):
        """Make `stream` torch's current stream for the duration: the halo exchange, the flag
        reductions and the torch ops between launches then run in launch order with the kernels
        (a caller stream other than the current one would otherwise race with them)."""
        import torch

        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    def run(self, mode: int, stream=None) -> dict:
        """One GAdmmCoordinator.g_admm_control(state, warm_start) for every platoon: returns
        cost (P,) (inf where the run failed), rounds and QP launches."""
        with self._on(stream):
            return self._run(mode, None)

    def _run(self, mode: int, stream=None) -> dict:
        import torch

        st = self.state
        st.fill_(_abi.GADMM_LIVE)
        self.rollout(mode, stream)
        if self.exchange is not None:
            self.exchange.reduce_flags(st)
        self._exchange()
        self.update(init=True, stream=stream)
        rounds = launches = 0
        per_platoon = torch.zeros(self.P, dtype=torch.int32, device=self.dev)
        for rounds in range(1, self.max_rounds + 1):
            per_platoon += ((st & _abi.GADMM_LIVE) != 0).to(torch.int32)
            for _ in range(self.admm_iters):
                self.solve(stream)
                self._exchange()
                self.update(stream=stream)
                launches += 1
            st &= ~_abi.GADMM_CHANGED
            self.switch(stream)
            if self.exchange is not None:
                self.exchange.reduce_flags(st)
            # platoons whose sequences did not change are done
            st &= ~(((st & _abi.GADMM_CHANGED) == 0).to(torch.int32) * _abi.GADMM_LIVE)
            if not bool(((st & _abi.GADMM_LIVE) != 0).any()):  # one host sync per round
                break
        failed = (st & _abi.GADMM_FAILED) != 0
        cost = self.cost.view(self.P, self.m).sum(dim=1)
        if self.exchange is not None:
            self.exchange.reduce_cost(cost)
        cost = torch.where(failed, torch.full_like(cost, float("inf")), cost)
        return {"cost": cost, "failed": failed, "rounds": rounds, "launches": launches, "platoon_rounds": per_platoon,
                "seq": self.seq.clone(), "u": self.u.clone()}

    def control(self, states, stream=None) -> dict:
        """TrackingGAdmmCoordinator.g_admm_control (:255-301) for every platoon.  states: (P, 2n)
        measured platoon states.  Returns u (B, N) of the best warm start, its cost (P,) (inf:
        no warm start succeeded -> the reference raises) and per-run details."""
        with self._on(stream):
            return self._control(states)

    def _control(self, states, stream=None) -> dict:
        import torch

        st = torch.as_tensor(states, dtype=torch.float64).to(self.dev).reshape(self.P, self.n, 2)
        self.params[:, :2] = st[:, self.lo:self.lo + self.m].reshape(self.B, 2)
        best_cost = torch.full((self.P,), float("inf"), dtype=torch.float64, device=self.dev)
        best_u = torch.zeros_like(self.u)
        best_ws = torch.zeros(self.P, dtype=torch.int32, device=self.dev)
        runs = []
        modes = [0] if self.prev_u is None else [0, 1]
        new_prev = self.prev_u.clone() if self.prev_u is not None else torch.zeros_like(self.u)
        for w, mode in enumerate(modes):
            r = self._run(mode, stream)
            runs.append(r)
            okB = (~r["failed"]).repeat_interleave(self.m)[:, None]
            better = r["cost"] < best_cost  # ties keep the earlier warm start (:290)
            best_cost = torch.where(better, r["cost"], best_cost)
            best_u = torch.where(better.repeat_interleave(self.m)[:, None], self.u, best_u)
            best_ws = torch.where(better, torch.full_like(best_ws, w + 1), best_ws)
            new_prev = torch.where(okB, self.u, new_prev)
        self.prev_u = new_prev
        self.last = {"u": best_u, "cost": best_cost, "warm_start": best_ws, "runs": runs}
        return self.last


class LocalMpc:
    """fleet_g_admm.LocalMpc (:22-205): the local problem's constants of one vehicle."""

    Q_x = Params.Q_x
    Q_u = Params.Q_u
    Q_du = Params.Q_du
    w = Params.w
    a_acc = Params.a_acc
    a_dec = Params.a_dec
    ts = Params.ts
    d_safe = Params.d_safe
    rho = RHO

    def __init__(self, N: int, pwa_system: dict, num_neighbours: int, my_index: int,
                 spacing_policy: SpacingPolicy = ConstantSpacingPolicy(50), leader: bool = False,
                 gears=None) -> None:
        self.horizon = self.N = N
        self.system = pwa_system
        self.num_neighbours, self.my_index, self.leader = num_neighbours, my_index, leader
        self.table = tables.system_from_dict(pwa_system, gears)
        self.problem = gadmm_problem(N, self.rho, spacing_policy, params=type(self))
        self.fixed_pars_init = {f"x_ref_{k}": np.zeros((2, 1)) for k in range(N + 1)} if leader else {}


class TrackingGAdmmCoordinator(MldAgent):
    """fleet_g_admm.py:208-301 over the device engine (one platoon; vehicle 0 is the leader)."""

    def __init__(self, N: int, ep_len: int, leader_x: np.ndarray, local_mpcs: list, local_fixed_parameters: list,
                 systems: list, vehicles: list, G: list, Adj: np.ndarray, rho: float, debug_plot: bool = False,
                 admm_iters: int = 50, max_rounds: int = 10) -> None:
        super().__init__(local_mpcs[0])
        self.N, self.ep_len, self.leader_x, self.vehicles = N, ep_len, leader_x, vehicles
        self.n = len(local_mpcs)
        self.nu_l = Vehicle.nu_l
        self.G, self.Adj, self.rho = G, Adj, rho
        self.admm_iters = admm_iters
        self.agents = [MldAgent(m) for m in local_mpcs]
        for i, g in enumerate(G):  # the engine implements the chain coupling of simulate (:341-353)
            if sorted(g) != [j for j in (i - 1, i, i + 1) if 0 <= j < self.n]:
                raise NotImplementedError("the device switching ADMM implements the chain coupling graph")
        self.best_warm_starts: list[int] = []
        self.solve_times: list[float] = []
        self.prev_sol = None
        self.prev_sol_time = 0.0
        prob = local_mpcs[0].problem
        self.engine = GAdmmEngine(prob, [m.table for m in local_mpcs], self.n, 1, admm_iters=admm_iters,
                                  max_rounds=max_rounds)

    def set_leader_traj(self, leader_traj) -> None:
        self.engine.set_leader(np.asarray(leader_traj, dtype=np.float64).reshape(2, self.N + 1))

    def on_timestep_end(self, env, episode: int, timestep: int) -> None:
        self.set_leader_traj(self.leader_x[:, timestep:timestep + self.N + 1])

    def on_episode_start(self, env, episode: int, state) -> None:
        self.set_leader_traj(self.leader_x[:, 0:self.N + 1])

    def g_admm_control(self, state, warm_start=None):
        import torch

        t0 = time.perf_counter()
        out = self.engine.control(np.asarray(state, dtype=np.float64).reshape(1, -1))
        torch.cuda.synchronize(self.engine.dev)
        self.prev_sol_time = time.perf_counter() - t0
        cost = float(out["cost"][0])
        if not np.isfinite(cost):
            self.solve_times.append(0.0)
            raise RuntimeError("No solution found for any of the warm starts")
        self.best_warm_starts.append(int(out["warm_start"][0]))
        self.solve_times.append(self.prev_sol_time)
        u = out["u"].cpu().numpy().reshape(self.n, self.N)
        self.prev_sol = [u[i:i + 1] for i in range(self.n)]
        return u, None, None, None

    def get_control(self, state, raises: bool = True):
        u, *_ = self.g_admm_control(state)
        return u[:, [0]], {}


def simulate(sim: Sim, save: bool = False, plot: bool = False, seed: int = 1, admm_iters: int = 100,
             max_rounds: int = 10, verbose: bool = False):
    """Closed-loop run of the switching-ADMM controller (fleet_g_admm.py:304-439)."""
    n, N, ep_len, ts = sim.n, sim.N, sim.ep_len, Params.ts
    if sim.vehicle_model_type != "pwa_gear":
        raise NotImplementedError()  # as the reference (:368-375)
    leader_x = sim.leader_trajectory.get_leader_trajectory()
    platoon = Platoon(n, vehicle_type=sim.vehicle_model_type, masses=sim.masses)
    systems = platoon.get_vehicle_system_dicts(ts)
    env = EpisodeMonitor(
        PlatoonEnv(n=n, platoon=platoon, leader_trajectory=sim.leader_trajectory, spacing_policy=sim.spacing_policy,
                   start_from_platoon=sim.start_from_platoon, ep_len=ep_len, verbose=verbose),
        max_episode_steps=ep_len,
    )
    G = [sorted(j for j in (i - 1, i, i + 1) if 0 <= j < n) for i in range(n)]
    Adj = np.zeros((n, n))
    for i in range(n):
        for j in G[i]:
            if j != i:
                Adj[i, j] = 1
    vehicles = platoon.get_vehicles()
    mpcs = [LocalMpc(N, systems[i], num_neighbours=len(G[i]) - 1, my_index=G[i].index(i),
                     spacing_policy=sim.spacing_policy, leader=i == 0, gears=tables.gears_of(vehicles[i]))
            for i in range(n)]
    agent = TrackingGAdmmCoordinator(N=N, ep_len=ep_len, leader_x=leader_x, local_mpcs=mpcs,
                                     local_fixed_parameters=[m.fixed_pars_init for m in mpcs], systems=systems,
                                     vehicles=vehicles, G=G, Adj=Adj, rho=LocalMpc.rho, admm_iters=admm_iters,
                                     max_rounds=max_rounds)
    agent.evaluate(env=env, episodes=1, seed=seed)
    X = env.observations[0].squeeze()
    U = env.actions[0].squeeze()
    R = env.rewards[0]
    if save:
        with open(f"switching_admm_{sim.id}_seed_{seed}.pkl", "wb") as f:
            for obj in (X, U, R, agent.solve_times, 0, env.unwrapped.viol_counter[0], leader_x):
                pickle.dump(obj, f)
    return X, U, R, agent, env
