"""Drop-in counterparts of the reference's local MPC objects, backed by libhvpsolve.so.

* :class:`MpcMld`       <- dmpcpwa ``MpcMld`` [EXT] as used by the reference:
                           ``__init__(system, N, thread_limit, constrain_first_state)``,
                           ``solve_mpc(state, raises) -> (u0, info)`` (called via
                           ``MldAgent.get_control``, fleet_decent_mld.py:316).
* :class:`LocalMpcMld`  <- fleet_decent_mld.py:21-223: the decentralised local MPC with its
                           cost / constraints (``setup_cost_and_constraints`` :61-208) and the
                           parameter setters ``set_leader_x / set_x_front / set_x_back``
                           (:210-223).

The Gurobi model the reference builds once is replaced by an ``hvp_problem`` + per-vehicle
``hvp_system`` table and a role bit-set; the setters write the instance parameter block that
``hvp_solve_batch`` reads.  ``info`` carries the reference's keys: ``x`` (2, N+1), ``u`` (1, N),
``cost``, ``run_time`` (s), ``nodes`` (region sequences solved: the node count analogue) and
``bin_vars`` (7N, the MLD binaries).
"""

from __future__ import annotations

import time

import numpy as np

from . import _abi, tables
from .params import ConstantSpacingPolicy, Params, SpacingPolicy
from .solver import BatchSolver

_SOLVERS: dict = {}


def _problem_key(p: _abi.HvpProblem) -> bytes:
    return bytes(p)


def shared_solver(problem: _abi.HvpProblem, systems: list[_abi.HvpSystem]) -> BatchSolver:
    """One handle per (problem constants, vehicle tables), reused by every MPC that shares them."""
    key = (_problem_key(problem), tuple(bytes(s) for s in systems))
    s = _SOLVERS.get(key)
    if s is None:
        s = BatchSolver(problem, systems)
        _SOLVERS[key] = s
    return s


class MpcMld:
    """PWA -> MLD hybrid MPC of one velocity-partitioned vehicle model (GPU solve)."""

    Q_x = Params.Q_x
    Q_u = Params.Q_u
    Q_du = Params.Q_du
    w = Params.w
    a_acc = Params.a_acc
    a_dec = Params.a_dec
    ts = Params.ts
    d_safe = Params.d_safe

    def __init__(self, system: dict, N: int, thread_limit: int | None = None, constrain_first_state: bool = True,
                 gears=None) -> None:
        if constrain_first_state:
            # the reference's platoon MPCs all pass constrain_first_state=False (fleet_decent_mld.py:47)
            raise NotImplementedError("only constrain_first_state=False (the platoon formulation) is supported")
        self.system = system
        self.N = N
        self.thread_limit = thread_limit  # no CPU thread pool: kept for signature compatibility
        self.n = 2
        self.m = 1
        self.table = tables.system_from_dict(system, gears)
        self.num_bin_vars = len(system["S"]) * N
        K = 2 * (N + 1)
        self._params = np.zeros(_abi.params_stride(N))
        self._K = K
        self.role = 0
        self.problem: _abi.HvpProblem | None = None
        self.x_pred: np.ndarray | None = None
        self.u_pred: np.ndarray | None = None
        self.cost_pred: float | None = None
        self.regions_pred: np.ndarray | None = None
        self.gears_pred: np.ndarray | None = None

    # ------------------------------------------------------------ parameter blocks
    def _block(self, which: int) -> slice:
        return slice(2 + which * self._K, 2 + (which + 1) * self._K)

    def _set(self, which: int, traj) -> None:
        a = np.asarray(traj, dtype=np.float64)
        if a.shape != (2, self.N + 1):
            raise ValueError(f"expected a (2, {self.N + 1}) trajectory, got {a.shape}")
        self._params[self._block(which)] = a.reshape(-1)

    def params_for(self, state) -> np.ndarray:
        p = self._params.copy()
        p[:2] = np.asarray(state, dtype=np.float64).reshape(-1)[:2]
        return p

    # ------------------------------------------------------------ solve
    def _solver(self) -> BatchSolver:
        if self.problem is None:
            raise RuntimeError("cost and constraints not set up")
        return shared_solver(self.problem, [self.table])

    def solve_mpc(self, state, raises: bool = True):
        t0 = time.perf_counter()
        res = self._solver().solve(np.zeros(1, np.int32), np.array([self.role], np.int32), self.params_for(state)[None])
        return self.absorb(res, 0, time.perf_counter() - t0, raises, state)

    def absorb(self, res, i: int, run_time: float, raises: bool, state=None):
        """Store solution i of a batch result the way solve_mpc returns it."""
        ok = int(res.status[i]) == _abi.OPTIMAL
        if not ok:
            if raises:
                raise RuntimeError(f"MPC for state {state} returned {_abi.STATUS_NAMES.get(int(res.status[i]))}")
            x = np.zeros((2, self.N + 1))
            u = np.zeros((1, self.N))
            cost = float("inf")
        else:
            x = res.x[i].copy()
            u = res.u[i].reshape(1, -1).copy()
            cost = float(res.cost[i])
        self.x_pred, self.u_pred, self.cost_pred = x, u, cost
        self.regions_pred = res.region[i].copy()
        self.gears_pred = res.gear[i].reshape(1, -1).astype(float)
        info = {"x": x, "u": u, "cost": cost, "run_time": run_time, "nodes": int(res.nodes[i]),
                "bin_vars": self.num_bin_vars, "status": int(res.status[i])}
        return u[:, [0]], info


class LocalMpcMld(MpcMld):
    """Local decentralised MPC of one vehicle in the platoon (fleet_decent_mld.py:21-223)."""

    def __init__(
        self,
        N: int,
        pwa_system: dict,
        spacing_policy: SpacingPolicy = ConstantSpacingPolicy(50),
        quadratic_cost: bool = True,
        is_front: bool = False,
        is_leader: bool = False,
        is_trailer: bool = False,
        thread_limit: int | None = None,
        accel_cnstr_tightening: float = 0.0,
        real_vehicle_as_reference: bool = False,
        gears=None,
    ) -> None:
        super().__init__(pwa_system, N, thread_limit=thread_limit, constrain_first_state=False, gears=gears)
        self.setup_cost_and_constraints(None, spacing_policy, quadratic_cost, is_front, is_leader, is_trailer,
                                        accel_cnstr_tightening, real_vehicle_as_reference)

    def setup_cost_and_constraints(self, u, spacing_policy=ConstantSpacingPolicy(50), quadratic_cost: bool = True,
                                   is_front: bool = False, is_leader=False, is_trailer=False,
                                   accel_cnstr_tightening: float = 0.0, real_vehicle_as_reference: bool = False):
        if not quadratic_cost:
            raise NotImplementedError("the GPU path implements the quadratic cost (min_2_norm) only")
        self.is_front, self.is_leader, self.is_trailer = is_front, is_leader, is_trailer
        self.spacing_policy = spacing_policy
        self.role = tables.role_bits(is_front, is_trailer, is_leader, real_vehicle_as_reference)
        self.problem = tables.problem(self.N, spacing_policy, quadratic_cost, accel_cnstr_tightening,
                                      params=type(self))

    def set_leader_x(self, leader_x) -> None:
        self._set(2, leader_x)

    def set_x_front(self, x_front) -> None:
        self._set(0, x_front)

    def set_x_back(self, x_back) -> None:
        self._set(1, x_back)
