"""Drop-in counterparts of the reference's local MPC objects, backed by libhvpsolve.so.

* :class:`MpcMld`       <- dmpcpwa ``MpcMld`` [EXT] as used by the reference:
                           ``__init__(system, N, thread_limit, constrain_first_state)``,
                           ``solve_mpc(state, raises) -> (u0, info)`` (called via
                           ``MldAgent.get_control``, fleet_decent_mld.py:316).
* :class:`MpcGear`      <- mpcs/mpc_gear.py:8-170: MLD MPC with discrete gears scaling the
                           throttle (``setup_gears``, ``solve_mpc -> [u_g0; gear0]``,
                           ``evaluate_cost``); :class:`LocalMpcGear` <- fleet_decent_mld.py:226-253.
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
        # quadratic_cost=False (min_1_norm, fleet_decent_mld.py:73-76): the local MILP by the
        # fixed-sequence LPs of csrc/hvp_l1.h, exhaustive enumeration up to N = 8 and branch and
        # bound over node LPs beyond (any horizon up to HVP_MAX_N)
        self.quadratic_cost = quadratic_cost
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


class MpcGear(MpcMld):
    """MLD MPC whose input is a throttle u_g scaled by a discrete gear (mpcs/mpc_gear.py:8-170).

    The reference adds gear binaries sigma (6 per step) with u = sum_j sigma_j b_j u_g and the
    gear's velocity window to the PWA model's region binaries; the GPU table enumerates the
    (gear, region) modes instead (:func:`hvp.tables.gear_system_from_dict`), so one mode choice
    per step carries both binary families and the same search / tie rule applies."""

    def __init__(self, system: dict, N: int, thread_limit: int | None = None,
                 constrain_first_state: bool = False) -> None:
        MpcMld.__init__(self, system, N, thread_limit=thread_limit, constrain_first_state=constrain_first_state)
        from .models import Vehicle

        self.table = tables.gear_system_from_dict(system)
        # delta (PWA regions) + sigma (gears) per step, as built by MpcMld + setup_gears
        self.num_bin_vars = (len(system["S"]) + len(Vehicle.b)) * N
        self.gears_ready = False

    def setup_gears(self, N: int, F, G) -> None:
        """mpcs/mpc_gear.py:30-114.  The control box F u_g <= G replaces F u <= G (:57-76)."""
        F = np.asarray(F, dtype=float).reshape(-1)
        G = np.asarray(G, dtype=float).reshape(-1)
        lo, hi = -np.inf, np.inf
        for f, g in zip(F, G):
            if f > 0:
                hi = min(hi, g / f)
            elif f < 0:
                lo = max(lo, g / f)
        self.table.umin, self.table.umax = lo, hi
        self.gears_ready = True

    def solve_mpc(self, state, raises: bool = True):
        """[u_g0; gear0] and info with info["u"] = vstack(u_g, gears) (mpc_gear.py:116-135)."""
        if not self.gears_ready:
            raise RuntimeError("setup_gears not called")
        t0 = time.perf_counter()
        res = self._solver().solve(np.zeros(1, np.int32), np.array([self.role], np.int32), self.params_for(state)[None])
        return self.absorb(res, 0, time.perf_counter() - t0, raises, state)

    def absorb(self, res, i: int, run_time: float, raises: bool, state=None):
        """Solution i of a batch result as MpcGear.solve_mpc returns it."""
        ok = int(res.status[i]) == _abi.OPTIMAL
        if not ok and raises:
            raise RuntimeWarning(f"gear mpc for state {state} is infeasible.")
        _, info = MpcMld.absorb(self, res, i, run_time, False, state)
        if ok:
            u_g = res.u[i].reshape(1, -1).copy()
            gears = res.gear[i].reshape(1, -1).astype(float)
        else:
            u_g = np.zeros((1, self.N))
            gears = 6 * np.ones((1, self.N))  # default: all gears 6 (:129-131)
        info["u"] = np.vstack((u_g, gears))
        self.gears_pred = gears
        return np.vstack((u_g[:, [0]], gears[:, [0]])), info

    def evaluate_cost(self, x0, u, j=None):
        """Cost of the fixed throttle u (1, N) and gears j (1, N) from x0 (mpc_gear.py:137-170);
        the string 'inf' when infeasible, as the reference returns.  j=None: the gears of the
        last solution (the reference leaves them free; its only use fixes them)."""
        u = np.asarray(u, dtype=float)
        if u.shape != (1, self.N):
            raise ValueError(f"Expected u shape {(1, self.N)}. Got {u.shape}.")
        if j is None:
            if self.gears_pred is None:
                raise ValueError("no gears given and no previous solution")
            j = self.gears_pred
        j = np.asarray(j).reshape(1, self.N).astype(np.int8)
        out = self._solver().evaluate(np.zeros(1, np.int32), np.array([self.role], np.int32),
                                      self.params_for(x0)[None], j, u)
        return float(out["cost"][0]) if int(out["status"][0]) == _abi.OPTIMAL else "inf"


class LocalMpcGear(LocalMpcMld, MpcGear):
    """fleet_decent_mld.py:226-253: LocalMpcMld's cost / constraints on the gear MPC, with the
    input cost on u_g."""

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
    ) -> None:
        MpcGear.__init__(self, pwa_system, N, thread_limit=thread_limit)
        self.setup_gears(N, pwa_system["F"], pwa_system["G"])
        self.setup_cost_and_constraints(None, spacing_policy, quadratic_cost, is_front, is_leader, is_trailer,
                                        accel_cnstr_tightening, real_vehicle_as_reference)

    def solve_mpc(self, state, raises: bool = True):
        return MpcGear.solve_mpc(self, state, raises)

    def absorb(self, res, i: int, run_time: float, raises: bool, state=None):
        return MpcGear.absorb(self, res, i, run_time, raises, state)
