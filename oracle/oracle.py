"""TEST INFRASTRUCTURE ONLY -- Python face of the CPU parity oracle (oracle/hvp_oracle.c).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module; the product (``hybrid-vehicle-platoon_amd/``) never does.

Besides the ctypes binding it restates, independently of the product package, the pieces of
the reference the checker needs as inputs:

* ``gear_pwa_system(m, ts)``   <- models.py:390-492 (PwaGearVehicle.build_gear_pwa_system)
                                  + models.py:370-387 (forward-Euler discretisation)
* ``friction_pwa_system(m, ts)`` <- models.py:272-332
* ``env_initial_state(n, seed)`` <- env.py:79-101 with the mpcrl seed derivation
                                  (SeedSequence(seed).generate_state(1)[0], model_validation.py:76)
* ``constant_velocity_prediction`` <- fleet_decent_mld.py:421-428, ``two_point_prediction`` <-
  :430-455 (two-point and saturated estimators), ``observe_states`` <- :348-419

Parity status: pinned to the reference's constants through the known answers listed in
SURVEY.md 8(c) (discretised tables, seed derivation, env init at seed 0) and, for the MIQP
layer, cross-checked against HiGHS (scipy.optimize.milp) on the reference's own big-M MLD
formulation with the L1 cost; the reference solver (Gurobi) itself cannot run here, so the
quadratic-cost MIQP optimum is "parity unpinned" against Gurobi and certified instead by
exhaustive sequence enumeration + per-QP KKT certificates.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None

# ------------------------------------------------------------------ reference constants
_B_GEAR = (4057, 2945, 2116, 1607, 1166, 838)
_VL = (3.94, 5.43, 7.56, 9.96, 13.70, 19.10)
_VH = (9.46, 13.04, 18.15, 23.90, 32.93, 45.84)
_CF, _MU, _G = 0.5, 0.01, 9.8
_VMIN, _VMAX = _VL[0], _VH[-1]


def _friction_constants():
    beta = 3 * _CF * _VMAX**2 / 16
    alpha = _VMAX / 2
    c1 = beta / alpha
    c2 = (_CF * _VMAX**2 - beta) / (_VMAX - alpha)
    return alpha, c1, c2, beta - alpha * c2


def _box():
    D = np.array([[1.0, 0], [-1, 0], [0, 1], [0, -1]])
    E = np.array([10000.0, -0.0, _VMAX, -_VMIN])
    F = np.array([1.0, -1.0])
    G = np.array([1.0, 1.0])
    return D, E, F, G


def gear_pwa_system(mass: float, ts: float = 1.0) -> dict:
    """Discrete 7-region gear PWA model as flat arrays (S[r][2][2], T[r][2], A[r][2][2], ...)."""
    alpha, c1, c2, d = _friction_constants()
    lim = [(_VH[i] - _VL[i]) / 2 + _VL[i] for i in range(1, 6)]
    cuts = [lim[0], lim[1], lim[2], alpha, lim[3], lim[4]]
    S = np.zeros((7, 2, 2))
    T = np.zeros((7, 2))
    for r in range(7):
        if r == 0:
            S[r] = [[0, 1], [0, 0]]
            T[r] = [cuts[0], 0]
        elif r == 6:
            S[r] = [[0, 0], [0, -1]]
            T[r] = [0, -cuts[5]]
        else:
            S[r] = [[0, 1], [0, -1]]
            T[r] = [cuts[r], -cuts[r - 1]]
    gear_of_region = [0, 1, 2, 3, 3, 4, 5]
    A = np.zeros((7, 2, 2))
    B = np.zeros((7, 2))
    c = np.zeros((7, 2))
    for r in range(7):
        fr = c2 if r >= 4 else c1
        A[r] = np.eye(2) + ts * np.array([[0, 1], [0, -fr / mass]])
        B[r] = ts * np.array([0, _B_GEAR[gear_of_region[r]] / mass])
        c[r] = ts * np.array([0, -_MU * _G - (d / mass if r >= 4 else 0.0)])
    D, E, F, G = _box()
    return dict(S=S, R=np.zeros((7, 2)), T=T, A=A, B=B, c=c, D=D, E=E, F=F, G=G,
                gear=np.array([1, 2, 3, 4, 4, 5, 6]))


def friction_pwa_system(mass: float, ts: float = 1.0) -> dict:
    alpha, c1, c2, d = _friction_constants()
    S = np.array([[[0, 1], [0, 0]], [[0, 0], [0, -1]]], dtype=float)
    T = np.array([[alpha, 0], [0, -alpha]])
    A = np.stack([np.eye(2) + ts * np.array([[0, 1], [0, -f / mass]]) for f in (c1, c2)])
    B = np.stack([ts * np.array([0, 1 / mass])] * 2)
    c = np.stack([ts * np.array([0, -_MU * _G]), ts * np.array([0, -_MU * _G - d / mass])])
    D, E, F, G = _box()
    return dict(S=S, R=np.zeros((2, 2)), T=T, A=A, B=B, c=c, D=D, E=E, F=F, G=G, gear=np.array([1, 2]))


def gear_friction_mld_system(mass: float, ts: float = 1.0) -> dict:
    """MpcGear's MIQP (mpcs/mpc_gear.py:30-114) on the pwa_friction model, restated as one PWA
    mode per (gear j, friction region r) with both binary families fixed:

    * u = sum_j b_j with b_j = sigma_j * Vehicle.b[j] * u_g (big-M rows :75-96) -> with
      sigma_j = 1 the velocity row reads v+ = A_r v + B_r Vehicle.b[j] u_g + c_r;
    * the control box F u <= G is replaced by F u_g <= G (:57-76), and the cost is on u_g
      (fleet_decent_mld.py:241 passes self.u_g to setup_cost_and_constraints);
    * sigma_j = 1 only if vl_j <= v_k <= vh_j (:98-110): two more region rows.

    Region rows per mode = the friction region's 2 rows + the gear's 2 rows.  Modes whose rows
    are jointly infeasible are dropped; order: gear-major, then friction region.  ``gear`` gives
    the gear label of each mode, ``friction`` its friction region."""
    fr = friction_pwa_system(mass, ts)
    S, T, A, B, c, gear, fric = [], [], [], [], [], [], []
    for j in range(6):
        for r in range(2):
            lo, hi = _VL[j], _VH[j]
            if r == 0:
                hi = min(hi, fr["T"][0][0])
            else:
                lo = max(lo, -fr["T"][1][1])
            if lo > hi:
                continue
            S.append(np.vstack([fr["S"][r], [[0, 1], [0, -1]]]))
            T.append(np.concatenate([fr["T"][r], [_VH[j], -_VL[j]]]))
            A.append(fr["A"][r])
            B.append(fr["B"][r] * _B_GEAR[j])
            c.append(fr["c"][r])
            gear.append(j + 1)
            fric.append(r)
    D, E, F, G = _box()
    nm = len(S)
    return dict(S=np.array(S), R=np.zeros((nm, 4)), T=np.array(T), A=np.array(A), B=np.array(B), c=np.array(c),
                D=D, E=E, F=F, G=G, gear=np.array(gear), friction=np.array(fric))


def env_seed(seed: int) -> int:
    return int(np.random.SeedSequence(seed).generate_state(1)[0])


def env_initial_state(n: int, seed: int) -> np.ndarray:
    """(2n,) int64 initial state of env.reset for the derived seed of `seed`."""
    rs = np.random.RandomState(env_seed(seed))
    vel = [30 * rs.random_sample() + 5 for _ in range(100)]
    pos = [3000.0]
    for _ in range(99):
        pos.append(-100 * rs.random_sample() + pos[-1] - 60)
    x = np.zeros(2 * n, dtype=np.int64)
    for i in range(n):
        p = max(pos)
        x[2 * i] = p
        x[2 * i + 1] = vel[i]
        pos.remove(p)
    return x


def constant_velocity_prediction(p: float, v: float, N: int, ts: float = 1.0) -> np.ndarray:
    """extrapolate_position_constant_vel (fleet_decent_mld.py:421-428)."""
    out = np.zeros((2, N + 1))
    out[:, 0] = (p, v)
    for k in range(N):
        out[0, k + 1] = out[0, k] + ts * out[1, k]
        out[1, k + 1] = out[1, k]
    return out


def two_point_prediction(p: float, v: float, v_prev: float, N: int, ts: float = 1.0,
                         saturated: bool = False) -> np.ndarray:
    """extrapolate_position_two_point_estimator (fleet_decent_mld.py:430-440): the velocity keeps
    changing by dv = v - v_prev every step; saturated (:442-455): only for the first floor(N/2)
    steps, constant after."""
    out = np.zeros((2, N + 1))
    out[:, 0] = (p, v)
    dv = v - v_prev
    steps = int(np.floor(N / 2)) if saturated else N
    for k in range(N):
        out[0, k + 1] = out[0, k] + ts * out[1, k]
        out[1, k + 1] = out[1, k] + (dv if k < steps else 0.0)
    return out


def observe_states(x, x_prev, N: int, leader_window, leader_index: int = 0, real_vehicle_as_reference: bool = False,
                   velocity_estimator: str = "none", ts: float = 1.0):
    """TrackingDecentMldCoordinator.observe_states (fleet_decent_mld.py:348-419) + the leader
    window of on_episode_start / on_timestep_end (:329-346) for ONE platoon, as the local-MPC
    parameter blocks [x0 | x_front | x_back | leader_x] and roles.  The first vehicle has no
    front prediction, the last no back prediction (zeros: those roles carry no such rows); the
    estimator is 'none' (constant velocity), 'two_point' or 'sat' (from x_prev's velocities)."""
    x = np.asarray(x, dtype=float).reshape(-1)
    n = len(x) // 2
    xp = x if x_prev is None else np.asarray(x_prev, dtype=float).reshape(-1)

    def pred(j):
        if velocity_estimator == "two_point":
            return two_point_prediction(x[2 * j], x[2 * j + 1], xp[2 * j + 1], N, ts)
        if velocity_estimator == "sat":
            return two_point_prediction(x[2 * j], x[2 * j + 1], xp[2 * j + 1], N, ts, saturated=True)
        return constant_velocity_prediction(x[2 * j], x[2 * j + 1], N, ts)

    params, roles = [], []
    zero = np.zeros((2, N + 1))
    for i in range(n):
        xf = pred(i - 1) if i > 0 else zero
        xb = pred(i + 1) if i < n - 1 else zero
        xl = np.asarray(leader_window, dtype=float).reshape(2, N + 1) if i == leader_index else zero
        params.append(np.concatenate([x[2 * i:2 * i + 2], xf.ravel(), xb.ravel(), xl.ravel()]))
        roles.append(role_bits(i, n, leader_index, real_vehicle_as_reference))
    return np.array(params), np.array(roles, dtype=np.int32)


# ------------------------------------------------------------------ controller constants
@dataclass
class Cfg:
    """Params of misc/common_controller_params.py:14-23 + spacing policy (d0, t0)."""

    Qx: tuple = (1.0, 0.0, 0.0, 0.1)
    Qu: float = 1.0
    Qdu: float = 0.0
    w: float = 1e4
    a_acc: float = 2.5
    a_dec: float = -2.0
    ts: float = 1.0
    d_safe: float = 25.0
    tight: float = 0.0
    d0: float = 50.0
    t0: float = 0.0

    def vector(self) -> np.ndarray:
        return np.array(list(self.Qx) + [self.Qu, self.Qdu, self.w, self.a_acc, self.a_dec, self.ts,
                                         self.d_safe, self.tight, self.d0, self.t0], dtype=np.float64)


ROLE_SAFE_FRONT, ROLE_SAFE_BACK, ROLE_TRACK_FRONT, ROLE_TRACK_BACK, ROLE_TRACK_LEADER, ROLE_LEADER_SPACING = (
    1, 2, 4, 8, 16, 32)


def role_bits(i: int, n: int, leader_index: int = 0, real_vehicle_as_reference: bool = False) -> int:
    """Role of vehicle i as set up in fleet_decent_mld.py:506-518 / :100-153."""
    is_front, is_trailer, is_leader = i == 0, i == n - 1, i == leader_index
    r = 0
    if not is_front:
        r |= ROLE_SAFE_FRONT
    if not is_trailer:
        r |= ROLE_SAFE_BACK
    if not is_front and not is_leader:
        r |= ROLE_TRACK_FRONT
    if not is_trailer and not is_leader:
        r |= ROLE_TRACK_BACK
    if is_leader:
        r |= ROLE_TRACK_LEADER
        if real_vehicle_as_reference:
            r |= ROLE_LEADER_SPACING
    return r


# ------------------------------------------------------------------ ctypes binding
def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(
        os.path.join(_HERE, "hvp_oracle.c")
    ):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        c_int = ctypes.c_int
        model_args = [c_int, c_int, c_int, dp, dp, dp, dp, dp, dp, c_int, dp, dp, c_int, dp, dp]
        L.oracle_solve_miqp.argtypes = model_args + [dp, c_int, c_int, dp, dp, dp, dp, c_int, dp, dp, ip, dp, dp, ip,
                                                     c_int]
        L.oracle_solve_miqp.restype = c_int
        L.oracle_count_candidates.argtypes = model_args + [dp, dp, ip, c_int]
        L.oracle_count_candidates.restype = c_int
        L.oracle_solve_qp.argtypes = model_args + [dp, c_int, c_int, ip, dp, dp, dp, dp, dp, dp]
        L.oracle_solve_qp.restype = c_int
        L.oracle_solve_batch.argtypes = [c_int, c_int, c_int, c_int, c_int, dp, dp, dp, dp, dp, dp, c_int, dp, dp,
                                         c_int, dp, dp, dp, c_int, ip, ip, dp, c_int, dp, dp, ip, dp, c_int]
        L.oracle_solve_batch.restype = c_int
        L.oracle_certify_batch.argtypes = [c_int, c_int, c_int, c_int, c_int, dp, dp, dp, dp, dp, dp, c_int, dp, dp,
                                           c_int, dp, dp, dp, c_int, ip, ip, dp, ip, dp, c_int]
        L.oracle_certify_batch.restype = c_int
        L.oracle_solve_admm_miqp.argtypes = model_args + [dp, c_int, ctypes.c_double, dp, c_int, dp, dp, ip, dp,
                                                          dp, dp]
        L.oracle_solve_admm_miqp.restype = c_int
        L.oracle_solve_gadmm_qp.argtypes = model_args + [dp, c_int, c_int, ctypes.c_double, dp, ip, dp, dp, dp, dp,
                                                         dp]
        L.oracle_solve_gadmm_qp.restype = c_int
        L.oracle_solve_cent.argtypes = [c_int, c_int, c_int, c_int, dp, dp, dp, dp, dp, dp, c_int, dp, dp, c_int, dp,
                                        dp, dp, c_int, dp, dp, dp, dp, ip, dp]
        L.oracle_solve_cent.restype = c_int
        L.oracle_set_cent_gap.argtypes = [ctypes.c_double]
        L.oracle_set_cent_gap.restype = None
        L.oracle_set_cent_cap.argtypes = [ctypes.c_long]
        L.oracle_set_cent_cap.restype = None
        L.oracle_set_cent_relax.argtypes = [ctypes.c_int]
        L.oracle_set_cent_relax.restype = None
        L.oracle_set_method.argtypes = [c_int]
        L.oracle_set_method.restype = None
        _lib = L
    return _lib


def _d(a) -> ctypes.POINTER(ctypes.c_double):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _i(a) -> ctypes.POINTER(ctypes.c_int):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def _model_arrays(sysd: dict):
    arr = {k: np.ascontiguousarray(np.asarray(sysd[k], dtype=np.float64)) for k in "SRTABcDEFG"}
    nreg = arr["S"].shape[0]
    nsr = arr["S"].shape[1]
    return nreg, nsr, arr


def _model_args(sysd: dict):
    nreg, nsr, a = _model_arrays(sysd)
    keep = a
    args = [nreg, nsr, _d(a["S"]), _d(a["R"]), _d(a["T"]), _d(a["A"]), _d(a["B"]), _d(a["c"]),
            a["D"].shape[0], _d(a["D"]), _d(a["E"]), a["F"].shape[0], _d(a["F"]), _d(a["G"])]
    return args, keep


@dataclass
class MiqpResult:
    x: np.ndarray  # (2, N+1)
    u: np.ndarray  # (N,)
    sigma: np.ndarray  # (N,) region indices
    cost: float
    n_candidates: int
    n_converged: int
    n_certified: int
    best_certified: bool
    status: int
    iters: int
    cand_obj: np.ndarray | None = None
    cand_sigma: np.ndarray | None = None


METHOD_ENUMERATE, METHOD_BNB = 0, 1


def set_method(method: int) -> None:
    """0: exhaustive enumeration of the region sequences (default); 1: depth-first branch and
    bound with relaxed-prefix bounds (hvp_oracle.c bnb_dfs), needed for N >= 10."""
    lib().oracle_set_method(int(method))


def solve_miqp(sysd: dict, cfg: Cfg, N: int, role: int, x0, xf, xb, xl, quadratic: bool = True,
               maxit: int = 200, want_candidates: bool = False) -> MiqpResult:
    L = lib()
    args, keep = _model_args(sysd)
    cv = cfg.vector()
    f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))  # noqa: E731
    x0, xf, xb, xl = f(x0).ravel(), f(xf), f(xb), f(xl)
    x_out = np.zeros((2, N + 1))
    u_out = np.zeros(N)
    sig = np.zeros(N, dtype=np.int32)
    info = np.zeros(7)
    cap = 20000 if want_candidates else 0
    cobj = np.zeros(max(cap, 1))
    csig = np.zeros((max(cap, 1), N), dtype=np.int32)
    rc = L.oracle_solve_miqp(N, *args, _d(cv), int(quadratic), int(role), _d(x0), _d(xf), _d(xb), _d(xl), maxit,
                             _d(x_out), _d(u_out), _i(sig), _d(info), _d(cobj), _i(csig), cap)
    del keep
    if rc != 0:
        raise RuntimeError(f"oracle_solve_miqp failed ({rc})")
    n = int(info[1])
    res = MiqpResult(x_out, u_out, sig, float(info[0]), n, int(info[2]), int(info[3]), bool(info[4]), int(info[5]),
                     int(info[6]))
    if want_candidates:
        res.cand_obj = cobj[:n].copy()
        res.cand_sigma = csig[:n].copy()
    return res


@dataclass
class AdmmResult:
    x: np.ndarray        # (2, N+1)
    u: np.ndarray        # (N,)
    sigma: np.ndarray    # (N,)
    cost: float
    x_front: np.ndarray  # (2, N+1) optimal front copy (zeros if the role has none)
    x_back: np.ndarray   # (2, N+1)
    n_qps: int
    status: int
    certified: bool


def admm_params(x0, y_front, z_front, y_back, z_back, leader_x) -> np.ndarray:
    """Parameter row of the ADMM local problem (include/hvp.h hvp_params_stride_admm)."""
    blocks = [np.asarray(b, dtype=np.float64).reshape(-1) for b in (y_front, z_front, y_back, z_back, leader_x)]
    return np.concatenate([np.asarray(x0, dtype=np.float64).reshape(-1)[:2]] + blocks)


def solve_admm_miqp(sysd: dict, cfg: Cfg, N: int, role: int, rho: float, params, maxit: int = 200,
                    quadratic: bool = True) -> AdmmResult:
    """LocalMpcADMM's MIQP (fleet_naive_admm.py:24-253) in the full (x, u, s, copies) space,
    branch and bound over the region sequences; see hvp_oracle.c oracle_solve_admm_miqp.
    quadratic=False: min_1_norm (LocalMpcADMM(quadratic_cost=False), :74-77) -- L1 tracking and
    input terms next to the quadratic ADMM terms of the copies."""
    L = lib()
    args, keep = _model_args(sysd)
    cv = cfg.vector()
    p = np.ascontiguousarray(np.asarray(params, dtype=np.float64).reshape(-1))
    assert p.size == 2 + 10 * (N + 1)
    x_out, u_out = np.zeros((2, N + 1)), np.zeros(N)
    sig, info = np.zeros(N, dtype=np.int32), np.zeros(7)
    xf, xb = np.zeros((2, N + 1)), np.zeros((2, N + 1))
    rl = int(role) | (0 if quadratic else 1 << 17)
    rc = L.oracle_solve_admm_miqp(N, *args, _d(cv), rl, float(rho), _d(p), maxit, _d(x_out), _d(u_out), _i(sig),
                                  _d(info), _d(xf), _d(xb))
    del keep
    if rc != 0:
        raise RuntimeError(f"oracle_solve_admm_miqp failed ({rc})")
    return AdmmResult(x_out, u_out, sig, float(info[0]), xf, xb, int(info[1]), int(info[5]), bool(info[4]))


def candidates(sysd: dict, cfg: Cfg, N: int, x0, cap: int = 200000) -> np.ndarray:
    L = lib()
    args, keep = _model_args(sysd)
    cv = cfg.vector()
    x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64)).ravel()
    out = np.zeros((cap, N), dtype=np.int32)
    n = L.oracle_count_candidates(N, *args, _d(cv), _d(x0), _i(out), cap)
    del keep
    if n < 0:
        raise RuntimeError("oracle_count_candidates: unsupported model")
    return out[: min(n, cap)].copy()


def solve_qp(sysd: dict, cfg: Cfg, N: int, role: int, sigma, x0, xf, xb, xl, quadratic: bool = True):
    """One fixed-sequence QP: returns (objective, converged, certified, z, (nz, m, neq))."""
    L = lib()
    args, keep = _model_args(sysd)
    cv = cfg.vector()
    f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))  # noqa: E731
    sig = np.ascontiguousarray(np.asarray(sigma, dtype=np.int32))
    z = np.zeros(256)
    info = np.zeros(8)
    L.oracle_solve_qp(N, *args, _d(cv), int(quadratic), int(role), _i(sig), _d(f(x0).ravel()), _d(f(xf)),
                      _d(f(xb)), _d(f(xl)), _d(z), _d(info))
    del keep
    nz = int(info[4])
    return float(info[0]), bool(info[1]), bool(info[2]), z[:nz].copy(), (nz, int(info[5]), int(info[6]))


def solve_batch(systems: list[dict], cfg: Cfg, N: int, sys_idx, roles, params, quadratic: bool = True,
                maxit: int = 200, nthreads: int = 1):
    """Batch of instances (params rows laid out as include/hvp.h hvp_params_stride)."""
    L = lib()
    nreg = np.asarray(systems[0]["S"]).shape[0]
    nsr = np.asarray(systems[0]["S"]).shape[1]
    st = {k: np.ascontiguousarray(np.stack([np.asarray(s[k], dtype=np.float64) for s in systems])) for k in
          "SRTABcDEFG"}
    B = len(sys_idx)
    sys_idx = np.ascontiguousarray(np.asarray(sys_idx, dtype=np.int32))
    roles = np.ascontiguousarray(np.asarray(roles, dtype=np.int32))
    params = np.ascontiguousarray(np.asarray(params, dtype=np.float64))
    cv = cfg.vector()
    x_out = np.zeros((B, 2, N + 1))
    u_out = np.zeros((B, N))
    sig = np.zeros((B, N), dtype=np.int32)
    info = np.zeros((B, 7))
    rc = L.oracle_solve_batch(B, N, len(systems), nreg, nsr, _d(st["S"]), _d(st["R"]), _d(st["T"]), _d(st["A"]),
                              _d(st["B"]), _d(st["c"]), st["D"].shape[1], _d(st["D"]), _d(st["E"]), st["F"].shape[1],
                              _d(st["F"]), _d(st["G"]), _d(cv), int(quadratic), _i(sys_idx), _i(roles), _d(params),
                              maxit, _d(x_out), _d(u_out), _i(sig), _d(info), nthreads)
    if rc != 0:
        raise RuntimeError("oracle_solve_batch failed")
    return x_out, u_out, sig, info


def certify_batch(systems: list[dict], cfg: Cfg, N: int, sys_idx, roles, params, sigma, quadratic: bool = True,
                  nthreads: int = 1):
    """KKT-certified optimum of every instance's fixed-sequence QP for the GIVEN sequences (the
    product's answers).  Returns (objective (B,), certified (B,) bool, u (B, N))."""
    L = lib()
    nreg = np.asarray(systems[0]["S"]).shape[0]
    nsr = np.asarray(systems[0]["S"]).shape[1]
    st = {k: np.ascontiguousarray(np.stack([np.asarray(s[k], dtype=np.float64) for s in systems])) for k in
          "SRTABcDEFG"}
    B = len(sys_idx)
    sys_idx = np.ascontiguousarray(np.asarray(sys_idx, dtype=np.int32))
    roles = np.ascontiguousarray(np.asarray(roles, dtype=np.int32))
    params = np.ascontiguousarray(np.asarray(params, dtype=np.float64))
    sig = np.ascontiguousarray(np.asarray(sigma, dtype=np.int32).reshape(B, N))
    out = np.zeros((B, 2 + N))
    rc = L.oracle_certify_batch(B, N, len(systems), nreg, nsr, _d(st["S"]), _d(st["R"]), _d(st["T"]), _d(st["A"]),
                                _d(st["B"]), _d(st["c"]), st["D"].shape[1], _d(st["D"]), _d(st["E"]),
                                st["F"].shape[1], _d(st["F"]), _d(st["G"]), _d(cfg.vector()), int(quadratic),
                                _i(sys_idx), _i(roles), _d(params), _i(sig), _d(out), nthreads)
    if rc != 0:
        raise RuntimeError("oracle_certify_batch failed")
    return out[:, 0].copy(), out[:, 1] != 0, out[:, 2:].copy()


def export_qp(sysd: dict, cfg: Cfg, N: int, role: int, sigma, x0, xf, xb, xl, quadratic: bool = True):
    """Dense (P, q, r0, Aeq, beq, G, h) of one fixed-sequence QP, for independent cross-checks."""
    L = lib()
    if not hasattr(L, "_export_set"):
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int)
        c_int = ctypes.c_int
        L.oracle_export_qp.argtypes = [c_int, c_int, c_int, dp, dp, dp, dp, dp, dp, c_int, dp, dp, c_int, dp, dp, dp,
                                       c_int, c_int, ip, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp, dp]
        L.oracle_export_qp.restype = c_int
        L._export_set = True
    args, keep = _model_args(sysd)
    cv = cfg.vector()
    f = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64))  # noqa: E731
    sig = np.ascontiguousarray(np.asarray(sigma, dtype=np.int32))
    P = np.zeros(200 * 200); q = np.zeros(200); A = np.zeros(40 * 200); b = np.zeros(40)
    G = np.zeros(420 * 200); h = np.zeros(420); dims = np.zeros(5)
    rc = L.oracle_export_qp(N, *args, _d(cv), int(quadratic), int(role), _i(sig), _d(f(x0).ravel()), _d(f(xf)),
                            _d(f(xb)), _d(f(xl)), _d(P), _d(q), _d(A), _d(b), _d(G), _d(h), _d(dims))
    del keep
    if rc != 0:
        raise RuntimeError("export failed")
    nz, ne, m = int(dims[0]), int(dims[1]), int(dims[2])
    return (P[: nz * nz].reshape(nz, nz), q[:nz].copy(), float(dims[3]), A[: ne * nz].reshape(ne, nz), b[:ne].copy(),
            G[: m * nz].reshape(m, nz), h[:m].copy())


class AdmmCoordinator:
    """Restatement of ADMMCoordinator.get_control (fleet_naive_admm.py:379-468) on oracle local
    solves, for the end-to-end parity of the ADMM iteration (test infrastructure).

    State carried across time steps as in the reference: y_front / y_back (never reset), the
    parameter blocks each local MPC was last given, and the last local solutions (warm start)."""

    def __init__(self, sysd: dict, cfg: Cfg, N: int, n: int, rho: float = 0.5, leader_index: int = 0,
                 quadratic: bool = True):
        self.sysd, self.cfg, self.N, self.n, self.rho = sysd, cfg, N, n, rho
        self.leader_index = leader_index
        self.quadratic = quadratic  # False: LocalMpcADMM(quadratic_cost=False), fleet_naive_admm.py:74-77
        K = (2, N + 1)
        self.y_front = [np.zeros(K) for _ in range(n)]
        self.y_back = [np.zeros(K) for _ in range(n)]
        self.z = [np.zeros(K) for _ in range(n)]
        self.blocks = [{"yf": np.zeros(K), "zf": np.zeros(K), "yb": np.zeros(K), "zb": np.zeros(K),
                        "xl": np.zeros(K)} for _ in range(n)]
        self.x_pred = [None] * n
        self.roles = [role_bits(i, n, leader_index) for i in range(n)]

    def set_leader_x(self, xl) -> None:
        self.blocks[self.leader_index]["xl"] = np.asarray(xl, dtype=float)

    def step(self, state, admm_iters: int, pool=None):
        """One time step (admm_iters ADMM iterations).  pool: an optional process pool
        (multiprocessing, spawn context) that runs the n local solves of an iteration in parallel
        -- the same solves, the same answers (fixture generation at configs[2]'s size)."""
        n, N, rho = self.n, self.N, self.rho
        x = np.asarray(state, dtype=float).reshape(n, 2)
        for i in range(n):  # warm start (:392-402)
            if i != 0 and self.x_pred[i - 1] is not None:
                xp = self.x_pred[i - 1]
                self.blocks[i]["yf"] = self.y_front[i].copy()
                self.blocks[i]["zf"] = np.hstack((xp[:, 1:], xp[:, [-1]]))
            if i != n - 1 and self.x_pred[i + 1] is not None:
                xp = self.x_pred[i + 1]
                self.blocks[i]["yb"] = self.y_back[i].copy()
                self.blocks[i]["zb"] = np.hstack((xp[:, 1:], xp[:, [-1]]))
        history = []
        for _ in range(admm_iters):
            args = []
            for i in range(n):  # x-update (:407-419)
                b = self.blocks[i]
                p = admm_params(x[i], b["yf"], b["zf"], b["yb"], b["zb"], b["xl"])
                args.append((self.sysd, self.cfg, N, self.roles[i], rho, p, 200, self.quadratic))
            res = pool.starmap(solve_admm_miqp, args) if pool is not None else [solve_admm_miqp(*a) for a in args]
            for i, r in enumerate(res):
                if r.status != 0:
                    raise RuntimeError(f"oracle ADMM local MIQP {i} status {r.status}")
            history.append(res)
            for i in range(n):  # z- and y-update (:421-447)
                if i == 0:
                    self.z[i] = 0.5 * (res[i].x + res[i + 1].x_front)
                    self.y_front[i + 1] = self.y_front[i + 1] + rho * (res[i + 1].x_front - self.z[i])
                elif i == n - 1:
                    self.z[i] = 0.5 * (res[i].x + res[i - 1].x_back)
                    self.y_back[i - 1] = self.y_back[i - 1] + rho * (res[i - 1].x_back - self.z[i])
                else:
                    self.z[i] = (res[i].x + res[i + 1].x_front + res[i - 1].x_back) / 3.0
                    self.y_front[i + 1] = self.y_front[i + 1] + rho * (res[i + 1].x_front - self.z[i])
                    self.y_back[i - 1] = self.y_back[i - 1] + rho * (res[i - 1].x_back - self.z[i])
            for i in range(n):  # set the local vars (:453-468)
                if i != 0:
                    self.blocks[i]["yf"], self.blocks[i]["zf"] = self.y_front[i].copy(), self.z[i - 1].copy()
                if i != n - 1:
                    self.blocks[i]["yb"], self.blocks[i]["zb"] = self.y_back[i].copy(), self.z[i + 1].copy()
        last = history[-1]
        for i in range(n):
            self.x_pred[i] = last[i].x
        return np.array([r.u[0] for r in last]), history


# ------------------------------------------------------------------ switching ADMM (fleet_g_admm.py)
@dataclass
class GAdmmQpResult:
    x: np.ndarray        # (2, N+1)
    u: np.ndarray        # (N,)
    x_front: np.ndarray  # (2, N+1) optimal copy of the vehicle ahead (zeros if none)
    x_back: np.ndarray   # (2, N+1) optimal copy of the vehicle behind (zeros if none)
    cost: float          # the local objective incl. every ADMM term (sol.f)
    status: int          # 0 ok, 1 infeasible / not converged
    certified: bool
    switch: int          # region-edge multiplier bits, see hvp_oracle.c oracle_solve_gadmm_qp


def gadmm_params(x0, y_front, z_front, y_back, z_back, leader_x, y_own, z_own) -> np.ndarray:
    """Parameter row of the switching-ADMM local problem (include/hvp.h hvp_params_stride_gadmm)."""
    blocks = [np.asarray(b, dtype=np.float64).reshape(-1)
              for b in (y_front, z_front, y_back, z_back, leader_x, y_own, z_own)]
    return np.concatenate([np.asarray(x0, dtype=np.float64).reshape(-1)[:2]] + blocks)


def solve_gadmm_qp(sysd: dict, cfg: Cfg, N: int, role: int, back_copy: bool, rho: float, params,
                   sigma) -> GAdmmQpResult:
    """fleet_g_admm.LocalMpc (:22-205) for a fixed switching sequence, in the full
    (x, u, s, copies) space; see hvp_oracle.c oracle_solve_gadmm_qp."""
    L = lib()
    args, keep = _model_args(sysd)
    cv = cfg.vector()
    p = np.ascontiguousarray(np.asarray(params, dtype=np.float64).reshape(-1))
    assert p.size == 2 + 14 * (N + 1)
    sig = np.ascontiguousarray(np.asarray(sigma, dtype=np.int32).reshape(-1))
    x_out, u_out = np.zeros((2, N + 1)), np.zeros(N)
    xf, xb, info = np.zeros((2, N + 1)), np.zeros((2, N + 1)), np.zeros(4)
    rc = L.oracle_solve_gadmm_qp(N, *args, _d(cv), int(role), int(bool(back_copy)), float(rho), _d(p), _i(sig),
                                 _d(x_out), _d(u_out), _d(xf), _d(xb), _d(info))
    del keep
    if rc != 0:
        raise RuntimeError(f"oracle_solve_gadmm_qp failed ({rc})")
    return GAdmmQpResult(x_out, u_out, xf, xb, float(info[0]), int(info[1]), bool(info[2]), int(info[3]))


def region_bands(sysd: dict) -> tuple[np.ndarray, np.ndarray]:
    """Velocity interval [vlo_r, vhi_r] of every region from its rows S x <= T (v-only rows)."""
    S, T = np.asarray(sysd["S"], dtype=float), np.asarray(sysd["T"], dtype=float).reshape(len(sysd["S"]), -1)
    lo, hi = np.full(len(S), -np.inf), np.full(len(S), np.inf)
    for r in range(len(S)):
        for row in range(S.shape[1]):
            s = S[r, row, 1]
            if S[r, row, 0] != 0.0 or s == 0.0:
                continue
            if s > 0:
                hi[r] = min(hi[r], T[r, row] / s)
            else:
                lo[r] = max(lo[r], T[r, row] / s)
    return lo, hi


def gadmm_role(i: int, n: int) -> tuple[int, bool]:
    """(role bits, back_copy) of vehicle i of a g_admm chain (fleet_g_admm.py:341-389: vehicle 0
    leads and tracks x_ref; every other vehicle tracks / keeps its distance to its front copy)."""
    role = ROLE_TRACK_LEADER if i == 0 else (ROLE_SAFE_FRONT | ROLE_TRACK_FRONT)
    return role, i < n - 1


class GAdmmCoordinator:
    """Restatement (test infrastructure) of TrackingGAdmmCoordinator.g_admm_control
    (fleet_g_admm.py:255-301) on top of GAdmmCoordinator / MpcSwitching of dmpcpwa 0.0.2 [EXT,
    absent: parity unpinned against it].  The switching-ADMM rule restated here (and run on the
    device by hvp/gadmm.py) -- Mallick, Dabiri, De Schutter, "switching ADMM" for PWA systems:

    per warm start u (n, N):
      1. rollout: x_{i,0} = state_i, sigma_{i,k} = first region whose closed velocity band holds
         v_{i,k}, x_{i,k+1} = A x + B u + c of that region (the discrete system dicts);
      2. z_i <- the rollout of vehicle i, y <- 0 (own block and both copies);
      3. rounds (at most max_rounds): admm_iters x [every vehicle solves its local QP for its
         sequence (x-update, Jacobi), z_j = mean of x_j and its copies held by j-1 (back copy)
         and j+1 (front copy), y += rho (x_aug - z)]; then every vehicle moves sigma_{i,k}
         (k = 1..N-1) across a velocity edge of its region whose row is active with multiplier
         > 1e-6 (into the region on the other side of that edge); no change anywhere -> stop;
      4. cost = sum of the local objectives of the last iteration (sol.f).
    Warm starts (:256-272): constant-velocity throttle (Vehicle.get_u_for_constant_vel,
    models.py:537-556) and, from the second step on, the shifted previous solution; the lowest
    cost wins, ties to the first (:285-293); the previous solution is that of the last warm start
    that succeeded."""

    def __init__(self, systems: list[dict], cfg: Cfg, N: int, rho: float = 0.5, admm_iters: int = 100,
                 max_rounds: int = 10):
        self.systems, self.cfg, self.N, self.rho = systems, cfg, N, rho
        self.n = len(systems)
        self.admm_iters, self.max_rounds = admm_iters, max_rounds
        self.bands = [region_bands(s) for s in systems]
        self.prev_u = None
        self.leader_x = np.zeros((2, N + 1))
        self.trace: list | None = None  # set to a list to record every local QP (fixtures)

    def set_leader_traj(self, leader_x) -> None:
        self.leader_x = np.asarray(leader_x, dtype=np.float64).reshape(2, self.N + 1)

    def u_const_vel(self, i: int, v: float) -> float:
        """get_u_for_constant_vel (models.py:537-556): region by the [0, 1e-4] buffer rule."""
        lo, hi = self.bands[i]
        s = self.systems[i]
        for r in range(len(lo)):
            if lo[r] - 1e-4 <= v <= hi[r]:
                a = float(np.asarray(s["A"][r])[1, 1])
                b = float(np.asarray(s["B"][r]).reshape(2)[1])
                c = float(np.asarray(s["c"][r]).reshape(2)[1])
                return ((1.0 - a) * v - c) / b
        raise RuntimeError("Didn't find any PWA region for the given speed!")

    def rollout(self, i: int, x0, u) -> tuple[np.ndarray, np.ndarray] | None:
        lo, hi = self.bands[i]
        s = self.systems[i]
        N = self.N
        X = np.zeros((2, N + 1))
        X[:, 0] = x0
        sig = np.zeros(N, dtype=np.int32)
        for k in range(N):
            v = X[1, k]
            r = next((r for r in range(len(lo)) if lo[r] <= v <= hi[r]), None)
            if r is None:
                return None
            sig[k] = r
            A, B, c = np.asarray(s["A"][r]), np.asarray(s["B"][r]).reshape(2), np.asarray(s["c"][r]).reshape(2)
            X[:, k + 1] = A @ X[:, k] + B * u[k] + c
        return X, sig

    def switch(self, i: int, sig: np.ndarray, bits: int) -> np.ndarray:
        lo, hi = self.bands[i]
        out = sig.copy()
        tol = lambda e: 1e-9 * (1.0 + abs(e))  # noqa: E731
        for k in range(1, self.N):
            r = int(sig[k])
            if (bits >> (2 * (k - 1))) & 1:  # lower edge of r active: into the region below
                cand = [q for q in range(len(lo)) if q != r and abs(hi[q] - lo[r]) <= tol(lo[r])]
            elif (bits >> (2 * (k - 1) + 1)) & 1:
                cand = [q for q in range(len(lo)) if q != r and abs(lo[q] - hi[r]) <= tol(hi[r])]
            else:
                continue
            if cand:
                out[k] = cand[0]
        return out

    def run(self, state, u_ws):
        """One GAdmmCoordinator.g_admm_control(state, warm_start=u_ws): (u (n, N), cost, info)
        or None when a rollout or a local QP fails (error / infeasibility flag)."""
        n, N, rho = self.n, self.N, self.rho
        x = np.asarray(state, dtype=np.float64).reshape(n, 2)
        X, sig = [], []
        for i in range(n):
            r = self.rollout(i, x[i], u_ws[i])
            if r is None:
                return None
            X.append(r[0])
            sig.append(r[1])
        Z = [X[i].copy() for i in range(n)]
        K = (2, N + 1)
        yo = [np.zeros(K) for _ in range(n)]
        yf = [np.zeros(K) for _ in range(n)]
        yb = [np.zeros(K) for _ in range(n)]
        rounds, res = 0, None
        for rounds in range(1, self.max_rounds + 1):
            for _ in range(self.admm_iters):
                res = []
                for i in range(n):
                    role, bc = gadmm_role(i, n)
                    zf = Z[i - 1] if i > 0 else np.zeros(K)
                    zb = Z[i + 1] if i < n - 1 else np.zeros(K)
                    xl = self.leader_x if i == 0 else np.zeros(K)
                    p = gadmm_params(x[i], yf[i], zf, yb[i], zb, xl, yo[i], Z[i])
                    r = solve_gadmm_qp(self.systems[i], self.cfg, N, role, bc, rho, p, sig[i])
                    if self.trace is not None:
                        self.trace.append((i, role, bc, p, sig[i].copy(), r))
                    if r.status != 0:
                        return None
                    res.append(r)
                for j in range(n):  # z-update
                    parts = [res[j].x]
                    if j > 0:
                        parts.append(res[j - 1].x_back)
                    if j < n - 1:
                        parts.append(res[j + 1].x_front)
                    Z[j] = sum(parts[1:], parts[0]) / len(parts)
                for i in range(n):  # y-update
                    yo[i] = yo[i] + rho * (res[i].x - Z[i])
                    if i > 0:
                        yf[i] = yf[i] + rho * (res[i].x_front - Z[i - 1])
                    if i < n - 1:
                        yb[i] = yb[i] + rho * (res[i].x_back - Z[i + 1])
            new = [self.switch(i, sig[i], res[i].switch) for i in range(n)]
            changed = any((new[i] != sig[i]).any() for i in range(n))
            sig = new
            if not changed:
                break
        u = np.stack([r.u for r in res])
        cost = float(sum(r.cost for r in res))
        return u, cost, {"rounds": rounds, "sigma": np.stack(sig), "x": np.stack([r.x for r in res])}

    def control(self, state):
        """TrackingGAdmmCoordinator.g_admm_control: best of the warm starts; returns the
        control trajectories u (n, N) of the winner and the per-warm-start details."""
        n, N = self.n, self.N
        x = np.asarray(state, dtype=np.float64).reshape(n, 2)
        warm = [np.stack([np.full(N, self.u_const_vel(i, x[i, 1])) for i in range(n)])]
        if self.prev_u is not None:
            warm.append(np.concatenate([self.prev_u[:, 1:], self.prev_u[:, -1:]], axis=1))
        best, best_cost, runs = None, float("inf"), []
        for w in warm:
            r = self.run(state, w)
            runs.append(r)
            if r is None:
                continue
            self.prev_u = r[0]
            if r[1] < best_cost:
                best, best_cost = r, r[1]
        if best is None:
            raise RuntimeError("No solution found for any of the warm starts")
        return best[0], best_cost, runs


# ------------------------------------------------------------------ centralised MLD (mpcs/cent_mld.py)
@dataclass
class CentResult:
    x: np.ndarray      # (n, 2, N+1)
    u: np.ndarray      # (n, N)
    sigma: np.ndarray  # (n, N)
    cost: float
    status: int        # 0 optimal, 1 infeasible
    n_qps: int


def set_cent_gap(gap: float) -> None:
    """Relative MIP gap of solve_cent's pruning (0 = exact; Gurobi's default MIPGap is 1e-4)."""
    lib().oracle_set_cent_gap(float(gap))


def set_cent_cap(cap: int) -> None:
    """QP budget per solve_cent call (0 = none; a capped search is a timing sample, not a result)."""
    lib().oracle_set_cent_cap(int(cap))


def set_cent_relax(on: bool) -> None:
    """Tail relaxation of the centralised search: True (default) = reachable intervals + virtual
    region (hvp_oracle.c:relax_tail), False = undecided steps without velocity dynamics / inputs."""
    lib().oracle_set_cent_relax(int(bool(on)))


def solve_cent(systems: list[dict], cfg: Cfg, N: int, x0, leader_x, leader_index: int = 0,
               real_vehicle_as_reference: bool = False, exhaustive: bool = False,
               quadratic: bool = True) -> CentResult:
    """MpcMldCent's MIQP (mpcs/cent_mld.py:48-182) for one platoon: full (x, u, s) space, branch
    and bound over the joint region sequences in time-major order (or exhaustive enumeration);
    ties to the lexicographically first joint sequence in that order (hvp_oracle.c oracle_solve_cent).
    quadratic=False: the min_1_norm cost (cent_mld.py:58-61), a MILP."""
    L = lib()
    n = len(systems)
    arrs = [_model_arrays(s)[2] for s in systems]
    nreg, nsr = _model_arrays(systems[0])[:2]
    st = {k: np.ascontiguousarray(np.stack([a[k] for a in arrs])) for k in "SRTABcDEFG"}
    cv = cfg.vector()
    x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).reshape(-1))
    xl = np.ascontiguousarray(np.asarray(leader_x, dtype=np.float64).reshape(2, N + 1))
    x_out, u_out = np.zeros((n, 2, N + 1)), np.zeros((n, N))
    sig, info = np.zeros((n, N), dtype=np.int32), np.zeros(3)
    role = (int(leader_index) | (256 if real_vehicle_as_reference else 0) | (65536 if exhaustive else 0)
            | (0 if quadratic else 131072))
    rc = L.oracle_solve_cent(n, N, nreg, nsr, _d(st["S"]), _d(st["R"]), _d(st["T"]), _d(st["A"]), _d(st["B"]),
                             _d(st["c"]), st["D"].shape[1], _d(st["D"]), _d(st["E"]), st["F"].shape[1], _d(st["F"]),
                             _d(st["G"]), _d(cv), role, _d(x0), _d(xl), _d(x_out), _d(u_out), _i(sig), _d(info))
    if rc != 0:
        raise RuntimeError(f"oracle_solve_cent failed ({rc})")
    return CentResult(x_out, u_out, sig, float(info[0]), int(info[1]), int(info[2]))


# ------------------------------------------------------------------ plant step (env.py / models.py)
_TRAC_T = ((253.54, 4056.7, 3042.0), (184.0, 2944.75, 2208.55), (132.22, 2115.6, 1586.7),
           (100 / 415, 1605.0, 1205.0), (72.88, 1166.0, 874.7), (52.4, 838.0, 628.3))   # models.py:13-20
_TRAC_V = ((2.0706, 4.12158, 9.29, 12.38), (2.85, 5.675, 12.7956, 17.06), (3.9705, 7.90316, 17.8105, 23.7474),
           (5.228, 10.42, 23.454, 31.2704), (7.203, 14.335, 32.31, 43.0802),
           (10.027, 19.956, 44.978, 59.9715))                                            # models.py:21-28


def _traction(v: float, j: int) -> float:
    """GearTransimission.get_traction (models.py:30-50), same operation order."""
    if not 1 <= j <= 6 or v < 2.0706 or v > 59.9715:
        raise RuntimeError("out of range")
    (v0, v1, v2, v3), (t0, t1, t2) = _TRAC_V[j - 1], _TRAC_T[j - 1]
    if v <= v0 or v >= v3:
        raise RuntimeError("out of range for gear")
    if v < v1:
        return ((v - v0) / (v1 - v0)) * (t1 - t0) + t0
    if v > v2:
        return t1 - ((v - v2) / (v3 - v2)) * (t1 - t2)
    return t1


def _gear_pwa(v: float) -> int:
    """PwaGearVehicle.get_gear_from_velocity (models.py:494-515) with v_gear_lim (:401-403)."""
    lim = [(_VH[i] - _VL[i]) / 2 + _VL[i] for i in range(1, 6)]
    for i in range(4):
        if lim[i] <= v < lim[i + 1]:
            return i + 2
    return 1 if v < lim[0] else 6


def env_step(x, u, masses, leader_state, u_prev=None, gears=None, leader_index: int = 0,
             real_vehicle_as_reference: bool = False, cfg: Cfg | None = None, ts: float = 1.0,
             quadratic: bool = True):
    """PlatoonEnv.step for one platoon (env.py:126-212; models.py:99-125, 236-257): returns
    (x_next (2n,), stage cost, violation 0/100, ok).  gears None: the PWA-gear model's gear of
    each velocity (env.py:198-204).  quadratic=False: lin_cost = ||Q e||_1 (env.py:122-124)."""
    cfg = cfg or Cfg()
    x = np.asarray(x, dtype=float).reshape(-1).copy()
    u = np.asarray(u, dtype=float).reshape(-1)
    n = len(u)
    up = u if u_prev is None else np.asarray(u_prev, dtype=float).reshape(-1)
    Q = np.diag([1.0, 0.1])  # PlatoonEnv.Q_x (env.py:16); Q_u = 1, Q_du = 0 (env.py:17-18)
    sp = lambda xi: np.array([-cfg.d0 - cfg.t0 * xi[1], 0.0])  # noqa: E731  spacing_policy.spacing
    xs = [x[2 * i:2 * i + 2] for i in range(n)]
    ref = np.asarray(leader_state, dtype=float).reshape(2)
    stage = (lambda e: float(e @ Q @ e)) if quadratic else (lambda e: float(np.abs(Q @ e).sum()))
    e = xs[0] - ref - sp(xs[0]) if real_vehicle_as_reference else xs[leader_index] - ref
    cost = stage(e)
    for i in range(1, n):
        e = xs[i] - xs[i - 1] - sp(xs[i])
        cost += stage(e)
    if quadratic:
        cost += sum(1.0 * u[i] ** 2 for i in range(n)) + sum(0.0 * (u[i] - up[i]) ** 2 for i in range(n))
    else:
        cost += sum(abs(1.0 * u[i]) for i in range(n)) + sum(abs(0.0 * (u[i] - up[i])) for i in range(n))
    close = any(xs[i][0] - xs[i + 1][0] < cfg.d_safe for i in range(n - 1))
    if real_vehicle_as_reference and ref[0] - xs[0][0] < cfg.d_safe:
        close = True
    j = [int(g) for g in gears] if gears is not None else [_gear_pwa(xs[i][1]) for i in range(n)]
    dt = ts / 10
    ok = True
    try:
        for _ in range(10):
            for i in range(n):
                p, v = x[2 * i], x[2 * i + 1]
                a0, a1 = v, -(0.5 * v ** 2) / masses[i] - 0.01 * 9.8
                b1 = _traction(v, j[i]) / masses[i]
                x[2 * i], x[2 * i + 1] = p + dt * (a0 + 0.0 * u[i]), v + dt * (a1 + b1 * u[i])
    except RuntimeError:
        ok = False
    return x, cost, 100 if close else 0, ok
