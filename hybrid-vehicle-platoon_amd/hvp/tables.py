"""PWA system dict  ->  solver tables (``hvp_system``) and controller constants (``hvp_problem``).

``system_from_dict`` accepts exactly what the reference hands to ``MpcMld``: the discrete
dict {S,R,T,A,B,c,D,E,F,G} of ``get_discrete_system`` (models.py:370-387, 397-492).  It checks
that the dict has the structure the GPU formulation relies on and raises otherwise:

* regions depend on velocity only (S[:,0] == 0, R == 0), so each region is a closed interval;
* p+ = p + ts v in every region (A[0] = [1, ts], B[0] = c[0] = 0), v+ = a v + b u + c, b > 0;
* D x <= E and F u <= G are boxes on (p, v) and u.
"""

from __future__ import annotations

import numpy as np

from . import _abi
from .params import ConstantSpacingPolicy, ConstantTimePolicy, Params, SpacingPolicy

UNBOUNDED = 1e300


def _interval(rows: np.ndarray, rhs: np.ndarray, col: int) -> tuple[float, float]:
    lo, hi = -UNBOUNDED, UNBOUNDED
    for r, t in zip(rows, rhs):
        others = np.delete(r, col)
        if np.any(others != 0):
            raise ValueError(f"constraint row {r} is not a bound on component {col}")
        s = r[col]
        if s > 0:
            hi = min(hi, t / s)
        elif s < 0:
            lo = max(lo, t / s)
        elif t < 0:
            return 1.0, -1.0  # 0 <= t violated: empty
    return lo, hi


def system_from_dict(sysd: dict, gears=None) -> _abi.HvpSystem:
    S = [np.asarray(s, dtype=float) for s in sysd["S"]]
    R = [np.asarray(r, dtype=float) for r in sysd["R"]]
    T = [np.asarray(t, dtype=float).reshape(-1) for t in sysd["T"]]
    A = [np.asarray(a, dtype=float) for a in sysd["A"]]
    B = [np.asarray(b, dtype=float).reshape(-1) for b in sysd["B"]]
    c = [np.asarray(v, dtype=float).reshape(-1) for v in sysd["c"]]
    nreg = len(S)
    if not 1 <= nreg <= _abi.MAX_REGIONS:
        raise ValueError(f"{nreg} regions not supported (max {_abi.MAX_REGIONS})")
    out = _abi.HvpSystem()
    out.n_regions = nreg
    ts = A[0][0, 1]
    if ts <= 0:
        raise ValueError("expected p+ = p + ts*v with ts > 0")
    out.ts = ts
    for r in range(nreg):
        if np.any(R[r] != 0) or np.any(S[r][:, 0] != 0):
            raise ValueError("regions must depend on the velocity only (S[:,0] == 0, R == 0)")
        if A[r][0, 0] != 1 or A[r][0, 1] != ts or A[r][1, 0] != 0 or B[r][0] != 0 or c[r][0] != 0:
            raise ValueError("expected p+ = p + ts*v in every region")
        if not B[r][1] > 0:
            raise ValueError("expected a positive input gain")
        lo, hi = _interval(S[r], T[r], 1)
        out.a[r], out.b[r], out.c[r] = A[r][1, 1], B[r][1], c[r][1]
        out.vlo[r], out.vhi[r] = lo, hi
        out.gear[r] = int(gears[r]) if gears is not None else r + 1
    D = np.asarray(sysd["D"], dtype=float)
    E = np.asarray(sysd["E"], dtype=float).reshape(-1)
    prow = [i for i in range(D.shape[0]) if D[i, 1] == 0]
    vrow = [i for i in range(D.shape[0]) if D[i, 0] == 0]
    if len(prow) + len(vrow) != D.shape[0]:
        raise ValueError("D x <= E must be a box")
    out.pmin, out.pmax = _interval(D[prow], E[prow], 0)
    out.vmin, out.vmax = _interval(D[vrow], E[vrow], 1)
    F = np.asarray(sysd["F"], dtype=float).reshape(-1, 1)
    G = np.asarray(sysd["G"], dtype=float).reshape(-1)
    out.umin, out.umax = _interval(F, G, 0)
    return out


def gear_system_from_dict(sysd: dict, b=None, vl=None, vh=None) -> _abi.HvpSystem:
    """Solver table of ``MpcGear.setup_gears`` (mpcs/mpc_gear.py:30-114) on a PWA system dict
    (``pwa_friction``: fleet_decent_mld.py:226-253 ``LocalMpcGear``).

    The MIQP has the PWA region binaries delta (2 friction regions) and the gear binaries sigma
    (6 gears) per step; with both fixed it is the convex QP of one *mode* (region r, gear j):

    * u = b_j * u_g (the four big-M rows of :75-96 with sigma_j = 1), so
      v+ = a_r v + (B_r b_j) u_g + c_r;
    * the control box F u <= G is moved onto u_g (:57-76), and the cost penalises u_g
      (setup_cost_and_constraints(self.u_g, ...), fleet_decent_mld.py:241);
    * gear j requires vl_j <= v_k <= vh_j (:98-110), region r its own velocity band.

    So the table holds one entry per non-empty (gear, region) mode, band = gear band ∩ region
    band, input gain B_r b_j and gear label j + 1 -- the search over modes is the search over
    (delta, sigma).  Modes are ordered gear-major (gear 1 first), then by region.
    """
    from .models import Vehicle

    b = list(Vehicle.b if b is None else b)
    vl = list(Vehicle.vl if vl is None else vl)
    vh = list(Vehicle.vh if vh is None else vh)
    base = system_from_dict(sysd)
    modes = []
    for j in range(len(b)):
        for r in range(base.n_regions):
            lo, hi = max(vl[j], base.vlo[r]), min(vh[j], base.vhi[r])
            if lo <= hi:
                modes.append((j, r, lo, hi))
    if len(modes) > _abi.MAX_REGIONS:
        raise ValueError(f"{len(modes)} (gear, region) modes exceed {_abi.MAX_REGIONS}")
    out = _abi.HvpSystem()
    for f in ("ts", "pmin", "pmax", "vmin", "vmax", "umin", "umax"):
        setattr(out, f, getattr(base, f))
    out.n_regions = len(modes)
    for m, (j, r, lo, hi) in enumerate(modes):
        out.a[m], out.b[m], out.c[m] = base.a[r], base.b[r] * b[j], base.c[r]
        out.vlo[m], out.vhi[m] = lo, hi
        out.gear[m] = j + 1
    return out


def gears_of(vehicle) -> list[int]:
    """Gear label per region (PwaGearVehicle: the gear implied by each region)."""
    g = getattr(vehicle, "REGION_GEAR", None)
    return list(g) if g is not None else list(range(1, len(vehicle.system["S"]) + 1))


def spacing_params(policy: SpacingPolicy) -> tuple[float, float]:
    if isinstance(policy, ConstantTimePolicy):
        return policy.d0, policy.t0
    if isinstance(policy, ConstantSpacingPolicy):
        return policy.d0, 0.0
    return float(getattr(policy, "d0", 0.0)), float(getattr(policy, "t0", 0.0))


def problem(N: int, spacing_policy: SpacingPolicy | None = None, quadratic_cost: bool = True,
            accel_cnstr_tightening: float = 0.0, params=Params, max_iter: int = 0, tol: float = 0.0,
            method: int = _abi.METHOD_AUTO) -> _abi.HvpProblem:
    """hvp_problem for LocalMpcMld's cost / constraints (fleet_decent_mld.py:24-31, 61-208)."""
    d0, t0 = spacing_params(spacing_policy or ConstantSpacingPolicy(50))
    p = _abi.HvpProblem()
    p.N = N
    p.quadratic_cost = 1 if quadratic_cost else 0
    Q = np.asarray(params.Q_x, dtype=float)
    p.Qx[:] = [Q[0, 0], Q[0, 1], Q[1, 0], Q[1, 1]]
    p.Qu = float(np.asarray(params.Q_u).reshape(-1)[0])
    p.Qdu = float(np.asarray(params.Q_du).reshape(-1)[0])
    p.w = float(params.w)
    p.a_acc, p.a_dec, p.ts_acc = float(params.a_acc), float(params.a_dec), float(params.ts)
    p.d_safe = float(params.d_safe)
    p.accel_tightening = float(accel_cnstr_tightening)
    p.spacing_d0, p.spacing_t0 = d0, t0
    p.max_iter = max_iter
    p.method = method
    p.tol = tol
    return p


def role_bits(is_front: bool, is_trailer: bool, is_leader: bool, real_vehicle_as_reference: bool = False) -> int:
    """HVP_ROLE_* of one LocalMpcMld (fleet_decent_mld.py:100-153, 191-208)."""
    r = 0
    if not is_front:
        r |= _abi.ROLE_SAFE_FRONT
    if not is_trailer:
        r |= _abi.ROLE_SAFE_BACK
    if not is_front and not is_leader:
        r |= _abi.ROLE_TRACK_FRONT
    if not is_trailer and not is_leader:
        r |= _abi.ROLE_TRACK_BACK
    if is_leader:
        r |= _abi.ROLE_TRACK_LEADER
        if real_vehicle_as_reference:
            r |= _abi.ROLE_LEADER_SPACING
    return r
