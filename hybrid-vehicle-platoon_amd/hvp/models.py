"""Vehicle / platoon models: the PWA tables the hot path is condensed from, plus the
nonlinear plant the environment integrates.

Restates the behaviour of the reference's ``models.py`` (numpy only, no gurobipy):

* ``GearTransmission.get_traction``      <- models.py:10-51   (traction curve per gear)
* ``Vehicle`` constants / ``step``        <- models.py:54-125  (nonlinear Euler step)
* ``Vehicle.get_gear_from_velocity``      <- models.py:161-174
* ``Platoon`` / ``step_platoon``          <- models.py:199-269 (10 Euler substeps)
* ``PwaFrictionVehicle``                  <- models.py:272-387 (2-region friction PWA)
* ``PwaGearVehicle``                      <- models.py:390-556 (7-region gear PWA)
* ``get_discrete_system``                 <- models.py:370-387 + dmpcrl ``forward_euler``
  (Ad = I + ts*A, Bd = ts*B, cd = ts*c, the same rule ``step_pwa`` uses at models.py:528-533)

The returned system dicts use the reference's keys ``S R T A B c D E F G`` with lists of
numpy arrays, so they can be handed to :class:`hvp.mpc.LocalMpcMld` exactly like the
reference hands them to ``MpcMld``.
"""

from __future__ import annotations

import warnings
from typing import Literal

import numpy as np

# Traction curve of each gear: three force levels and four velocity knots (models.py:13-28).
_TRACTION_T = (
    (253.54, 4056.7, 3042.0),
    (184.0, 2944.75, 2208.55),
    (132.22, 2115.6, 1586.7),
    (100.0 / 415.0, 1605.0, 1205.0),
    (72.88, 1166.0, 874.7),
    (52.4, 838.0, 628.3),
)
_TRACTION_V = (
    (2.0706, 4.12158, 9.29, 12.38),
    (2.85, 5.675, 12.7956, 17.06),
    (3.9705, 7.90316, 17.8105, 23.7474),
    (5.228, 10.42, 23.454, 31.2704),
    (7.203, 14.335, 32.31, 43.0802),
    (10.027, 19.956, 44.978, 59.9715),
)


class GearTransmission:
    """Piecewise-linear traction force F(v, gear) (rise, plateau, fall)."""

    t = _TRACTION_T
    v = _TRACTION_V

    def get_traction(self, v: float, j: int) -> float:
        if not 1 <= j <= 6:
            raise RuntimeError(f"Gear value out of range 1 - 6: {j}.")
        if v < _TRACTION_V[0][0] or v > _TRACTION_V[-1][-1]:
            raise RuntimeError(f"Velocity value out of range: {v}.")
        (v0, v1, v2, v3), (f_lo, f_top, f_end) = _TRACTION_V[j - 1], _TRACTION_T[j - 1]
        if v <= v0 or v >= v3:
            raise RuntimeError(f"Velocity {v} out of range {v0} - {v3} for gear {j}.")
        if v < v1:
            return f_lo + (f_top - f_lo) * (v - v0) / (v1 - v0)
        if v > v2:
            return f_top - (f_top - f_end) * (v - v2) / (v3 - v2)
        return f_top


# keep the reference's (misspelt) class name available for drop-in imports
GearTransimission = GearTransmission


class Vehicle:
    """Nonlinear hybrid vehicle: x = (position, velocity), u = normalised throttle."""

    nx_l = 2
    nu_l = 1
    c_fric = 0.5
    mu = 0.01
    grav = 9.8
    w_min = 105
    w_max = 630
    p = [14.203, 10.310, 7.407, 5.625, 4.083, 2.933]
    b = [4057, 2945, 2116, 1607, 1166, 838]  # max traction force per gear
    vl = [3.94, 5.43, 7.56, 9.96, 13.70, 19.10]
    vh = [9.46, 13.04, 18.15, 23.90, 32.93, 45.84]
    v_min, v_max = vl[0], vh[-1]
    u_min, u_max = -1.0, 1.0
    p_min, p_max = 0.0, 10000.0
    Te_max = 80

    def __init__(self, m: float = 800) -> None:
        self.m = m
        self.gear_model = GearTransmission()

    # continuous-time drift and input gain of the nonlinear model (models.py:99-112)
    def _drift(self, v: float) -> tuple[float, float]:
        return v, -(self.c_fric * v * v) / self.m - self.mu * self.grav

    def step(self, x: np.ndarray, u: float, j: int, ts: float) -> np.ndarray:
        """One explicit Euler step of the nonlinear model (models.py:114-125)."""
        # the reference tests |u| against 1 + 1e5 (sic, models.py:116) -- kept as is
        if abs(u) > 1 + 1e5:
            raise ValueError("Control u is bounded -1 <= u <= 1.")
        v = float(x[1, 0])
        if v < _TRACTION_V[0][0] or v > _TRACTION_V[-1][-1]:
            raise RuntimeError(f"Velocity {v} of vehicle exceeds true model bounds.")
        dp, dv = self._drift(v)
        dv += self.gear_model.get_traction(v, j) / self.m * u
        return x + ts * np.array([[dp], [dv]])

    def get_gear_from_velocity(self, v: float) -> int:
        if v < self.v_min or v > self.v_max:
            warnings.warn(f"Velocity {v} is not within bounds {self.v_min}/{self.v_max}")
            return 1 if v < self.v_min else 6
        for g, (lo, hi) in enumerate(zip(self.vl, self.vh)):
            if lo < v < hi:
                return g + 1
        raise ValueError(f"No gear found for velocity {v}")

    def get_u_for_constant_vel(self, v: float, j: int) -> float:
        if not 1 <= j <= 6:
            raise ValueError(f"{j} is not a valid gear.")
        return (self.c_fric * v * v + self.mu * self.m * self.grav) / self.b[j - 1]

    def get_discrete_system(self, ts: float) -> dict:
        # the nonlinear gear MPC (MpcNonlinearGear, a non-convex MIQCP) is out of scope
        raise NotImplementedError("nonlinear vehicle model has no PWA/MLD system dict")

    def box_constraints(self):
        """D x <= E, F u <= G (models.py:146-151, identical in every vehicle class)."""
        D = np.array([[1, 0], [-1, 0], [0, 1], [0, -1]])
        E = np.array([[self.p_max], [-self.p_min], [self.v_max], [-self.v_min]])
        F = np.array([[1], [-1]])
        G = np.array([[self.u_max], [-self.u_min]])
        return D, E, F, G


def _col(*vals) -> np.ndarray:
    return np.array(vals, dtype=float).reshape(-1, 1)


class PwaFrictionVehicle(Vehicle):
    """Friction c*v^2 replaced by two affine pieces split at v_max/2 (models.py:272-332)."""

    beta = (3 * Vehicle.c_fric * Vehicle.v_max**2) / 16
    alpha = Vehicle.v_max / 2
    c1 = beta / alpha
    c2 = (Vehicle.c_fric * Vehicle.v_max**2 - beta) / (Vehicle.v_max - alpha)
    d = beta - alpha * c2

    def __init__(self, m: float = 800) -> None:
        super().__init__(m)
        self.system = self.build_friction_pwa_system(m)

    def _pieces(self, mass: float):
        """(A, c) for the low- and high-velocity friction piece."""
        A_lo = np.array([[0.0, 1.0], [0.0, -self.c1 / mass]])
        A_hi = np.array([[0.0, 1.0], [0.0, -self.c2 / mass]])
        c_lo = _col(0.0, -self.mu * self.grav)
        c_hi = _col(0.0, -self.mu * self.grav - self.d / mass)
        return (A_lo, c_lo), (A_hi, c_hi)

    def _assemble(self, S, T, A, B, c):
        D, E, F, G = self.box_constraints()
        R = [np.zeros((2, 1)) for _ in S]
        return {"S": S, "R": R, "T": T, "A": A, "B": B, "c": c, "D": D, "E": E, "F": F, "G": G}

    def build_friction_pwa_system(self, mass: float, bound_velocity: bool = False):
        (A_lo, c_lo), (A_hi, c_hi) = self._pieces(mass)
        if bound_velocity:
            S = [np.array([[0, 1], [0, -1]])] * 2
            T = [_col(self.alpha, -self.v_min), _col(self.v_max, -self.alpha)]
        else:
            S = [np.array([[0, 1], [0, 0]]), np.array([[0, 0], [0, -1]])]
            T = [_col(self.alpha, 0), _col(0, -self.alpha)]
        Bm = _col(0.0, 1.0 / mass)
        return self._assemble([s.copy() for s in S], T, [A_lo, A_hi], [Bm, Bm.copy()], [c_lo, c_hi])

    def get_discrete_system(self, ts: float) -> dict:
        """Forward-Euler discretisation of every region (models.py:370-387)."""
        disc = dict(self.system)
        disc["A"] = [np.eye(2) + ts * A for A in self.system["A"]]
        disc["B"] = [ts * B for B in self.system["B"]]
        disc["c"] = [ts * c for c in self.system["c"]]
        return disc

    def find_region(self, x: np.ndarray, u: np.ndarray) -> int:
        """First region with S x + R u <= T + [0, 1e-4] (models.py:519-526 buffer rule)."""
        buf = _col(0.0, 1e-4)
        for i, (S, R, T) in enumerate(zip(self.system["S"], self.system["R"], self.system["T"])):
            if np.all(S @ x + R @ u <= T + buf):
                return i
        raise RuntimeError(f"Didn't find PWA region for x: {x} and u: {u}")


class PwaGearVehicle(PwaFrictionVehicle):
    """Seven velocity regions: friction piece x gear (models.py:390-492).

    Region r has velocity interval [lim[r-1], lim[r]] with lim = (v_gear_lim[0..2], alpha,
    v_gear_lim[3..4]); gear per region is (1, 2, 3, 4, 4, 5, 6); friction switches at alpha.
    """

    REGION_GEAR = (1, 2, 3, 4, 4, 5, 6)

    def __init__(self, m: float = 800) -> None:
        Vehicle.__init__(self, m)
        self.system = self.build_gear_pwa_system(m)

    def build_gear_pwa_system(self, mass: float, bound_velocity: bool = False):
        # gear-switch velocities: midpoints of the gear bands 2..6 (models.py:401-403)
        self.v_gear_lim = [(self.vh[i] - self.vl[i]) / 2 + self.vl[i] for i in range(1, 6)]
        g = self.v_gear_lim
        cuts = [g[0], g[1], g[2], self.alpha, g[3], g[4]]  # 6 cuts -> 7 regions
        lower = [None] + cuts
        upper = cuts + [None]
        S, T = [], []
        for lo, hi in zip(lower, upper):
            if lo is None and not bound_velocity:
                S.append(np.array([[0, 1], [0, 0]]))
                T.append(_col(hi, 0))
            elif hi is None and not bound_velocity:
                S.append(np.array([[0, 0], [0, -1]]))
                T.append(_col(0, -lo))
            else:
                S.append(np.array([[0, 1], [0, -1]]))
                T.append(_col(self.v_max if hi is None else hi, -(self.v_min if lo is None else lo)))
        (A_lo, c_lo), (A_hi, c_hi) = self._pieces(mass)
        A, c, B = [], [], []
        for r, gear in enumerate(self.REGION_GEAR):
            high_friction = r >= 4
            A.append((A_hi if high_friction else A_lo).copy())
            c.append((c_hi if high_friction else c_lo).copy())
            B.append(_col(0.0, self.b[gear - 1] / mass))
        return self._assemble(S, T, A, B, c)

    def get_gear_from_velocity(self, v: float) -> int:
        """Gear implied by the PWA regions (half-open bands, models.py:494-515)."""
        g = self.v_gear_lim
        for i in range(4):
            if g[i] <= v < g[i + 1]:
                return i + 2
        if v < g[0]:
            if v < self.v_min:
                warnings.warn(f"Velocity {v} is below min {self.v_min}; using first gear.")
            return 1
        if v >= g[-1]:
            if v > self.v_max:
                warnings.warn(f"Velocity {v} is above max {self.v_max}; using last gear.")
            return 6
        raise RuntimeError(f"Didn't find any gear for the given speed {v}")

    def step_pwa(self, x: np.ndarray, u: np.ndarray, ts: float) -> np.ndarray:
        r = self.find_region(x, u)
        s = self.system
        return (np.eye(2) + ts * s["A"][r]) @ x + ts * s["B"][r] @ u + ts * s["c"][r]

    def get_u_for_constant_vel(self, v: float) -> float:
        x = _col(0.0, v)
        r = self.find_region(x, np.zeros((1, 1)))
        s = self.system
        return (-s["A"][r][1, 1] * v - s["c"][r][1, 0]) / s["B"][r][1, 0]


_VEHICLE_TYPES = {
    "nonlinear": Vehicle,
    "pwa_friction": PwaFrictionVehicle,
    "pwa_gear": PwaGearVehicle,
}


class Platoon:
    """n vehicles of one model type (models.py:199-269)."""

    nx_l = Vehicle.nx_l
    nu_l = Vehicle.nu_l

    def __init__(
        self,
        n: int,
        vehicle_type: Literal["nonlinear", "pwa_friction", "pwa_gear"],
        masses: list | None = None,
    ) -> None:
        if vehicle_type not in _VEHICLE_TYPES:
            raise ValueError(f"{vehicle_type} is not a valid vehicle type.")
        cls = _VEHICLE_TYPES[vehicle_type]
        if masses is not None and len(masses) != n:
            raise ValueError(f"Required {n} vehicles masses. Got {len(masses)}.")
        self.n = n
        self.vehicles = [cls(m=masses[i]) if masses is not None else cls() for i in range(n)]

    def get_vehicles(self):
        return self.vehicles

    def step_platoon(self, x: np.ndarray, u: np.ndarray, j: np.ndarray, ts: float) -> np.ndarray:
        if x.shape != (self.nx_l * self.n, 1) or u.shape != (self.n, 1) or j.shape != (self.n, 1):
            raise ValueError("Dimension error in x, u, or j.")
        dt = ts / 10  # 10 Euler sub-steps per sample (models.py:245-246)
        x = np.asarray(x, dtype=float)
        for _ in range(10):
            x = np.vstack(
                [
                    veh.step(x[2 * i : 2 * i + 2], float(u[i, 0]), int(j[i, 0]), dt)
                    for i, veh in enumerate(self.vehicles)
                ]
            )
        return x

    def get_gear_from_vehicle_velocity(self, i: int, v: float) -> int:
        veh = self.vehicles[i]
        if not isinstance(veh, PwaGearVehicle):
            raise RuntimeError(f"Gear from velocity asked but vehicle {i} is not a PWA gear vehicle.")
        return veh.get_gear_from_velocity(v)

    def get_vehicle_system_dicts(self, ts: float) -> list[dict]:
        return [veh.get_discrete_system(ts) for veh in self.vehicles]
