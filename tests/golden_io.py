"""Loading of the committed golden fixtures for the product-side tests."""

from __future__ import annotations

import glob
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixture_names() -> list[str]:
    """The decentralised local-MIQP fixtures (the ADMM and centralised ones have their own layouts,
    the min_1_norm ones are listed by :func:`l1_fixture_names`)."""
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("admm_", "gadmm_", "cent_", "l1_")))


def l1_fixture_names() -> list[str]:
    """The decentralised local-MILP fixtures of the min_1_norm cost (quadratic_cost=False)."""
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, "l1_*.npz")))


def load(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


class CfgParams:
    """A Params-like class (misc/common_controller_params.py:14-23) built from an oracle cfg vector."""

    def __init__(self, v) -> None:
        v = np.asarray(v, dtype=float)
        self.Q_x = v[0:4].reshape(2, 2)
        self.Q_u = np.array([[v[4]]])
        self.Q_du = np.array([[v[5]]])
        self.w = v[6]
        self.a_acc, self.a_dec, self.ts, self.d_safe = v[7], v[8], v[9], v[10]
        self.tight, self.d0, self.t0 = v[11], v[12], v[13]


def product_problem(fx: dict):
    """hvp_problem + system tables of a fixture, through the product's own table builders."""
    from hvp import tables
    from hvp.models import PwaGearVehicle
    from hvp.params import ConstantTimePolicy

    from hvp.models import PwaFrictionVehicle

    cp = CfgParams(fx["cfg"])
    prob = tables.problem(int(fx["N"]), ConstantTimePolicy(cp.d0, cp.t0), bool(int(fx.get("quadratic", 1))),
                          accel_cnstr_tightening=cp.tight, params=cp)
    systems = []
    for m in fx["masses"]:
        if int(fx.get("model", 0)) == 1:  # LocalMpcGear on pwa_friction
            veh = PwaFrictionVehicle(float(m))
            systems.append(tables.gear_system_from_dict(veh.get_discrete_system(float(cp.ts))))
        else:
            veh = PwaGearVehicle(float(m))
            systems.append(tables.system_from_dict(veh.get_discrete_system(float(cp.ts)), tables.gears_of(veh)))
    return prob, systems


def expected_gears(fx: dict):
    """Gear label per step of the expected solutions."""
    if "exp_gear" in fx:
        return fx["exp_gear"]
    return np.array([1, 2, 3, 4, 4, 5, 6])[fx["exp_region"]]
