"""Known answers derived from the reference's constants; no GPU needed.

Pins both restatements of the model layer -- the product's (hvp.models / hvp.env) and the
oracle's (oracle/oracle.py) -- to the same numbers.
"""

from __future__ import annotations

import json
import os

import numpy as np
import pytest

import oracle as O
from golden_io import GOLDEN

KA = json.load(open(os.path.join(GOLDEN, "known_answers.json")))


def test_seed_derivation():
    from hvp.env import derive_env_seed

    assert derive_env_seed(0) == 2968811710 == KA["seed0_env_seed"]  # model_validation.py:76
    assert O.env_seed(0) == 2968811710


def test_env_init_seed0_n10():
    from hvp.env import derive_env_seed, initial_platoon_state

    want = KA["survey_values"]["env_init_n10_seed0"]
    assert initial_platoon_state(10, derive_env_seed(0)).ravel().tolist() == want
    assert O.env_initial_state(10, 0).tolist() == want


@pytest.mark.parametrize("seed", [0, 1, 7, 123])
def test_env_init_product_equals_oracle(seed):
    from hvp.env import derive_env_seed, initial_platoon_state

    for n in (1, 2, 5, 10, 20):
        assert initial_platoon_state(n, derive_env_seed(seed)).ravel().tolist() == O.env_initial_state(n, seed).tolist()


def test_gear_pwa_tables_m800():
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    d = veh.get_discrete_system(1)
    sv = KA["survey_values"]
    ad = [round(a[1, 1], 6) for a in d["A"]]
    assert ad == [sv["Ad22"][0]] * 4 + [sv["Ad22"][1]] * 3
    assert [round(b[1, 0], 5) for b in d["B"]] == [round(v, 5) for v in sv["Bd2"]]
    assert [round(c[1, 0], 6) for c in d["c"]] == [sv["cd2"][0]] * 4 + [sv["cd2"][1]] * 3
    assert np.allclose(veh.v_gear_lim, KA["v_gear_lim"])
    assert np.isclose(veh.alpha, KA["alpha"])
    # the oracle's independent restatement gives the same tables
    g = O.gear_pwa_system(800.0)
    for r in range(7):
        assert np.allclose(d["A"][r], g["A"][r], rtol=0, atol=1e-15)
        assert np.allclose(d["B"][r].ravel(), g["B"][r], rtol=0, atol=1e-15)
        assert np.allclose(d["c"][r].ravel(), g["c"][r], rtol=0, atol=1e-15)
        assert np.allclose(d["S"][r], g["S"][r]) and np.allclose(d["T"][r].ravel(), g["T"][r])


def test_friction_continuity_at_alpha():
    """PWA friction pieces meet at alpha (c1 alpha == c2 alpha + d): regions 3/4 coincide there."""
    from hvp.models import PwaFrictionVehicle as V

    assert np.isclose(V.c1 * V.alpha, V.c2 * V.alpha + V.d)


def test_region_gear_map_and_gear_from_velocity():
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    assert list(veh.REGION_GEAR) == KA["region_gear"]
    lims = KA["v_gear_lim"]
    assert veh.get_gear_from_velocity(5.0) == 1
    assert veh.get_gear_from_velocity(lims[0]) == 2  # half-open bands (models.py:494-515)
    assert veh.get_gear_from_velocity(lims[-1]) == 6
    assert veh.get_gear_from_velocity(20.0) == 4


def test_leader_trajectories():
    from hvp.params import ConstantVelocityLeaderTrajectory, StopAndGoLeaderTrajectory

    x = ConstantVelocityLeaderTrajectory(3000, 20, 200, 1).get_leader_trajectory()
    assert x.shape == (2, 200) and x[0, 0] == 3000 and x[0, 199] == 3000 + 199 * 20 and np.all(x[1] == 20)
    sg = StopAndGoLeaderTrajectory(3000, 20, 10, [30, 50], 200, 1, vf=30).get_leader_trajectory()
    assert sg[1, 30] == 20 and sg[1, 31] == 10 and sg[1, 50] == 10 and sg[1, 51] == 30
    assert sg[0, 31] == sg[0, 30] + 20 and sg[0, 32] == sg[0, 31] + 10


def test_nonlinear_plant_step():
    """Vehicle.step (models.py:114-125) with the traction curve (models.py:30-51)."""
    from hvp.models import GearTransmission, Platoon

    gt = GearTransmission()
    assert np.isclose(gt.get_traction(10.0, 3), 2115.6)  # plateau of gear 3
    p = Platoon(2, "pwa_gear")
    x = np.array([[100.0], [15.0], [50.0], [15.0]])
    xn = p.step_platoon(x, np.array([[0.0], [0.0]]), np.array([[3], [3]]), 1.0)
    # zero throttle: 10 sub-steps of the friction-only dynamics
    v, pos = 15.0, 100.0
    for _ in range(10):
        pos, v = pos + 0.1 * v, v + 0.1 * (-(0.5 * v * v) / 800 - 0.01 * 9.8)
    assert np.isclose(xn[0, 0], pos) and np.isclose(xn[1, 0], v)
