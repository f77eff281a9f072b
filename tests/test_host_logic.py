"""Host-side logic of the product package (no GPU): table building, roles, the batched
instance builder, the environment restatement and the drop-in classes' parameter plumbing."""

from __future__ import annotations

import numpy as np
import pytest

import oracle as O
from instances import decent_instances, leader_window


def gear_table(mass=800.0):
    from hvp import tables
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(mass)
    return tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))


def test_system_table_from_reference_dict():
    t = gear_table()
    g = O.gear_pwa_system(800.0)
    assert t.n_regions == 7 and t.ts == 1.0
    assert list(t.gear)[:7] == [1, 2, 3, 4, 4, 5, 6]
    for r in range(7):
        assert t.a[r] == g["A"][r][1, 1] and t.b[r] == g["B"][r][1] and t.c[r] == g["c"][r][1]
    assert t.vlo[0] < -1e299 and t.vhi[6] > 1e299  # unbounded first / last region
    assert np.isclose(t.vhi[0], 9.235) and np.isclose(t.vlo[6], 32.47)
    assert (t.pmin, t.pmax, t.vmin, t.vmax, t.umin, t.umax) == (0.0, 10000.0, 3.94, 45.84, -1.0, 1.0)


def test_table_rejects_unsupported_models():
    from hvp import tables
    from hvp.models import PwaGearVehicle

    d = PwaGearVehicle(800).get_discrete_system(1)
    bad = dict(d)
    bad["S"] = [np.array([[1, 1], [0, 0]])] + list(d["S"][1:])  # position-dependent region
    with pytest.raises(ValueError):
        tables.system_from_dict(bad)
    bad = dict(d)
    bad["B"] = [np.array([[0.1], [1.0]])] + list(d["B"][1:])  # input acting on position
    with pytest.raises(ValueError):
        tables.system_from_dict(bad)


def test_friction_model_table():
    from hvp import tables
    from hvp.models import PwaFrictionVehicle

    t = tables.system_from_dict(PwaFrictionVehicle(900).get_discrete_system(1))
    assert t.n_regions == 2 and np.isclose(t.vhi[0], 22.92) and np.isclose(t.vlo[1], 22.92)


@pytest.mark.parametrize("n,leader,rvr", [(2, 0, False), (10, 0, False), (5, 2, False), (5, 0, True), (1, 0, False)])
def test_roles_match_reference_setup(n, leader, rvr):
    from hvp import tables

    for i in range(n):
        assert tables.role_bits(i == 0, i == n - 1, i == leader, rvr) == O.role_bits(i, n, leader, rvr)


@pytest.mark.parametrize("n,N", [(2, 5), (10, 5), (7, 3)])
def test_batched_builder_matches_per_vehicle_builder(n, N):
    from hvp.batched import decent_params_from_states

    states = np.stack([O.env_initial_state(n, s).astype(float) for s in range(5)])
    P, R = decent_params_from_states(states, N, leader_window(N))
    ref = [decent_instances(states[s], N, leader_window(N)) for s in range(5)]
    assert np.array_equal(P, np.concatenate([r[0] for r in ref]))
    assert np.array_equal(R, np.concatenate([r[1] for r in ref]))


def test_two_point_and_saturated_estimators():
    from hvp.batched import extrapolate

    e = extrapolate(100.0, 20.0, 4, 1.0, dv=1.0)
    assert e[1].tolist() == [20, 21, 22, 23, 24] and e[0, 1] == 120 and e[0, 2] == 141
    s = extrapolate(100.0, 20.0, 4, 1.0, dv=1.0, sat=True)
    assert s[1].tolist() == [20, 21, 22, 22, 22]


def test_env_step_cost_and_violations():
    from hvp.env import PlatoonEnv
    from hvp.models import Platoon
    from hvp.params import ConstantSpacingPolicy, ConstantVelocityLeaderTrajectory

    n = 3
    env = PlatoonEnv(n, Platoon(n, "pwa_gear"), ep_len=10,
                     leader_trajectory=ConstantVelocityLeaderTrajectory(3000, 20, 60, 1),
                     spacing_policy=ConstantSpacingPolicy(50))
    x, _ = env.reset(seed=O.env_seed(0))
    assert x.dtype == np.int64 and x.ravel().tolist() == O.env_initial_state(n, 0).tolist()
    u = np.zeros((n, 1))
    xs = np.asarray(x, float)
    want = (xs[0:2].ravel() - [3000, 20]) @ np.diag([1, 0.1]) @ (xs[0:2].ravel() - [3000, 20])
    for i in range(1, n):
        e = xs[2 * i:2 * i + 2].ravel() - xs[2 * i - 2:2 * i].ravel() - [-50, 0]
        want += e @ np.diag([1, 0.1]) @ e
    x1, r, *_ = env.step(u)
    assert np.isclose(r, want)
    assert env.step_counter == 1 and x1.shape == (2 * n, 1)
    # force a violation: vehicles 20 m apart
    env.x = np.array([[3000.0], [20.0], [2980.0], [20.0], [2900.0], [20.0]])
    env.step(u)
    assert env.viol_counter[-1][1] == 100


def test_local_mpc_parameter_plumbing():
    """LocalMpcMld's setters write the params block hvp_solve_batch reads (no solve)."""
    from hvp.models import PwaGearVehicle
    from hvp.mpc import LocalMpcMld

    N = 5
    veh = PwaGearVehicle(800)
    m = LocalMpcMld(N, veh.get_discrete_system(1), is_front=False, is_leader=False, is_trailer=False)
    xf = O.constant_velocity_prediction(3100, 20, N)
    xb = O.constant_velocity_prediction(2900, 20, N)
    m.set_x_front(xf)
    m.set_x_back(xb)
    p = m.params_for(np.array([[3000.0], [21.0]]))
    K = 2 * (N + 1)
    assert p[:2].tolist() == [3000.0, 21.0]
    assert np.array_equal(p[2:2 + K], xf.ravel()) and np.array_equal(p[2 + K:2 + 2 * K], xb.ravel())
    assert m.role == O.role_bits(1, 3)
    assert m.num_bin_vars == 7 * N
    with pytest.raises(ValueError):
        m.set_x_front(np.zeros((2, N)))
    # min_1_norm: the same plumbing, the problem carries quadratic_cost = 0 (hvp_l1.h on the device)
    l1 = LocalMpcMld(N, veh.get_discrete_system(1), quadratic_cost=False)
    assert l1.problem.quadratic_cost == 0 and l1.role == O.role_bits(1, 3)
