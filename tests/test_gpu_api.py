"""The reference-shaped API on the GPU: LocalMpcMld.solve_mpc, MldAgent, the batched
TrackingDecentMldCoordinator and a short closed-loop simulate()."""

from __future__ import annotations

import numpy as np
import pytest

import oracle as O
from instances import split_params

pytestmark = pytest.mark.gpu


def test_local_mpc_solve_mpc_matches_oracle(gpu_available):
    from hvp.models import PwaGearVehicle
    from hvp.mpc import LocalMpcMld

    N = 5
    veh = PwaGearVehicle(800)
    m = LocalMpcMld(N, veh.get_discrete_system(1), is_front=False, is_trailer=False, gears=veh.REGION_GEAR)
    x = O.env_initial_state(3, 0).astype(float)
    xf = O.constant_velocity_prediction(x[0], x[1], N)
    xb = O.constant_velocity_prediction(x[4], x[5], N)
    m.set_x_front(xf)
    m.set_x_back(xb)
    u0, info = m.solve_mpc(x[2:4].reshape(2, 1))
    ref = O.solve_miqp(O.gear_pwa_system(800.0), O.Cfg(), N, O.role_bits(1, 3), x[2:4], xf, xb, np.zeros((2, N + 1)))
    assert u0.shape == (1, 1) and info["u"].shape == (1, N) and info["x"].shape == (2, N + 1)
    assert np.abs(info["u"][0] - ref.u).max() <= 1e-6
    assert abs(info["cost"] - ref.cost) <= 1e-9 * abs(ref.cost)
    # nodes: QPs of the branch-and-bound search (Gurobi NodeCount analogue), far below the
    # number of sequences an exhaustive search would solve
    assert info["bin_vars"] == 7 * N and 0 < info["nodes"] < ref.n_candidates and info["run_time"] > 0
    assert list(m.gears_pred[0].astype(int)) == [PwaGearVehicle.REGION_GEAR[r] for r in ref.sigma]


def test_infeasible_raises_or_returns_zeros(gpu_available):
    from hvp.models import PwaGearVehicle
    from hvp.mpc import LocalMpcMld

    N = 5
    veh = PwaGearVehicle(800)
    m = LocalMpcMld(N, veh.get_discrete_system(1), is_front=True, is_leader=True, is_trailer=False)
    lead = np.stack([9950 + 40 * np.arange(N + 1), np.full(N + 1, 40.0)])
    m.set_leader_x(lead)
    m.set_x_back(O.constant_velocity_prediction(9790, 30, N))
    with pytest.raises(RuntimeError):
        m.solve_mpc(np.array([[9870.0], [30.0]]))  # the position box cannot be respected
    u0, info = m.solve_mpc(np.array([[9870.0], [30.0]]), raises=False)
    assert np.all(u0 == 0) and info["cost"] == float("inf")


def test_closed_loop_simulate(gpu_available):
    from hvp.decent import simulate
    from hvp.params import Sim

    class Short(Sim):
        n = 4
        N = 5
        ep_len = 12

    X, U, R, agent, env = simulate(Short(), seed=1)
    # the stage cost is a (1, 1) array as PlatoonEnv.get_stage_cost computes it (env.py:126-212;
    # results_analysis/perf_n.py reads sum(R)[0, 0])
    assert X.shape == (13, 8) and U.shape == (12, 4) and np.asarray(R).shape == (12, 1, 1)
    assert np.all(np.abs(U) <= 1 + 1e-9)
    assert (agent.solve_times[:12] > 0).all() and (agent.node_counts[:12] >= 1).all()
    # the first action is the batched solution of the t = 0 problems, identical to the oracle
    x0 = X[0]
    lead = np.stack([3000 + 20.0 * np.arange(6), np.full(6, 20.0)])
    for i in range(4):
        xf = O.constant_velocity_prediction(x0[2 * i - 2], x0[2 * i - 1], 5) if i else np.zeros((2, 6))
        xb = O.constant_velocity_prediction(x0[2 * i + 2], x0[2 * i + 3], 5) if i < 3 else np.zeros((2, 6))
        ref = O.solve_miqp(O.gear_pwa_system(800.0), O.Cfg(), 5, O.role_bits(i, 4), x0[2 * i:2 * i + 2], xf, xb,
                           lead if i == 0 else np.zeros((2, 6)))
        assert abs(U[0][i] - ref.u[0]) <= 1e-6


def test_local_mpc_gear_matches_oracle_and_evaluates(gpu_available):
    """LocalMpcGear on pwa_friction (fleet_decent_mld.py:226-253, mpcs/mpc_gear.py): returns
    [u_g0; gear0], info["u"] = vstack(u_g, gears), gears_pred; evaluate_cost of the optimal
    (u_g, gears) reproduces the optimal cost, and an infeasible throttle gives 'inf'."""
    from hvp.models import PwaFrictionVehicle
    from hvp.mpc import LocalMpcGear

    N = 5
    veh = PwaFrictionVehicle(800)
    g = O.gear_friction_mld_system(800.0)
    x = O.env_initial_state(3, 2).astype(float)
    xf = O.constant_velocity_prediction(x[0], x[1], N)
    xb = O.constant_velocity_prediction(x[4], x[5], N)
    m = LocalMpcGear(N, veh.get_discrete_system(1))
    m.set_x_front(xf)
    m.set_x_back(xb)
    u0, info = m.solve_mpc(x[2:4].reshape(2, 1))
    ref = O.solve_miqp(g, O.Cfg(), N, O.role_bits(1, 3), x[2:4], xf, xb, np.zeros((2, N + 1)))
    assert ref.status == 0
    assert u0.shape == (2, 1) and info["u"].shape == (2, N)
    assert np.abs(info["u"][0] - ref.u).max() <= 1e-6
    assert list(info["u"][1].astype(int)) == list(g["gear"][ref.sigma])
    assert abs(info["cost"] - ref.cost) <= 1e-9 * abs(ref.cost)
    assert info["bin_vars"] == 8 * N
    assert np.array_equal(m.gears_pred, info["u"][[1]])
    c = m.evaluate_cost(x[2:4].reshape(2, 1), info["u"][[0]], info["u"][[1]])
    assert abs(c - ref.cost) <= 1e-9 * abs(ref.cost)
    # full throttle in first gear at ~20 m/s is outside gear 1's window -> infeasible
    assert m.evaluate_cost(x[2:4].reshape(2, 1), np.ones((1, N)), np.ones((1, N))) == "inf"


def test_closed_loop_simulate_gear_model(gpu_available):
    from hvp.decent import simulate
    from hvp.params import Sim

    class ShortGear(Sim):
        n = 3
        N = 5
        ep_len = 8
        vehicle_model_type = "pwa_friction"

    X, U, R, agent, env = simulate(ShortGear(), seed=3)
    assert X.shape == (9, 6) and U.shape == (8, 6)
    assert np.all(np.abs(U[:, :3]) <= 1 + 1e-9)
    assert set(np.unique(U[:, 3:]).astype(int)) <= set(range(1, 7))
