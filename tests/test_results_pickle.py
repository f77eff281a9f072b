"""The results files of ``simulate(save=True)`` read back the way the reference's analysis
scripts read them.

Writer: 7 sequential ``pickle.dump`` calls X, U, R, solve_times, node_counts, violations,
leader_x (fleet_decent_mld.py:548-559; fleet_naive_admm.py, fleet_cent_mld.py alike; g_admm
dumps 0 for the node counts, fleet_g_admm.py:435-437).  Reader: results_analysis/perf_n.py:78-91
-- 7 ``pickle.load`` calls in that order, then ``sum(R)[0, 0]``, ``min/max(solve_times)[0]``,
``sum(solve_times)[0] / len(solve_times)``, ``max(node_counts)[0]``, ``sum(violations) / 100``.
The files are written by this repository's own code (a trusted pickle round trip).
"""

from __future__ import annotations

import glob
import pickle

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sim(n: int, N: int, ep_len: int):
    from hvp.params import ConstantSpacingPolicy, ConstantVelocityLeaderTrajectory, Params, Sim

    class Small(Sim):
        pass

    Small.n, Small.N, Small.ep_len = n, N, ep_len
    Small.spacing_policy = ConstantSpacingPolicy(50)
    Small.leader_trajectory = ConstantVelocityLeaderTrajectory(p=3000, v=20, trajectory_len=ep_len + 50, ts=Params.ts)
    Small.id = f"test_n_{n}_N_{N}"
    return Small()


def _read_like_perf_n(path: str):
    with open(path, "rb") as file:  # results_analysis/perf_n.py:78-84
        X = pickle.load(file)
        U = pickle.load(file)
        R = pickle.load(file)
        solve_times = pickle.load(file)
        node_counts = pickle.load(file)
        violations = pickle.load(file)
        leader_state = pickle.load(file)
        assert file.read() == b""  # exactly 7 objects
    return X, U, R, solve_times, node_counts, violations, leader_state


@pytest.mark.parametrize("controller", ["decent", "admm", "cent"])
def test_simulate_pickle_reads_like_perf_n(gpu_available, tmp_path, monkeypatch, controller):
    import importlib

    monkeypatch.chdir(tmp_path)
    n, N, T = 3, 5, 6
    sim = _sim(n, N, T)
    mod = importlib.import_module(f"hvp.{controller}")
    kw = {"admm_iters": 4} if controller == "admm" else {}
    mod.simulate(sim, save=True, seed=3, **kw)
    files = glob.glob(str(tmp_path / "*.pkl"))
    assert len(files) == 1
    X, U, R, solve_times, node_counts, violations, leader_state = _read_like_perf_n(files[0])
    assert np.asarray(X).shape == (T + 1, 2 * n)
    assert np.asarray(U).shape[0] == T
    # the analysis expressions of perf_n.py:86-91
    track = sum(R)[0, 0]
    assert np.isfinite(track) and track > 0
    assert min(solve_times)[0] >= 0 and max(solve_times)[0] >= min(solve_times)[0]
    assert np.isfinite(sum(solve_times)[0] / len(solve_times))
    assert len(solve_times) == T
    assert max(node_counts)[0] >= 1
    assert sum(violations) / 100 >= 0 and len(violations) == T
    assert np.asarray(leader_state).shape == (2, T + 50)


def test_gadmm_pickle_has_seven_objects(gpu_available, tmp_path, monkeypatch):
    from hvp import gadmm

    monkeypatch.chdir(tmp_path)
    n, N, T = 3, 5, 3
    gadmm.simulate(_sim(n, N, T), save=True, seed=3, admm_iters=10)
    (path,) = glob.glob(str(tmp_path / "*.pkl"))
    X, U, R, solve_times, node_counts, violations, leader_state = _read_like_perf_n(path)
    assert node_counts == 0  # fleet_g_admm.py:435-437 dumps 0
    assert np.isfinite(sum(R)[0, 0]) and len(solve_times) == T and len(violations) == T
