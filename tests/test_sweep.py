"""The n x N x seed sweep driver (hvp.sweep; configs[4], the reference's n_sweep_3.py).

CPU: the shard map covers every (n, N, seed) exactly once for any world size, and a world-2
gloo job agrees (each rank computes its share, the gathered shares partition the grid).
GPU: a sweep point's device closed loop reproduces the host simulate() of the decentralised
controller (hvp.decent.simulate, the reference's fleet_decent_mld.simulate surface) seed by seed,
and its results files read back like results_analysis/perf_n.py reads them.
"""

from __future__ import annotations

import glob
import os
import pickle

import numpy as np
import pytest

POINTS = [(n, N) for N in (5, 10, 15) for n in (5, 10, 15, 20)]


@pytest.mark.parametrize("world", [1, 2, 3, 8, 13])
def test_shard_partitions_the_grid(world):
    from hvp.sweep import shard

    seen = []
    for r in range(world):
        for n, N, seeds in shard(POINTS, 100, r, world):
            seen += [(n, N, s) for s in seeds]
    assert sorted(seen) == sorted((n, N, s) for n, N in POINTS for s in range(100))
    # every rank does a share of every point (work balance across cheap and expensive points)
    if world <= 100:
        assert all({(n, N) for n, N, _ in shard(POINTS, 100, r, world)} == set(POINTS) for r in range(world))


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist

    from hvp.sweep import shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    mine = [(n, N, s) for n, N, seeds in shard(POINTS, 100, rank, world) for s in seeds]
    out = [None] * world
    dist.all_gather_object(out, mine)
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_shard_map_gloo_world2():
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=120)
    for p in procs:
        p.join(60)
    allu = out[0] + out[1]
    assert len(allu) == len(set(allu)) == len(POINTS) * 100
    assert not set(out[0]) & set(out[1])


@pytest.mark.gpu
def test_sweep_point_matches_host_simulate(gpu_available, tmp_path):
    from hvp import decent
    from hvp.params import Sim_n_task_2
    from hvp.sweep import run_point

    n, N, T, seeds = 4, 5, 6, [0, 1, 2]
    res = run_point(n, N, seeds, ep_len=T, out_dir=str(tmp_path))
    for k, s in enumerate(seeds):
        sim = Sim_n_task_2(n, seed=s, N=N)
        sim.ep_len = T
        X, U, R, agent, env = decent.simulate(sim, seed=s)
        np.testing.assert_allclose(res["X"][:, k], np.asarray(X).reshape(T + 1, -1), rtol=0, atol=1e-6)
        np.testing.assert_allclose(res["U"][:, k], np.asarray(U).reshape(T, -1), rtol=0, atol=1e-6)
        np.testing.assert_allclose(res["R"][:, k], np.asarray(R).reshape(-1), rtol=1e-9)
        assert np.array_equal(res["viol"][:, k], np.asarray(env.unwrapped.viol_counter[0]))
    files = sorted(glob.glob(os.path.join(tmp_path, "*.pkl")))
    assert len(files) == len(seeds)
    with open(files[0], "rb") as f:  # results_analysis/perf_n.py:78-91
        X, U, R, solve_times, node_counts, violations, leader_state = (pickle.load(f) for _ in range(7))
    assert np.isfinite(sum(R)[0, 0]) and min(solve_times)[0] > 0 and max(node_counts)[0] >= 1
    assert len(violations) == T and np.asarray(leader_state).shape[0] == 2


@pytest.mark.gpu
def test_sweep_warm_incumbent_keeps_the_episodes(gpu_available):
    """N > 8: the previous step's sequences (shifted) tried as incumbents of the next step's local
    searches change the QP counts only -- the closed-loop episodes are bit-identical."""
    from hvp.sweep import run_point

    a = run_point(5, 10, [0, 1, 2, 3], ep_len=6, warm_incumbent=True)
    b = run_point(5, 10, [0, 1, 2, 3], ep_len=6, warm_incumbent=False)
    for k in ("X", "U", "R", "viol"):
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.gpu
def test_run_points_blocks_equal_one_batch(gpu_available):
    """run_points (seed blocks on concurrent host threads / streams) gives every seed the same
    episode as one batch of all seeds: the blocks share nothing (numpy's global generator, which
    the task_2 masses and env.reset seed, is drawn under a lock)."""
    from hvp.sweep import run_point, run_points

    seeds = list(range(8))
    one = run_point(6, 5, seeds, ep_len=5)
    blocks, _ = run_points(6, 5, seeds, ep_len=5, device=0, out_dir=None, estimator="none", streams=2)
    X = np.concatenate([b["X"] for b in blocks], axis=1)
    R = np.concatenate([b["R"] for b in blocks], axis=1)
    np.testing.assert_array_equal(X, one["X"])
    np.testing.assert_array_equal(R, one["R"])


def test_ep_len_beyond_the_leader_trajectory_raises():
    """Sim_n_task_2's leader trajectory holds ep_len (150) + 50 samples: a longer episode is
    refused up front with a clear error (before any device work)."""
    from hvp.sweep import run_point

    with pytest.raises(ValueError, match="leader samples"):
        run_point(5, 10, [0], ep_len=190)
