"""Multi-process sharding of the benchmark workload (gloo, world_size 2, CPU).

bench.py gives every rank a disjoint seed range and never exchanges solver data; the only
collectives are the timing barrier and the MAX over ranks.  This checks the shard layout and
the aggregation with the same torch.distributed calls on the gloo backend.
"""

from __future__ import annotations

import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, S, n, N, out):
    import sys

    import torch
    import torch.distributed as dist

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "hybrid-vehicle-platoon_amd"))
    sys.path.insert(0, root)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    params, roles = bench.make_inputs(range(rank * S, (rank + 1) * S), n, N)
    # a stand-in "solve time" that differs per rank: the reported time must be the max
    t = torch.tensor([0.1 * (rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    gathered = [torch.zeros(S * n, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(params[:, 0].copy()))
    if rank == 0:
        out.put((float(t.item()), [g.numpy() for g in gathered], params.shape))
    dist.barrier()
    dist.destroy_process_group()


def test_seed_shards_are_disjoint_and_time_is_max_over_ranks():
    world, S, n, N = 2, 6, 4, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, n, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, gathered, shape = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.isclose(t, 0.2)
    assert shape == (S * n, 2 + 6 * (N + 1))
    # rank r owns seeds [r S, (r+1) S): its first-vehicle positions equal the single-process build
    import bench

    full, _ = bench.make_inputs(range(world * S), n, N)
    assert np.array_equal(np.concatenate(gathered), full[:, 0])


def _run_bench(args: list, env_extra: dict | None = None):
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240)


def test_bench_gpus_n_launches_n_ranks():
    """bench.py --gpus 2 without an external launcher starts two ranks itself (gloo in --dry-run),
    prints rank 0's line once with n_gpus 2, and the ranks hold disjoint seed blocks."""
    import json

    r = _run_bench(["--gpus", "2", "--no-cpu", "--dry-run", "--platoons", "7", "--steps", "3"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["backend"] == "gloo" and d["steps"] == 3
    assert d["seed_ranges"] == [[0, 7], [7, 14]]


def test_bench_launcher_fails_when_a_rank_fails():
    """A rank that cannot run makes the launcher exit non-zero (no silent one-GPU line)."""
    r = _run_bench(["--gpus", "2", "--no-cpu", "--dry-run", "--platoons", "-1"])
    assert r.returncode != 0
    r = _run_bench(["--gpus", "2", "--no-cpu", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
