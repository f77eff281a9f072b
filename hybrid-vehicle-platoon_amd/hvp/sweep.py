"""The n x N x seed sweep of the decentralised controller (configs[4], the reference's
n_sweep*.py loops over ``simulate(Sim_n_task_2(n, seed), save=True)``) as ONE job on the device.

Every (n, N) point runs its seeds as one batch of platoons in closed loop on the GPU -- the
neighbour predictions (hvp_decent_params_batch), the n local MIQPs of every platoon
(hvp_solve_batch) and PlatoonEnv.step (hvp_env_step_batch) per time step, ``ep_len`` steps --
with the task_2 setting of misc/common_controller_params.py:54-76: per-vehicle masses
U(700, 1000) drawn with ``np.random.seed(seed)``, constant-time spacing (10, 3), the
stop-and-go leader.  Each seed's episode is written as the reference's results file (7 pickles:
X, U, R, solve_times, node_counts, violations, leader_x; fleet_decent_mld.py:548-559), named as
the reference names it, so results_analysis/* reads a sweep directory unchanged.

Multi-GPU: one process per GPU (torch.distributed.run); every rank takes a contiguous share of
the seeds of EVERY point (``shard``), so each rank's work mixes the cheap and the expensive
points alike; no collective in the data path, a gather of the per-rank summaries at the end.
Within a GPU a point's seeds run as ``--streams`` blocks at once (a host thread and HIP stream
each, ``run_points``), so one block's kernels fill the CUs the other's level tails leave.

    python -m hvp.sweep --out results/ [--n 5 10 15 20] [--N 5 10 15] [--seeds 100] [--ep-len 150]
"""

from __future__ import annotations

import argparse
import json
import os
import pickle
import threading
import time

import numpy as np

from . import tables
from .env import derive_env_seed, initial_platoon_state
from .models import Platoon
from .params import Params, Sim_n_task_2


# run_points runs several run_point calls at once on host threads; the reference-style setup code
# draws from numpy's global generator, so that part is serialised
_RNG_LOCK = threading.Lock()


def shard(points, n_seeds: int, rank: int, world: int):
    """Work of `rank`: for every (n, N) point a contiguous block of the seeds 0..n_seeds-1 (the
    first n_seeds % world ranks get one more).  Together the ranks cover every (n, N, seed)
    exactly once."""
    base, extra = divmod(n_seeds, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return [(n, N, list(range(lo, hi))) for n, N in points if hi > lo]


def run_point(n: int, N: int, seeds, ep_len: int = 150, device: int = 0, out_dir: str | None = None,
              velocity_estimator: str = "none", warm_incumbent: bool = True) -> dict:
    """Closed-loop episodes of the decentralised controller for `seeds` (one platoon each) at
    (n, N), all on the device.  Returns per-seed X (T+1, 2n), U (T, n), R (T,), violations (T,),
    node_counts (T,), and the step times; writes the reference's results files if out_dir."""
    import torch

    from .envdev import DeviceEnv
    from .solver import BatchSolver

    S, T = len(seeds), ep_len
    dev = torch.device("cuda", device)
    with _RNG_LOCK:  # Sim_n_task_2 and env.reset seed numpy's GLOBAL generator (params.py, env.py)
        sims = [Sim_n_task_2(n, seed=int(s), N=N) for s in seeds]
        x_init = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(-1).astype(np.float64)
                           for s in seeds])
    leader_x = sims[0].leader_trajectory.get_leader_trajectory()  # (2, ep_len + 50), seed-independent
    if T + N + 1 > leader_x.shape[1]:  # Sim_n_task_2 builds the trajectory for its own ep_len (150)
        raise ValueError(f"ep_len {T} with N = {N} needs {T + N + 1} leader samples; the Sim_n_task_2 "
                         f"trajectory holds {leader_x.shape[1]} (ep_len <= {leader_x.shape[1] - N - 1})")
    systems, masses = [], []
    for sim in sims:
        pl = Platoon(n, vehicle_type="pwa_gear", masses=sim.masses)
        vehicles = pl.get_vehicles()
        for i, d in enumerate(pl.get_vehicle_system_dicts(Params.ts)):
            systems.append(tables.system_from_dict(d, tables.gears_of(vehicles[i])))
        masses.append(sim.masses)
    solver = BatchSolver(tables.problem(N, sims[0].spacing_policy), systems, device=device)
    B = S * n
    solver.reserve(B)
    lx = torch.from_numpy(np.ascontiguousarray(leader_x)).to(dev)
    x = torch.from_numpy(x_init).to(dev)
    env = DeviceEnv(solver, torch.tensor(masses, dtype=torch.float64, device=dev))
    t_sys = torch.arange(B, dtype=torch.int32, device=dev)
    out = solver.alloc_outputs(B, dev)
    params = torch.empty((B, solver.params_stride), dtype=torch.float64, device=dev)
    roles = torch.empty(B, dtype=torch.int32, device=dev)
    X = torch.empty((T + 1, S, 2 * n), dtype=torch.float64, device=dev)
    U = torch.empty((T, S, n), dtype=torch.float64, device=dev)
    R = torch.empty((T, S), dtype=torch.float64, device=dev)
    V = torch.empty((T, S), dtype=torch.int32, device=dev)
    NODES = torch.empty((T, S), dtype=torch.int32, device=dev)
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    X[0] = x
    x_prev = x.clone()
    u = torch.empty((S, n), dtype=torch.float64, device=dev)
    u_prev = None
    # the previous step's sequences shifted by one step (last region repeated) as a second initial
    # incumbent of the next step's local searches (N > 8; pruning only, the answers do not change)
    hint = torch.full((B, N), -1, dtype=torch.int8, device=dev)
    if N > 8 and warm_incumbent:
        solver.set_region_hint(hint)
    step_s = np.zeros(T)
    for t in range(T):
        t0 = time.perf_counter()
        win = lx[:, t:t + N + 1].unsqueeze(0).expand(S, 2, N + 1).contiguous()
        solver.decent_params_device(x, win, x_prev=x_prev, estimator=velocity_estimator, params=params, roles=roles)
        solver.solve_device(t_sys, roles, params, out, retry_overflow=N > 8)
        u.copy_(out["u"][:, 0].view(S, n))
        hint[:, :-1] = out["region"][:, 1:]
        hint[:, -1] = out["region"][:, -1]
        bad.add_((out["status"] != 0).sum())
        NODES[t] = out["nodes"].view(S, n).max(dim=1).values
        x_prev.copy_(x)
        st = env.step(x, u, lx[:, t].unsqueeze(0).expand(S, 2).contiguous(), u_prev=u_prev)
        u_prev = u.clone()
        R[t] = st["cost"]
        V[t] = st["viol"]
        U[t] = u
        X[t + 1] = x
        torch.cuda.current_stream(dev).synchronize()  # this run's stream (run_points runs several at once)
        step_s[t] = time.perf_counter() - t0
    if int(bad.item()):
        raise RuntimeError(f"sweep point n={n} N={N}: {int(bad.item())} local MIQPs not optimal")
    h = lambda a: a.cpu().numpy()  # noqa: E731
    Xh, Uh, Rh, Vh, Nh = h(X), h(U), h(R), h(V), h(NODES)
    res = {"n": n, "N": N, "seeds": list(seeds), "step_s": step_s, "X": Xh, "U": Uh, "R": Rh, "viol": Vh,
           "nodes": Nh, "leader_x": leader_x}
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        # the batch's step time is every seed's solve time (the reference records the slowest
        # agent of a step, fleet_decent_mld.py:336-339; here all agents of all seeds share a launch)
        for k, (sim, s) in enumerate(zip(sims, seeds)):
            with open(os.path.join(out_dir, f"decent_vest_{velocity_estimator}_{sim.id}_seed_{s}.pkl"), "wb") as f:
                for obj in (Xh[:, k], Uh[:, k], Rh[:, k].reshape(T, 1, 1), step_s.reshape(T, 1),
                            Nh[:, k].reshape(T, 1).astype(float), Vh[:, k].astype(float), leader_x):
                    pickle.dump(obj, f)
    return res


def run_points(n: int, N: int, seeds, ep_len: int, device: int, out_dir, estimator: str, streams: int = 2):
    """run_point over `streams` blocks of the seeds at once, each block on its own host thread and
    HIP stream (the blocks are independent platoons; one block's kernels fill the GPU while the
    other's launches finish or synchronise).  Returns the per-block results and the wall time."""
    import torch

    seeds = list(seeds)
    K = max(1, min(streams, len(seeds)))
    blocks = [seeds[len(seeds) * j // K:len(seeds) * (j + 1) // K] for j in range(K)]
    res, errs = [None] * K, []

    def work(j):
        try:
            stream = torch.cuda.Stream(torch.device("cuda", device))
            with torch.cuda.stream(stream):
                res[j] = run_point(n, N, blocks[j], ep_len, device, out_dir, estimator)
        except BaseException as e:  # noqa: BLE001 -- re-raised on the caller's thread
            errs.append(e)

    t0 = time.perf_counter()
    if K == 1:
        res[0] = run_point(n, N, blocks[0], ep_len, device, out_dir, estimator)
    else:
        th = [threading.Thread(target=work, args=(j,)) for j in range(K)]
        for h in th:
            h.start()
        for h in th:
            h.join()
    if errs:
        raise errs[0]
    return res, time.perf_counter() - t0


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--n", type=int, nargs="+", default=[5, 10, 15, 20])
    ap.add_argument("--N", type=int, nargs="+", default=[5, 10, 15])
    ap.add_argument("--seeds", type=int, default=100)
    ap.add_argument("--ep-len", type=int, default=150)
    ap.add_argument("--out", default=None, help="directory of the results files (none: summary only)")
    ap.add_argument("--estimator", default="none", choices=["none", "two_point", "sat"])
    ap.add_argument("--streams", type=int, default=1,
                    help="seed blocks run concurrently per point (host threads / streams); measured 68 s vs 70 s "
                         "for the full grid, so 1 by default")
    args = ap.parse_args(argv)

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    points = [(n, N) for N in args.N for n in args.n]
    t0 = time.perf_counter()
    summary = []
    for n, N, seeds in shard(points, args.seeds, rank, world):
        rs, wall = run_points(n, N, seeds, args.ep_len, local, args.out, args.estimator, args.streams)
        R = np.concatenate([r["R"] for r in rs], axis=1)
        ep_s = wall if len(rs) > 1 else float(rs[0]["step_s"].sum())  # concurrent blocks: wall time incl. setup
        summary.append({"n": n, "N": N, "seeds": len(seeds), "episode_s": ep_s,
                        "platoon_steps_per_s": len(seeds) * args.ep_len / ep_s,
                        "mean_return": float(R.sum(axis=0).mean()),
                        "violation_steps": int(sum((r["viol"] > 0).sum() for r in rs)),
                        "max_nodes": int(max(r["nodes"].max() for r in rs))})
        print(json.dumps({"rank": rank, **summary[-1]}), flush=True)
    elapsed = time.perf_counter() - t0
    if dist:
        gathered = [None] * world
        dist.all_gather_object(gathered, {"rank": rank, "elapsed_s": elapsed, "points": summary})
        dist.destroy_process_group()
    else:
        gathered = [{"rank": rank, "elapsed_s": elapsed, "points": summary}]
    if rank == 0:
        total = sum(p["seeds"] for g in gathered for p in g["points"]) * args.ep_len
        print(json.dumps({"sweep": {"points": len(points), "seeds": args.seeds, "ep_len": args.ep_len, "ranks": world,
                                    "platoon_steps": total, "elapsed_s": max(g["elapsed_s"] for g in gathered),
                                    "platoon_steps_per_s": total / max(g["elapsed_s"] for g in gathered)}}),
              flush=True)


if __name__ == "__main__":
    main()
