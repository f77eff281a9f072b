#!/usr/bin/env python3
"""Throughput benchmark of the decentralised hybrid-MPC hot path on MI355X.

Metric (BASELINE.json): MPC timesteps/s for whole platoons, decentralised MLD, n = 10, N = 5
(configs[1]).  One *step* = one pass of the hot path over one batch: every vehicle of
``--platoons`` platoons (per GPU) solves its local MIQP (fleet_decent_mld.py:314-326) for one
platoon timestep.  ``value`` = platoon-timesteps solved by all ranks / wall time of the timed
region (max over ranks).  Inputs are synthetic random-init platoon states (env.py:70-116
distribution, seed s -> SeedSequence(s) derived env seed), constant-velocity neighbour
predictions and the constant-velocity leader window, resident in HBM before timing starts.

Multi-GPU: one process per GPU; every rank owns a disjoint range of seeds (weak scaling, no
collective in the data path -- the platoons are independent); the barrier / MAX-reduction only
brackets the timing.  Either an external launcher starts the ranks (torch.distributed.run sets
WORLD_SIZE / RANK / LOCAL_RANK), or ``--gpus N`` without WORLD_SIZE makes this process a launcher:
it starts N rank processes itself (never touching the GPU), prints rank 0's line and fails if any
rank fails.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "hybrid-vehicle-platoon_amd"))

HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector peak (spec)


def dense_qp_bytes(N: int) -> int:
    """bytes of one dense fixed-sequence QP, 8 (n_w^2 + m n_w + m + n_w)."""
    nw, m = 3 * N + 2, 14 * N + 4
    return 8 * (nw * nw + m * nw + m + nw)


def instance_io_bytes(N: int) -> int:
    """params in + u, x, cost out per local MIQP (+ N bytes of sigma)."""
    return 8 * (2 + 6 * (N + 1) + N + 2 * (N + 1) + 1) + N


def loaded_lib_sha() -> str:
    """SHA-256 of the libhvpsolve.so this process loads (HVP_LIB or the in-tree build)."""
    from hvp import _abi

    return _abi.lib_sha256()


def profiled(kernel: str, tag: str):
    """Per-launch PMC figures of `kernel` from the newest committed profiles/r*_<tag>_summary.json
    whose ``lib_sha256`` stamp is the library this process loads (profiles/run_profiles.sh runs
    this bench's workload `tag` under rocprofv3 and stamps the summary with the library's hash).
    A summary of another build is never used: (None, reason) instead."""
    import glob

    sha = loaded_lib_sha()
    stale = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{tag}_summary.json")), reverse=True):
        with open(path) as f:
            meta = json.load(f)
        d = meta["kernels"].get(kernel)
        if not d:
            continue
        if meta.get("lib_sha256") != sha:
            stale = stale or os.path.relpath(path, ROOT)
            continue
        return d, os.path.relpath(path, ROOT)
    why = (f"newest profile of this workload ({stale}) is of another build of libhvpsolve.so" if stale
           else f"no committed profile of workload {tag}")
    return None, why


def step_traffic(tag: str, per_solve: str = "k_bnb_finish") -> dict | None:
    """HBM bytes of EVERY product kernel of one solve: sum over the kernels of
    the hash-matched profile of hbm_bytes x launches, divided by the launches of `per_solve` (one per
    solve), with the per-kernel split.  None without a matching profile."""
    import glob

    sha = loaded_lib_sha()
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{tag}_summary.json")), reverse=True):
        with open(path) as f:
            meta = json.load(f)
        if meta.get("lib_sha256") != sha:
            continue
        ks = meta["kernels"]
        solves = (ks.get(per_solve) or {}).get("calls")
        if not solves:
            return None
        per = {k: d["hbm_bytes"] * d["calls"] / solves for k, d in ks.items()
               if k.startswith("k_") and "hbm_bytes" in d and d.get("calls")}
        return {"bytes_per_solve": sum(per.values()), "by_kernel": per, "solves_profiled": solves,
                "profile": os.path.relpath(path, ROOT)}
    return None


def qp_roofline(qp_step_ms: float, kernels: list, notional_bytes: float, tag: str) -> dict:
    """Roofline of the QP kernels of one step, from the live HIP-event time of their launches
    (qp_step_ms) and the per-launch PMC figures of profiles/ (the same bench workload):

      bound "fp64"   the kernels are FP64-VALU / latency bound (dense fixed-sequence QPs built
                     in registers): achieved = PMC FP64 FLOPs of the step's
                     QP launches, masked lanes removed (f64_flop_active = 64-lane FLOP count x
                     SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU)), / qp_step_ms; peak 78.6.
      traffic        PMC HBM bytes of the same launches (2 FETCH_SIZE + WRITE_SIZE) per step;
                     "hbm" reports traffic / qp_step_ms against 8 TB/s.
      survey_8d      SURVEY 8(d)'s notional dense-QP bytes (never moved by these kernels), as a
                     labelled side figure only.
    kernels: [(name, launches per step)]; tag: the profiled workload (profiles/r*_<tag>_summary.json)."""
    flop = flop_all = traffic = 0.0
    srcs, prof_ms, why = set(), {}, None
    for name, count in kernels:
        d, src = profiled(name, tag)
        if not d or "f64_flop_active" not in d or "hbm_bytes" not in d:
            why = src if not d else f"{src} lacks the PMC passes of {name}"
            flop = None
            break
        flop += d["f64_flop_active"] * count
        flop_all += d["f64_flop"] * count
        traffic += d["hbm_bytes"] * count
        srcs.add(src)
        prof_ms[name] = d.get("avg_ms")
    t = qp_step_ms * 1e-3
    out = {"bound": "fp64", "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "kernel": "+".join(k for k, _ in kernels),
           "launches_per_step": sum(c for _, c in kernels), "qp_ms_per_step": qp_step_ms,
           "kernel_avg_ms": qp_step_ms / max(1, sum(c for _, c in kernels)),
           "survey_8d": {"note": "notional dense-QP bytes of SURVEY 8(d), not moved by the kernels",
                         "bytes_per_step": notional_bytes, "GB_per_s": notional_bytes / t / 1e9}}
    if flop is None:
        out.update({"achieved": None, "frac": None, "traffic": None, "lib_sha256": loaded_lib_sha(),
                    "note": f"{why}: roofline not reported (profiles/run_profiles.sh profiles this build)"})
        return out
    achieved = flop / t / 1e12
    out.update({"achieved": achieved, "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                "flop_per_step": flop, "flop_per_step_all_lanes": flop_all,
                "frac_all_lanes": flop_all / t / 1e12 / FP64_PEAK_TFLOPS,
                "hbm": {"achieved": traffic / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": traffic / t / 1e9 / HBM_PEAK_GBS},
                "profile": sorted(srcs), "profile_avg_ms": prof_ms, "lib_sha256": loaded_lib_sha()})
    return out


def timed_roofline(kernels: list, K: int, qp_ms_handles: list, ms_per_step: float, tag: str) -> dict:
    """Roofline of the configuration the headline times: K handles on K streams.  The PMC figures
    come from the profile of the same command (workload `tag`, profile_streams = K); per step the
    K handles run K x (launches per handle) launches.
      frac_step     PMC FP64 FLOPs of one step's QP launches (masked lanes removed) / ms_per_step, the
                    driver-visible time of the whole step (overlap and every other kernel included)
      frac_kernel   FLOPs per launch / the average launch duration measured live in the timed region
                    (each handle's HIP events around its launches in the last timed step; the K
                    streams' launches overlap, so a launch takes longer than alone)"""
    launches = sum(c for _, c in kernels)
    out = {"profile_streams": K, "launches_per_step": K * launches, "ms_per_step": ms_per_step,
           "qp_ms_per_handle": qp_ms_handles,
           "kernel_avg_ms": sum(qp_ms_handles) / max(1, K * launches)}
    flop = traffic = 0.0
    srcs = set()
    for name, count in kernels:
        d, src = profiled(name, tag)
        if not d or "f64_flop_active" not in d or "hbm_bytes" not in d:
            out.update({"frac_step": None, "frac_kernel": None,
                        "note": (src if not d else f"{src} lacks the PMC passes of {name}") +
                                f": profiles/profile_all.sh OUT {tag} profiles this build"})
            return out
        flop += d["f64_flop_active"] * count * K
        traffic += d["hbm_bytes"] * count * K
        srcs.add(src)
        out.setdefault("profile_avg_ms", {})[name] = d.get("avg_ms")
    out.update({"flop_per_step": flop, "traffic": traffic, "profile": sorted(srcs),
                "achieved_step": flop / (ms_per_step * 1e-3) / 1e12,
                "frac_step": flop / (ms_per_step * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                "achieved_kernel": flop / (K * launches) / (out["kernel_avg_ms"] * 1e-3) / 1e12,
                "hbm_step": {"achieved": traffic / (ms_per_step * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": traffic / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS}})
    out["frac_kernel"] = out["achieved_kernel"] / FP64_PEAK_TFLOPS
    return out


def seed_range(rank: int, S: int) -> range:
    """The platoon seeds of one rank: a contiguous block of S, disjoint across ranks."""
    return range(rank * S, (rank + 1) * S)


def free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(argv: list, world: int) -> int:
    """``--gpus N`` without an external launcher: start N rank processes of this script (RANK =
    LOCAL_RANK = r, WORLD_SIZE = N, rendezvous on 127.0.0.1), forward rank 0's output, and return
    the first non-zero exit code.  This process never initialises the GPU (no exec either: the
    ranks are children).  A rank that fails ends the others, which would otherwise wait in a
    collective for it."""
    import subprocess
    import tempfile

    port = free_port()
    procs, outs = [], []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out = tempfile.TemporaryFile(mode="w+") if r == 0 else None
        outs.append(out)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env, stdout=out))
    rc = 0
    live = set(range(world))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c
                print(f"bench.py: rank {r} exited with {c}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    outs[0].seek(0)
    sys.stdout.write(outs[0].read())
    sys.stdout.flush()
    return rc


def bench_dry_run(args, world: int, rank: int, dist) -> None:
    """--dry-run: the multi-rank protocol without a GPU (gloo): seed shards, barrier + timed region
    around an empty step, MAX over ranks, rank 0's line with every rank's seed range."""
    import torch

    S = args.platoons
    seeds = seed_range(rank, S)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ranges = [[seeds.start, seeds.stop]]
    if dist:
        tt = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        allr = [None] * world
        dist.all_gather_object(allr, [seeds.start, seeds.stop])
        ranges = allr
    if rank == 0:
        print(json.dumps({"metric": "dry run (no GPU work)", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": dt / max(args.steps, 1) * 1e3,
                          "seed_ranges": ranges, "backend": dist.get_backend() if dist else None}), flush=True)


def make_inputs(seeds, n: int, N: int):
    """(params, roles, sys) for n-vehicle platoons at t = 0 (vectorised over seeds)."""
    from hvp.batched import decent_params_from_states
    from hvp.env import derive_env_seed, initial_platoon_state

    states = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(-1).astype(np.float64)
                       for s in seeds])
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    params, roles = decent_params_from_states(states, N, lead)
    return params, roles


def cpu_baseline(n: int, N: int, budget_s: float, threads: int, quadratic: bool = True):
    """The CPU oracle (oracle/hvp_oracle.c, OpenMP over instances) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    sysd = O.gear_pwa_system(800.0)
    O.set_method(O.METHOD_BNB if N > 8 else O.METHOD_ENUMERATE)  # exhaustive past N = 8 is ~1e4+ QPs/vehicle
    done = 0
    t0 = time.perf_counter()
    chunk = max(threads, 1) * 2
    seed = 10_000_000
    # min_1_norm past N = 8: one oracle MILP takes seconds, so the sample is vehicles (one per core per
    # round), scaled by 1 / n per platoon step
    per_vehicle = not quadratic and N > 8
    if per_vehicle:
        chunk = max(threads, 1)
    while done == 0 or time.perf_counter() - t0 < budget_s:
        params, roles = make_inputs(range(seed, seed + chunk), n, N)
        if per_vehicle:  # one vehicle of each platoon, its position rotating with the seed
            pick = np.arange(chunk) * n + (seed + np.arange(chunk)) % n
            params, roles = params[pick], roles[pick]
        seed += chunk
        O.solve_batch([sysd], O.Cfg(), N, np.zeros(len(roles), np.int32), roles, params, quadratic=quadratic,
                      nthreads=threads)
        done += chunk
    dt = time.perf_counter() - t0
    if per_vehicle:
        return {"value": done / n / dt, "unit": "platoon-timesteps/s", "cores": threads, "kind": "port",
                "sample": f"{done} local MILPs (min_1_norm, N={N}) of platoons' vehicles by oracle/hvp_oracle.c, "
                          f"{dt:.1f} s; rate / {n} vehicles per platoon step"}
    return {"value": done / dt, "unit": "platoon-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{done} platoons x {n} local {'MIQPs' if quadratic else 'MILPs (min_1_norm)'} (N={N}) by "
                      f"oracle/hvp_oracle.c, {dt:.1f} s"}


def hostref_baseline(n: int, N: int, budget_s: float, threads: int, method: int = 0, quadratic: bool = True):
    """The product's lane algorithm compiled for the host cores (extra, fairer CPU number)."""
    import ctypes

    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle

    if not os.path.exists(_abi.HOSTREF_PATH):
        return None
    L = ctypes.CDLL(_abi.HOSTREF_PATH)
    veh = PwaGearVehicle(800)
    S = (_abi.HvpSystem * 1)(tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh)))
    prob = tables.problem(N, quadratic_cost=quadratic, method=method)
    done, seed = 0, 20_000_000
    chunk = max(threads, 1) * 16
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        params, roles = make_inputs(range(seed, seed + chunk), n, N)
        seed += chunk
        B = len(roles)
        bufs = [np.zeros((B, N)), np.zeros((B, 2, N + 1)), np.zeros((B, N), np.int8), np.zeros(B),
                np.zeros(B, np.int32), np.zeros(B, np.int32), np.zeros(B, np.int32)]
        f = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        L.hvp_hostref_solve_batch(ctypes.byref(prob), S, B, f(np.zeros(B, np.int32)), f(roles),
                                  f(np.ascontiguousarray(params)), *[f(b) for b in bufs], threads)
        done += chunk
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "platoon-timesteps/s", "cores": threads,
            "sample": f"{done} platoons, same lane algorithm built with g++ -O2 -fopenmp"}


def leader_windows(T: int, N: int, S: int, dev):
    """Constant-velocity leader (p = 3000 + 20 t, v = 20): per step t its window (S, 2, N+1)
    and state (S, 2), resident on the device."""
    import torch

    lx = np.stack([3000.0 + 20.0 * np.arange(T + N + 1), np.full(T + N + 1, 20.0)])
    wins = torch.from_numpy(np.ascontiguousarray(np.stack([np.broadcast_to(lx[:, t:t + N + 1], (S, 2, N + 1))
                                                           for t in range(T)]))).to(dev)
    lead = torch.from_numpy(np.ascontiguousarray(np.stack([np.broadcast_to(lx[:, t], (S, 2)) for t in range(T)]))).to(dev)
    return wins, lead


def bench_admm(args, world: int, rank: int, local: int, dist) -> None:
    """configs[2]: fleet_naive_admm in closed loop on the device.  One step = one platoon
    timestep of ADMMCoordinator.get_control (fleet_naive_admm.py:379-477: warm start from the
    shifted previous solutions, y carried across steps as the reference never resets it
    (:357-359), admm_iters x (n local MIQPs per platoon + the z/y update)) followed by
    PlatoonEnv.step on the device (hvp_env_step_batch); the next step starts from the new states
    and the moved leader window."""
    import torch

    from hvp import tables
    from hvp.admm import AdmmEngine, admm_problem
    from hvp.env import derive_env_seed, initial_platoon_state
    from hvp.envdev import DeviceEnv
    from hvp.models import PwaGearVehicle

    n, N, S, iters = args.n, args.N, args.platoons, args.admm_iters
    # --cost l1: LocalMpcADMM(quadratic_cost=False) (fleet_naive_admm.py:74-77), the node QPs by the
    # wave interior point with the copies as variables
    quadratic = args.cost == "quadratic"
    veh = PwaGearVehicle(800)
    system = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    seeds = seed_range(rank, S)
    states = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(-1).astype(np.float64)
                       for s in seeds])
    T = args.warmup + args.steps + 1
    dev = torch.device("cuda", local)
    wins, lead = leader_windows(T, N, S, dev)
    notopt = torch.zeros((), dtype=torch.int64, device=dev)
    bad = torch.zeros((), dtype=torch.int64, device=dev)
    # --streams K: the platoons split over K engines, each stepped by its own host thread on its
    # own HIP stream (platoons are independent; one engine's level tails are filled by the other)
    K = max(1, args.streams)
    groups = []
    for j in range(K):
        a, b = S * j // K, S * (j + 1) // K
        P = b - a
        roles = [tables.role_bits(i == 0, i == n - 1, i == 0) for i in range(n)] * P
        eng = AdmmEngine(admm_problem(N, 0.5, quadratic_cost=quadratic), [system], np.zeros(n * P, np.int32), roles,
                         n, P, device=local,
                         warm_incumbent=False if args.no_warm_incumbent else None)
        groups.append({"eng": eng, "P": P, "env": DeviceEnv(eng.solver, torch.full((P, n), 800.0, dtype=torch.float64,
                                                                                  device=dev)),
                       "x": torch.from_numpy(states[a:b]).to(dev), "u": torch.empty((P, n), dtype=torch.float64,
                                                                                      device=dev),
                       "u_prev": None, "wins": [w[a:b].contiguous() for w in wins],
                       "lead": [ld[a:b].contiguous() for ld in lead],
                       "notopt": torch.zeros((), dtype=torch.int64, device=dev),
                       "bad": torch.zeros((), dtype=torch.int64, device=dev),
                       "stream": torch.cuda.current_stream(dev) if K == 1 else torch.cuda.Stream(dev)})

    def group_step(g, t, on_solve=None):
        with torch.cuda.stream(g["stream"]):
            g["eng"].set_leader_device(g["wins"][t])
            o = g["eng"].step(g["x"], iters, stream=g["stream"], on_solve=on_solve)
            g["u"].copy_(o["u"][:, 0].view(g["P"], n))
            g["notopt"].add_((o["status"] != 0).sum())
            r = g["env"].step(g["x"], g["u"], g["lead"][t], u_prev=g["u_prev"])
            g["bad"].add_(r["status"].sum())
            g["u_prev"] = g["u"].clone()

    def step(t, on_solve=None):
        if K == 1 or on_solve is not None:
            for g in groups:
                group_step(g, t, on_solve)
            return
        import threading

        errs = []

        def run(g):
            try:
                group_step(g, t)
            except BaseException as e:  # noqa: BLE001 -- re-raised on the main thread
                errs.append(e)

        th = [threading.Thread(target=run, args=(g,)) for g in groups]
        for h in th:
            h.start()
        for h in th:
            h.join()
        if errs:
            raise errs[0]

    for t in range(args.warmup):
        step(t)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + args.steps):
        step(t)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    for g in groups:
        notopt.add_(g["notopt"])
        bad.add_(g["bad"])
    # QP-launch timing and work counters of one more step (stats synchronise per iteration)
    acc = {"qp_ms": 0.0, "qps": 0, "it": 0}

    def on_solve(solver):
        st = solver.stats()
        acc["qp_ms"] += st.qp_ms
        acc["qps"] += st.n_candidates
        acc["it"] += st.qp_iterations

    step(args.warmup + args.steps, on_solve=on_solve)
    value = S * world * args.steps / dt
    notional = acc["qps"] * dense_qp_bytes(N) + iters * n * S * instance_io_bytes(N)
    # per-launch PMC figures of one engine's launches (profile: --streams 1 --platoons S/K); the
    # event pass above ran the K engines one after the other, so acc["qp_ms"] is their summed time
    qk = ([("k_l1_root", iters * K), ("k_l1_bound", iters * N * K)] if not quadratic
          else [("k_bnb_root_coop", iters * K), ("k_bnb_bound_coop", iters * N * K)] if N > 8
          else [("k_bnb_root", iters * K), ("k_bnb_bound", iters * N * K)])
    result = {
        "metric": f"MPC timesteps/sec (whole platoon) at n={n} N={N} naive_admm ({iters} ADMM iterations)"
                  + ("" if quadratic else " min_1_norm"),
        "value": value, "unit": "platoon-timesteps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: env.reset random-init platoon states (seeded), constant-velocity leader; closed loop "
                "on the device (ADMM control + plant step), y and the warm starts carried across steps",
        "config": {"workload": f"fleet_naive_admm n={n} N={N} pwa_gear closed loop (configs[2])", "n_vehicles": n,
                   "horizon": N, "admm_iters": iters, "rho": 0.5, "platoons_per_gpu": S,
                   "cost": "min_2_norm" if quadratic else "min_1_norm",
                   "local_miqps_per_step": iters * n * S * world, "warm_incumbent": N > 8 and not args.no_warm_incumbent,
                   "streams_per_gpu": K, "parallelism": f"seeds-sharded x{world}"},
        "roofline": qp_roofline(acc["qp_ms"], qk, notional, f"admm_n{n}_N{N}" + ("" if quadratic else "_l1")
                                + f"_P{S // K}"),
        "qps_per_step": acc["qps"], "qp_iters_per_qp": acc["it"] / max(acc["qps"], 1),
        "not_optimal_total": int(notopt.item()), "plant_failures_total": int(bad.item()),
    }
    if rank == 0 and not args.no_cpu and args.cpu_budget > 0 and world == 1 and quadratic:
        result["cpu_baseline"] = cpu_baseline_admm(n, N, iters, min(args.cpu_budget, 20.0), cpu_threads())
        result["cpu_baseline_1core"] = cpu_baseline_admm(n, N, iters, min(args.cpu_budget, 20.0) * 0.5, 1)
    elif rank == 0 and not args.no_cpu and args.cpu_budget > 0 and world == 1:
        result["cpu_baseline"] = cpu_baseline_admm_l1(n, N, iters, min(args.cpu_budget, 20.0), cpu_threads())
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def cpu_threads() -> int:
    """Host cores a CPU baseline may use: the pool gives each GPU a 16-core share (OMP_NUM_THREADS=16
    on the box; nproc shows the whole machine)."""
    return min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")), 16)


def run_cpu_workers(worker, args: tuple, threads: int, budget_s: float, seed0: int) -> list:
    """`threads` copies of a one-core baseline worker on disjoint seed ranges, as separate processes
    (spawn: fresh interpreters that never touch the GPU; the coordinators are Python loops around
    oracle calls, so threads would serialise on the GIL).  Each returns its own (done, seconds, ...)."""
    if threads <= 1:
        return [worker(*args, budget_s, seed0)]
    import concurrent.futures as cf
    import multiprocessing as mp

    with cf.ProcessPoolExecutor(threads, mp_context=mp.get_context("spawn")) as ex:
        futs = [ex.submit(worker, *args, budget_s, seed0 + 1_000_000 * k) for k in range(threads)]
        return [f.result() for f in futs]


def _admm_worker(n: int, N: int, iters: int, budget_s: float, seed0: int):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    sysd = O.gear_pwa_system(800.0)
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    done, seed, t0 = 0, seed0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        c = O.AdmmCoordinator(sysd, O.Cfg(), N, n)
        c.set_leader_x(lead)
        c.step(O.env_initial_state(n, seed).astype(float), iters)
        seed += 1
        done += 1
    return done, time.perf_counter() - t0


def cpu_baseline_admm(n: int, N: int, iters: int, budget_s: float, threads: int = 1):
    """The oracle coordinator (oracle.AdmmCoordinator: restated fleet_naive_admm get_control on
    oracle local MIQPs), one platoon step at a time per core, on `threads` cores."""
    res = run_cpu_workers(_admm_worker, (n, N, iters), threads, budget_s, 30_000_000)
    done = sum(r[0] for r in res)
    return {"value": sum(r[0] / r[1] for r in res), "unit": "platoon-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{done} platoon steps x {iters} ADMM iterations x {n} local MIQPs (N={N}), oracle, "
                      f"{max(r[1] for r in res):.1f} s on {threads} core(s)"}


def _admm_l1_worker(n: int, N: int, budget_s: float, seed0: int):
    """Local min_1_norm MILPs of the first ADMM iteration (the oracle coordinator's own parameter rows:
    warm-start blocks of a fresh coordinator, vehicles in order, platoon after platoon), one at a time
    until the budget is spent (at least one)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    sysd = O.gear_pwa_system(800.0)
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    done, seed, t0 = 0, seed0, time.perf_counter()
    while done == 0 or time.perf_counter() - t0 < budget_s:
        c = O.AdmmCoordinator(sysd, O.Cfg(), N, n, quadratic=False)
        c.set_leader_x(lead)
        x = O.env_initial_state(n, seed).astype(float).reshape(n, 2)
        for i in range(n):
            b = c.blocks[i]
            p = O.admm_params(x[i], b["yf"], b["zf"], b["yb"], b["zb"], b["xl"])
            O.solve_admm_miqp(sysd, O.Cfg(), N, c.roles[i], c.rho, p, 200, False)
            done += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        seed += 1
    return done, time.perf_counter() - t0


def cpu_baseline_admm_l1(n: int, N: int, iters: int, budget_s: float, threads: int = 1):
    """naive-ADMM min_1_norm on the oracle: a platoon step is iters x n local MILPs (~20 s each at
    N = 10 on one core, so a whole step is far beyond a bounded sample); the sample times first-iteration
    local MILPs and scales their rate by 1 / (iters n)."""
    res = run_cpu_workers(_admm_l1_worker, (n, N), threads, budget_s, 40_000_000)
    done = sum(r[0] for r in res)
    rate = sum(r[0] / r[1] for r in res)
    return {"value": rate / (iters * n), "unit": "platoon-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{done} local min_1_norm MILPs (N={N}) of the first ADMM iteration, oracle, "
                      f"{max(r[1] for r in res):.1f} s on {threads} core(s); rate / ({iters} iterations x {n} "
                      f"vehicles) per platoon step"}


def gadmm_qp_bytes(N: int) -> int:
    """SURVEY 8(d) dense-QP bytes of one switching-ADMM local QP (fleet_g_admm.LocalMpc with x
    condensed): n_w = u (N) + slack (N+1) + two neighbour copies 2 (N+1) each, m = 14 N + 4."""
    nw, m = 6 * N + 5, 14 * N + 4
    return 8 * (nw * nw + m * nw + m + nw)


def bench_gadmm(args, world: int, rank: int, local: int, dist) -> None:
    """configs[3]: fleet_g_admm, one step = TrackingGAdmmCoordinator.g_admm_control (both warm
    starts: constant velocity + shifted previous solution; each a rollout and rounds of
    admm_iters x (local QPs + consensus) + switching) for every platoon on the device.
    --gadmm-layout replicas: every rank owns whole platoons (seed-sharded, no collective);
    vehicles: every rank owns a block of vehicles of all platoons, RCCL halo send/recv of the
    boundary vehicles after every local-QP launch."""
    import torch

    from hvp import tables
    from hvp.env import derive_env_seed, initial_platoon_state
    from hvp.gadmm import GAdmmEngine, HaloExchange, gadmm_problem
    from hvp.models import PwaGearVehicle

    n, N, S, iters = args.n, args.N, args.platoons, args.admm_iters
    sharded = args.gadmm_layout == "vehicles" and world > 1
    veh = PwaGearVehicle(800)
    system = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    seed0 = 0 if sharded else rank * S
    states = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(-1).astype(np.float64)
                       for s in range(seed0, seed0 + S)])
    ex = HaloExchange(S, n, N, rank, world) if sharded else None
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    # --streams K (replicas): the platoons split over K engines, each driven by its own host thread
    # on its own HIP stream (the engine synchronises once per switching round; the other engine's
    # launches fill the GPU meanwhile)
    K = 1 if sharded else max(1, args.streams)
    dev = torch.device("cuda", local)
    groups = []
    for j in range(K):
        a, b = S * j // K, S * (j + 1) // K
        eng = GAdmmEngine(gadmm_problem(N, 0.5), [system] * n, n, b - a, device=local, admm_iters=iters,
                          max_rounds=args.max_rounds, exchange=ex)
        eng.set_leader(lead)
        groups.append({"eng": eng, "x": torch.from_numpy(states[a:b]).to(dev),
                       "stream": torch.cuda.current_stream(dev) if K == 1 else torch.cuda.Stream(dev), "out": None})

    def control(g):
        with torch.cuda.stream(g["stream"]):
            g["out"] = g["eng"].control(g["x"])

    def step():
        if K == 1:
            control(groups[0])
            return
        import threading

        errs = []

        def run(g):
            try:
                control(g)
            except BaseException as e:  # noqa: BLE001 -- re-raised on the main thread
                errs.append(e)

        th = [threading.Thread(target=run, args=(g,)) for g in groups]
        for h in th:
            h.start()
        for h in th:
            h.join()
        if errs:
            raise errs[0]

    step()  # t = 0 (one warm start): establishes the previous solution
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rounds = launches = 0
    for _ in range(args.steps):
        step()
        for g in groups:
            rounds += sum(r["rounds"] for r in g["out"]["runs"])
            launches += sum(r["launches"] for r in g["out"]["runs"])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ok = all(bool(torch.isfinite(g["out"]["cost"]).all().item()) for g in groups)
    if dist:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # per-launch time of the local-QP kernel: HIP events on the launch stream over one more step
    # (the groups one after the other)
    qp_ev = []
    for g in groups:
        eng = g["eng"]
        solve = eng.solve

        def timed_solve(stream=None, solve=solve):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            solve(stream)
            b.record()
            qp_ev.append((a, b))

        eng.solve = timed_solve
        control(g)
        torch.cuda.synchronize()
        eng.solve = solve
    qp_ms = [a.elapsed_time(b) for a, b in qp_ev]
    n_qp_launch = len(qp_ms)
    qp_avg = float(np.mean(qp_ms))
    live_qps = sum(g["eng"].P * g["eng"].m for g in groups) / K  # upper bound: platoons that stopped switching skip their lanes
    notional = live_qps * n_qp_launch * (gadmm_qp_bytes(N) + 8 * (2 + 14 * (N + 1)))
    platoons_total = S * (1 if sharded else world)
    value = platoons_total * args.steps / dt
    result = {
        "metric": f"MPC timesteps/sec (whole platoon) at n={n} N={N} g_admm ({iters} ADMM iterations)",
        "value": value, "unit": "platoon-timesteps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if sharded else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic: env.reset random-init platoon states (seeded), constant-velocity leader; every timed "
                "step is a g_admm_control with both warm starts (previous solution from the preceding call)",
        "config": {"workload": f"fleet_g_admm n={n} N={N} pwa_gear (configs[3])", "n_vehicles": n, "horizon": N,
                   "admm_iters": iters, "max_rounds": args.max_rounds, "rho": 0.5, "platoons_per_gpu": S,
                   "streams_per_gpu": K,
                   "parallelism": (f"vehicles-sharded x{world} (RCCL halo send/recv per ADMM iteration)" if sharded
                                   else f"seeds-sharded x{world} (replicas, no collective)")},
        # the engines' QP launches timed one engine after the other (HIP events on the launch
        # stream); per-launch PMC figures of one engine (profile: --streams 1 --platoons S/K)
        "roofline": qp_roofline(qp_avg * n_qp_launch, [("k_gadmm_qp_coop" if N > 8 else "k_gadmm_qp", n_qp_launch)],
                                notional, f"gadmm_n{n}_N{N}_P{S // K}"),
        "admm_rounds_per_step": rounds / args.steps, "qp_launches_per_step": launches / args.steps,
        "all_feasible": ok,
    }
    if ex is not None:
        result["halo_bytes_per_exchange"] = ex.bytes_per_call
    if rank == 0 and not args.no_cpu and args.cpu_budget > 0 and world == 1:
        result["cpu_baseline"] = cpu_baseline_gadmm(n, N, iters, args.max_rounds, min(args.cpu_budget, 30.0),
                                                    cpu_threads())
        result["cpu_baseline_1core"] = cpu_baseline_gadmm(n, N, iters, args.max_rounds,
                                                          min(args.cpu_budget, 30.0) * 0.5, 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def _gadmm_worker(n: int, N: int, iters: int, max_rounds: int, budget_s: float, seed0: int):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    systems = [O.gear_pwa_system(800.0)] * n
    done, qps, seed, t_run = 0, 0, seed0, 0.0
    while t_run < budget_s:
        co = O.GAdmmCoordinator(systems, O.Cfg(), N, admm_iters=iters, max_rounds=max_rounds)
        co.set_leader_traj(lead)
        st = O.env_initial_state(n, seed).astype(float)
        co.control(st)
        co.trace = []
        t0 = time.perf_counter()
        co.control(st)
        t_run += time.perf_counter() - t0
        qps += len(co.trace)
        seed += 1
        done += 1
    return done, t_run, qps


def cpu_baseline_gadmm(n: int, N: int, iters: int, max_rounds: int, budget_s: float, threads: int = 1):
    """The oracle coordinator (oracle.GAdmmCoordinator, full-space local QPs), one platoon's
    g_admm_control at a time per core (both warm starts: a preceding untimed call), `threads` cores."""
    res = run_cpu_workers(_gadmm_worker, (n, N, iters, max_rounds), threads, budget_s, 40_000_000)
    done, qps = sum(r[0] for r in res), sum(r[2] for r in res)
    return {"value": sum(r[0] / r[1] for r in res), "unit": "platoon-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{done} g_admm_control calls (n={n}, N={N}, {iters} ADMM iterations, {qps} local QPs), "
                      f"oracle, {max(r[1] for r in res):.1f} s on {threads} core(s)"}


def bench_closed_loop(args, world: int, rank: int, local: int, dist) -> None:
    """fleet_decent_mld closed loop on the device: one step = observe_states (neighbour
    predictions, hvp_decent_params_batch) + the n local MIQPs of every platoon (hvp_solve_batch)
    + PlatoonEnv.step (hvp_env_step_batch: 10 Euler sub-steps of the nonlinear plant, stage cost,
    violations).  The platoons move: step t uses the states produced by step t - 1."""
    import torch

    from hvp import tables
    from hvp.env import derive_env_seed, initial_platoon_state
    from hvp.envdev import DeviceEnv
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    n, N, S = args.n, args.N, args.platoons
    veh = PwaGearVehicle(800)
    system = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    solver = BatchSolver(tables.problem(N), [system], device=local)
    dev = torch.device("cuda", local)
    x0 = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(-1).astype(np.float64)
                   for s in seed_range(rank, S)])
    T = args.warmup + args.steps + N + 2
    lx = np.stack([3000.0 + 20.0 * np.arange(T), np.full(T, 20.0)])
    wins = torch.from_numpy(np.ascontiguousarray(np.stack([np.broadcast_to(lx[:, t:t + N + 1], (S, 2, N + 1))
                                                           for t in range(args.warmup + args.steps)]))).to(dev)
    lead = torch.from_numpy(np.ascontiguousarray(np.stack([np.broadcast_to(lx[:, t], (S, 2))
                                                           for t in range(args.warmup + args.steps)]))).to(dev)
    B = S * n
    solver.reserve(B)
    env = DeviceEnv(solver, torch.full((S, n), 800.0, dtype=torch.float64, device=dev))
    x = torch.from_numpy(x0).to(dev)
    t_sys = torch.zeros(B, dtype=torch.int32, device=dev)
    out = solver.alloc_outputs(B, dev)
    params = torch.empty((B, solver.params_stride), dtype=torch.float64, device=dev)
    roles = torch.empty(B, dtype=torch.int32, device=dev)
    u = torch.empty((S, n), dtype=torch.float64, device=dev)
    u_prev = [None]
    viol = torch.zeros(S, dtype=torch.int64, device=dev)
    bad = torch.zeros(S, dtype=torch.int64, device=dev)
    notopt = torch.zeros((), dtype=torch.int64, device=dev)

    def step(t):
        solver.decent_params_device(x, wins[t], params=params, roles=roles)
        solver.solve_device(t_sys, roles, params, out)
        u.copy_(out["u"][:, 0].view(S, n))
        st = env.step(x, u, lead[t], u_prev=u_prev[0])
        u_prev[0] = u.clone()
        viol.add_(st["viol"])
        bad.add_(st["status"])
        notopt.add_((out["status"] != 0).sum())

    for t in range(args.warmup):
        step(t)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for t in range(args.warmup, args.warmup + args.steps):
        step(t)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    s = solver.stats()
    value = S * world * args.steps / dt
    result = {
        "metric": f"MPC timesteps/sec (whole platoon) at n={n} N={N} decent_mld closed loop",
        "value": value, "unit": "platoon-timesteps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: env.reset random-init platoon states (seeded), constant-velocity leader; the platoons "
                "move under the nonlinear plant, every step from the previous step's states",
        "config": {"workload": f"fleet_decent_mld n={n} N={N} pwa_gear closed loop (observe_states + local MIQPs + "
                               "PlatoonEnv.step on the device)", "n_vehicles": n, "horizon": N,
                   "platoons_per_gpu": S, "parallelism": f"seeds-sharded x{world}"},
        "qp_kernel_ms_last_step": s.qp_ms, "solve_ms_last_step": s.last_ms,
        "not_optimal_total": int(notopt.item()), "plant_failures_total": int(bad.sum().item()),
        "violation_steps_total": int((viol // 100).sum().item()),
    }
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def cent_qp_bytes(n: int, N: int) -> int:
    """SURVEY.md 8(d) dense bytes of one centralised fixed-sequence QP (condensed like the local
    QP: u (nN) and slacks (n(N+1)) free, m = 13N + 3 rows per vehicle), 8 (n_w^2 + m n_w + m + n_w)."""
    nw, m = n * (2 * N + 1), n * (13 * N + 3)
    return 8 * (nw * nw + m * nw + m + nw)


def bench_cent(args, world: int, rank: int, local: int, dist) -> None:
    """fleet_cent_mld.py (mpcs/cent_mld.py MpcMldCent): one step = the centralised MIQP of every
    platoon of the rank's seed range (MldAgent.get_control -> solve_mpc), one wavefront per
    platoon running the whole branch and bound (csrc/hvp_cent_bnb.h); platoons are independent
    (seed-sharded, no collective)."""
    import torch

    from hvp import tables
    from hvp.cent import CentSolver, cent_problem
    from hvp.env import derive_env_seed, initial_platoon_state
    from hvp.models import PwaGearVehicle

    n, N, S = args.n, args.N, args.platoons
    veh = PwaGearVehicle(800)
    system = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    dev = torch.device("cuda", local)
    seeds = seed_range(rank, S)
    x0 = np.stack([initial_platoon_state(n, derive_env_seed(int(s))).reshape(n, 2).astype(np.float64) for s in seeds])
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    # --streams K: the platoons over K handles, each solved by its own host thread on its own HIP
    # stream (a solve synchronises once per round of subtree tasks; the other fills the GPU)
    K = max(1, args.streams)
    groups = []
    for j in range(K):
        a, b = S * j // K, S * (j + 1) // K
        sv = CentSolver(cent_problem(N), [system], device=local)
        groups.append((sv, torch.zeros((b - a, n), dtype=torch.int32, device=dev), torch.from_numpy(x0[a:b]).to(dev),
                       torch.from_numpy(np.ascontiguousarray(np.broadcast_to(lead, (b - a, 2, N + 1)))).to(dev),
                       sv.alloc_outputs(b - a, n, dev),
                       torch.cuda.current_stream(dev) if K == 1 else torch.cuda.Stream(dev)))
    solver = groups[0][0]

    def solve_group(g):
        sv, ts, tx, tl, o, stm = g
        with torch.cuda.stream(stm):
            sv.solve_device(ts, tx, tl, max_nodes=args.max_nodes, out=o, stream=stm)

    def run():
        if K == 1:
            solve_group(groups[0])
            return
        import threading

        errs = []

        def work(g):
            try:
                solve_group(g)
            except BaseException as e:  # noqa: BLE001 -- re-raised on the main thread
                errs.append(e)

        th = [threading.Thread(target=work, args=(g,)) for g in groups]
        for h in th:
            h.start()
        for h in th:
            h.join()
        if errs:
            raise errs[0]

    for _ in range(args.warmup):
        run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    status = np.concatenate([g[4]["status"].cpu().numpy() for g in groups])
    nodes = np.concatenate([g[4]["nodes"].cpu().numpy() for g in groups])
    iters = np.concatenate([g[4]["iters"].cpu().numpy() for g in groups])
    if dist:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    # kernel time: HIP events the library records around the search kernels on the solve stream
    # (K streams: their searches overlap, so the step's wall time)
    # kernel time of the roofline: one more step as ONE handle over all S platoons (the launch size
    # of the committed profile, run_profiles.sh ... --streams 1), HIP events around its kernels
    if K == 1:
        run()
        kernel_ms = solver.stats().last_ms
    else:
        sv1 = CentSolver(cent_problem(N), [system], device=local)
        sv1.solve_device(torch.zeros((S, n), dtype=torch.int32, device=dev), torch.from_numpy(x0).to(dev),
                         torch.from_numpy(np.ascontiguousarray(np.broadcast_to(lead, (S, 2, N + 1)))).to(dev),
                         max_nodes=args.max_nodes, out=sv1.alloc_outputs(S, n, dev))
        torch.cuda.synchronize()
        kernel_ms = sv1.stats().last_ms
        del sv1
    qps = int(nodes.sum())
    notional = qps * cent_qp_bytes(n, N) + S * 8 * (2 * n + 2 * (N + 1) + n * (3 * N + 2) + 1)
    n_opt = int((status == 0).sum())
    value = S * world * args.steps / dt
    q = np.percentile(nodes, [50, 90, 99, 100])
    result = {
        "metric": f"MPC timesteps/sec (whole platoon) at n={n} N={N} cent_mld (QP cap {args.max_nodes} per platoon)",
        "value": value, "unit": "platoon-timesteps/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: env.reset random-init platoon states (seeded), constant-velocity leader",
        "config": {"workload": f"fleet_cent_mld n={n} N={N} pwa_gear (MpcMldCent)", "n_vehicles": n, "horizon": N,
                   "platoons_per_gpu": S, "max_nodes": args.max_nodes, "streams_per_gpu": K,
                   "parallelism": f"seeds-sharded x{world}"},
        "value_optimal_only": n_opt * world * args.steps / dt,
        "roofline": qp_roofline(kernel_ms, cent_kernels(f"cent_n{n}_N{N}_P{S}"), notional, f"cent_n{n}_N{N}_P{S}"),
        "qps_per_step": qps, "qp_iters_per_qp": float(iters.sum()) / max(qps, 1),
        "nodes_per_platoon": {"p50": float(q[0]), "p90": float(q[1]), "p99": float(q[2]), "max": float(q[3])},
        # the heaviest searches of the rank (seed, QPs, status): where the step's time goes
        "heaviest": [[int(seeds[j]), int(nodes[j]), int(status[j])] for j in np.argsort(-nodes, kind="stable")[:8]],
        "status_counts": {"optimal": int((status == 0).sum()), "infeasible": int((status == 1).sum()),
                          "node_limit": int((status == 2).sum()), "overflow": int((status == 3).sum())},
    }
    if rank == 0 and not args.no_cpu and args.cpu_budget > 0 and world == 1:
        result["cpu_baseline"] = cpu_baseline_cent(n, N, min(args.cpu_budget, 30.0), qps / S, cpu_threads())
        result["cpu_baseline_1core"] = cpu_baseline_cent(n, N, min(args.cpu_budget, 30.0) * 0.5, qps / S, 1)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


def cent_kernels(tag: str) -> list:
    """The search kernels of one centralised solve: k_cent_bnb once, then (split search, heavy
    platoons) the rounds of k_cent_tasks and k_cent_final.  The number of task rounds per solve
    is read from the same profile (launches of k_cent_tasks per launch of k_cent_bnb; every solve
    of the profiled run has the same inputs, so the same rounds)."""
    out = [("k_cent_bnb", 1)]
    d_bnb, _ = profiled("k_cent_bnb", tag)
    d_t, _ = profiled("k_cent_tasks", tag)
    if d_bnb and d_t and d_bnb.get("calls"):
        out += [("k_cent_tasks", d_t["calls"] / d_bnb["calls"]), ("k_cent_final", 1)]
    return out


def _cent_worker(n: int, N: int, budget_s: float, seed0: int):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    systems = [O.gear_pwa_system(800.0)] * n
    lead = np.stack([3000.0 + 20.0 * np.arange(N + 1), np.full(N + 1, 20.0)])
    O.set_cent_cap(2000)
    done, qps, seed = 0, 0, seed0
    t0 = time.perf_counter()
    try:
        while time.perf_counter() - t0 < budget_s:
            r = O.solve_cent(systems, O.Cfg(), N, O.env_initial_state(n, seed).astype(float), lead)
            qps += r.n_qps
            done += 1
            seed += 1
    finally:
        O.set_cent_cap(0)
    return done, time.perf_counter() - t0, qps


def cpu_baseline_cent(n: int, N: int, budget_s: float, qps_per_platoon: float, threads: int = 1):
    """The oracle's centralised MIQP (oracle_solve_cent: full-space dense IPM per QP, the same
    joint branch and bound, so the same QPs per platoon), one platoon at a time per core on
    `threads` cores.  Bounded sample: platoons from seed 10^7 up, each search capped at 2000 QPs,
    until the budget is spent; the measured QP rate is scaled to platoon-timesteps/s by the GPU
    run's mean QPs per platoon (same seeds' distribution, same search order)."""
    res = run_cpu_workers(_cent_worker, (n, N), threads, budget_s, 10_000_000)
    done, qps = sum(r[0] for r in res), sum(r[2] for r in res)
    rate = sum(r[2] / r[1] for r in res)
    return {"value": rate / max(qps_per_platoon, 1.0), "unit": "platoon-timesteps/s", "cores": threads, "kind": "port",
            "sample": f"{qps} QPs of oracle_solve_cent in {max(r[1] for r in res):.1f} s on {threads} core(s) "
                      f"({done} platoons, search capped at 2000 QPs each) = {rate:.1f} QPs/s, / {qps_per_platoon:.0f} "
                      f"QPs per platoon (GPU run mean)"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--platoons", type=int, default=16384, help="platoons per GPU per step")
    ap.add_argument("--n", type=int, default=10)
    ap.add_argument("--N", type=int, default=5)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU-oracle baseline (0 = skip)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--method", choices=["auto", "enum", "bnb"], default="auto",
                    help="region-sequence search (include/hvp.h HVP_METHOD_*)")
    ap.add_argument("--controller", choices=["decent", "admm", "gadmm", "cent"], default="decent",
                    help="decent: fleet_decent_mld (configs[1]); admm: fleet_naive_admm (configs[2]); "
                         "gadmm: fleet_g_admm (configs[3]); cent: fleet_cent_mld (MpcMldCent)")
    ap.add_argument("--max-nodes", type=int, default=2000000, help="cent: QPs per platoon cap")
    ap.add_argument("--closed-loop", action="store_true",
                    help="decent: every step = neighbour predictions + local MIQPs + plant step, all on the device")
    ap.add_argument("--admm-iters", type=int, default=None, help="default 20 (admm) / 100 (gadmm)")
    ap.add_argument("--max-rounds", type=int, default=10, help="gadmm: switching rounds cap")
    ap.add_argument("--streams", type=int, default=None,
                    help="platoons split over this many handles / HIP streams (decent: one host thread; admm, "
                         "gadmm replicas, cent: one host thread each); default: 3 for decent min_2_norm "
                         "(profiles/r04m_bench_*), 1 for the min_1_norm simplex path, whose LP kernels fill the "
                         "chip alone (231k vs 207k platoon-steps/s, profiles/r04i_bench_l1_*), 2 otherwise "
                         "(DESIGN.md section 4)")
    ap.add_argument("--no-warm-incumbent", action="store_true",
                    help="admm: do not try the previous iteration's sequences as incumbents (A/B)")
    ap.add_argument("--gadmm-layout", choices=["replicas", "vehicles"], default="replicas")
    ap.add_argument("--cost", choices=["quadratic", "l1"], default="quadratic",
                    help="decent: min_2_norm (default) or min_1_norm (the MILP variant; --method auto = branch and "
                         "bound, enum = exhaustive enumeration up to N = 8)")
    ap.add_argument("--no-roofline-pass", action="store_true",
                    help="decent: skip the untimed one-handle pass that times the QP launches for the roofline "
                         "(profile runs of the multi-stream configuration, so the trace holds its launches only)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU work: start the ranks (gloo), shard the seeds, run the timing protocol around an "
                         "empty step and print the line (tests the --gpus N launcher on a CPU)")
    args = ap.parse_args()
    if args.streams is None:
        simplex_l1 = (args.controller == "decent" and args.cost == "l1" and args.N <= 8
                      and os.environ.get("HVP_L1_SIMPLEX", "1") != "0")
        # decent min_2_norm: 3 (the root level and the dive leaves occupy a quarter of the CUs for
        # ~0.6 ms per solve; a third stream's levels fill the rest: 7.09-7.14M vs 6.74-6.98M on the
        # same box, profiles/r04m_bench_*); min_1_norm simplex: 1; the ADMM forms, cent: 2
        args.streams = 1 if simplex_l1 else (3 if args.controller == "decent" else 2)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.platoons < 1 or args.steps < 1 or args.warmup < 0:
        sys.exit("bench.py: --platoons and --steps must be >= 1, --warmup >= 0")

    import torch

    dist = None
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist

            dist.init_process_group("gloo")
        bench_dry_run(args, world, rank, dist)
        if dist:
            dist.destroy_process_group()
        return
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from hvp import tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    if args.admm_iters is None:
        args.admm_iters = 100 if args.controller == "gadmm" else 20
    if args.controller == "admm":
        return bench_admm(args, world, rank, local, dist)
    if args.controller == "gadmm":
        return bench_gadmm(args, world, rank, local, dist)
    if args.controller == "cent":
        return bench_cent(args, world, rank, local, dist)
    if args.closed_loop:
        return bench_closed_loop(args, world, rank, local, dist)
    n, N, S = args.n, args.N, args.platoons
    veh = PwaGearVehicle(800)
    system = tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))
    method = {"auto": 0, "enum": 1, "bnb": 2}[args.method]
    quadratic = args.cost == "quadratic"
    if not quadratic and method == 0:
        method = 2  # min_1_norm AUTO: branch and bound at every horizon (hvp_lane.h kAutoEnumMaxNL1)
    # each rank owns a disjoint seed range: platoons are independent (weak scaling)
    params, roles = make_inputs(seed_range(rank, S), n, N)
    B = len(roles)
    dev = torch.device("cuda", local)
    t_params_all = torch.from_numpy(params).to(dev)
    t_roles_all = torch.from_numpy(roles).to(dev)
    # --streams K: the platoons split into K handles on K HIP streams (the levels of one handle's
    # search are serial; K independent searches let one fill the CUs another's level tail leaves)
    K = max(1, args.streams)
    cuts = [(S * j // K) * n for j in range(K + 1)]
    chunks = []
    for j in range(K):
        a, b = cuts[j], cuts[j + 1]
        sv = BatchSolver(tables.problem(N, quadratic_cost=quadratic, method=method), [system], device=local)
        sv.reserve(b - a)
        chunks.append((sv, torch.zeros(b - a, dtype=torch.int32, device=dev), t_roles_all[a:b].contiguous(),
                       t_params_all[a:b].contiguous(), sv.alloc_outputs(b - a, dev),
                       torch.cuda.current_stream(dev) if K == 1 else torch.cuda.Stream(dev)))
    solver = chunks[0][0]

    # long horizons: a heavy-tailed search can outgrow an instance's workspace share; those
    # instances are re-solved inside the step (one synchronisation), so every step is complete
    retry = N > 8 or not quadratic

    def step():
        for sv, ts, tr, tp, o, stm in chunks:
            with torch.cuda.stream(stm):
                sv.solve_device(ts, tr, tp, o, stream=stm, retry_overflow=retry)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    ok = all(bool((c[4]["status"] == 0).all().item()) for c in chunks)  # the timed steps' own results
    # the QP launches of the LAST timed step as they ran in the timed configuration (K handles on K
    # streams, overlapping): each handle's HIP events around its launches (read after the region)
    timed_qp_ms = [float(c[0].stats().qp_ms) for c in chunks]
    if dist:
        tt = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    # per-launch kernel time (HIP events recorded by the library on the solve stream around the
    # QP launches) and work counters: a second pass of the same steps, outside the timed region
    # (reading them synchronises the stream after every step), as ONE handle over the whole batch
    # -- the launch size of the committed profile (run_profiles.sh ... --streams 1)
    if args.no_roofline_pass:
        # (profiling runs of the K-stream configuration: only its own launches in the trace; the work
        # counters of the last timed step stand for every step)
        ev = None
    elif K == 1:
        ev = chunks[0]
    else:
        sv1 = BatchSolver(tables.problem(N, quadratic_cost=quadratic, method=method), [system], device=local)
        sv1.reserve(B)
        ev = (sv1, torch.zeros(B, dtype=torch.int32, device=dev), t_roles_all, t_params_all,
              sv1.alloc_outputs(B, dev), torch.cuda.current_stream(dev))
    qp_ms, cand, iters, fallback = [], 0, 0, 0
    if ev is None:
        sts = [c[0].stats() for c in chunks]
        qp_ms = [sum(float(x.qp_ms) for x in sts)]
        cand = args.steps * sum(x.n_candidates for x in sts)
        iters = args.steps * sum(x.qp_iterations for x in sts)
        fallback = args.steps * sum(x.n_fallback for x in sts)
    for _ in range(args.steps if ev is not None else 0):
        sv, ts, tr, tp, o, stm = ev
        sv.solve_device(ts, tr, tp, o, stream=stm)
        s = sv.stats()
        qp_ms.append(s.qp_ms)
        cand += s.n_candidates
        iters += s.qp_iterations
        fallback += s.n_fallback
    del ev

    steps_total = S * world * args.steps
    value = steps_total / dt
    bnb = method != 1
    # QP time per step: the root kernel + the N bound launches (B&B) or K_qp_gi (enumeration),
    # each bracketed by HIP events the library records on the solve stream
    qp_step_ms = float(np.mean(qp_ms))
    cand_per_step = cand / args.steps
    notional = cand_per_step * dense_qp_bytes(N) + B * instance_io_bytes(N)
    simplex = N <= 8 and os.environ.get("HVP_L1_SIMPLEX", "1") != "0"  # min_1_norm LPs: per-lane simplex
    env = os.environ.get
    if bnb and not quadratic:
        if not simplex:
            qk = [("k_l1_root", 1), ("k_l1_bound", N)]
        elif env("HVP_LP_REFILL", "32") == "0":
            qk = [("k_lp_root", 1), ("k_lp_bound", N)]
        elif env("HVP_LP_ROOT_REFILL", "1") == "0":
            qk = [("k_lp_root", 1), ("k_lp_bound_refill", N)]
        else:  # the root level, the dive leaves and the N levels through the refill kernel
            qk = [("k_lp_bound_refill", N + 2)]
    elif bnb:
        if N > 8:
            qk = [("k_bnb_root_coop", 1), ("k_bnb_bound_coop", N)]
        elif env("HVP_ROOT_REFILL", "1") == "0":
            qk = [("k_bnb_root", 1), ("k_bnb_bound_refill", N)]
        else:  # root level + dive leaves + N levels, all through the refill kernel
            qk = [("k_bnb_bound_refill", N + 2)]
    else:
        qk = [("k_qp_gi", 1)] if quadratic else [("k_qp_lp" if simplex else "k_qp_l1", 1)]
    # the PMC figures are per launch over the WHOLE batch (the profile runs this workload with
    # --streams 1); qp_step_ms is the HIP-event time of those launches in the one-handle pass
    prof_tag = f"decent_n{n}_N{N}" + ("" if bnb else "_enum") + ("" if quadratic else "_l1") + f"_P{S}"
    roofline = qp_roofline(qp_step_ms, qk, notional, prof_tag)
    # every launch of the step (instance prep, levels, tie rule, outputs): bytes per solve of the
    # whole batch against the instance I/O (SURVEY 8(d)'s per-instance bytes x B)
    st = step_traffic(prof_tag) if bnb else None
    if st:
        st["instance_io_bytes"] = B * instance_io_bytes(N)
        st["x_instance_io"] = st["bytes_per_solve"] / st["instance_io_bytes"]
    roofline["traffic_step"] = st
    roofline["time_basis"] = (f"HIP events around the QP launches of one handle over all {S} platoons (the timed "
                              f"region splits them over {K} streams, whose launches overlap)")
    roofline["profile_streams"] = 1
    if K > 1:
        # the timed configuration itself: PMC figures of the same bench command with --streams K
        # (workload tag ..._s<K>, per launch of one handle over S/K platoons) against (a) the
        # driver-visible ms_per_step and (b) the live per-launch HIP-event time of the timed region
        roofline["timed"] = timed_roofline(qk, K, timed_qp_ms, dt / args.steps * 1e3,
                                           f"decent_n{n}_N{N}" + ("" if bnb else "_enum") + ("" if quadratic else "_l1")
                                           + f"_P{S}_s{K}")

    result = {
        "metric": f"MPC timesteps/sec (whole platoon) at n={n} N={N} decent_mld" + ("" if quadratic else " min_1_norm"),
        "value": value,
        "unit": "platoon-timesteps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic: env.reset random-init platoon states (seeded), constant-velocity neighbour "
                "predictions, constant-velocity leader",
        "config": {"workload": (f"fleet_decent_mld n={n} N={N} pwa_gear"
                                + (" (configs[1])" if (n, N) == (10, 5) else " (configs[4] sweep point)")),
                   "n_vehicles": n, "horizon": N, "search": "branch-and-bound" if bnb else "enumeration",
                   "cost": "min_2_norm (MIQP)" if quadratic else "min_1_norm (MILP)",
                   "platoons_per_gpu": S, "local_miqps_per_step": B * world, "streams_per_gpu": K,
                   "parallelism": f"seeds-sharded x{world}"},
        "roofline": roofline,
        "qps_per_step": cand_per_step,
        "qp_iters_per_candidate": iters / max(cand, 1),
        "ipm_fallbacks_per_step": fallback / args.steps,
        "all_optimal": ok,
    }
    if rank == 0 and not args.no_cpu and args.cpu_budget > 0 and world == 1:
        # every core this job may use: the pool gives each GPU a 16-core share (OMP_NUM_THREADS=16
        # on the box; nproc shows the whole machine), plus a 1-core run
        threads = cpu_threads()
        result["cpu_baseline"] = cpu_baseline(n, N, args.cpu_budget, threads, quadratic)
        result["cpu_baseline_1core"] = cpu_baseline(n, N, args.cpu_budget * 0.5, 1, quadratic)
        hr = hostref_baseline(n, N, min(args.cpu_budget, 10.0), threads, method, quadratic)
        if hr:
            result["cpu_same_algorithm"] = hr
            result["cpu_same_algorithm_1core"] = hostref_baseline(n, N, min(args.cpu_budget, 10.0) * 0.5, 1, method,
                                                                  quadratic)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
