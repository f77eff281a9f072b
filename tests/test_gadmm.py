"""Switching ADMM (fleet_g_admm.py, configs[3]).

CPU: the product's lane algorithm for the local QP (csrc/hvp_admm.h with the own-state ADMM
term, built for the host) against the oracle's full (x, u, s, copies)-space solve on traced
local problems (golden gadmm_local_N*.npz), including the region-edge multiplier bits the
switching rule reads; the oracle coordinator against its fixtures; the vehicle-sharding halo
exchange with gloo (world sizes 2 and 3).
GPU (marked): the same local problems through hvp_gadmm_solve (lane kernel at N = 5, 16-lane
group kernel at N = 10); the device coordinator (GAdmmEngine: rollout, ADMM rounds, switching,
warm-start selection) against the oracle coordinator over two time steps; the vehicle-sharded
engine (two shards in lockstep on one GPU) against the unsharded one.
"""

from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np
import pytest

import oracle as O
from golden_io import load
from instances import leader_window

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hybrid-vehicle-platoon_amd")


def _system():
    from hvp import tables
    from hvp.models import PwaGearVehicle

    veh = PwaGearVehicle(800)
    return tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))


def _check_local(fx, u, x, xf, xb, cost, status, edge):
    assert np.array_equal(status, fx["exp_status"])
    ok = fx["exp_status"] == 0
    ce = fx["exp_cost"][ok]
    assert np.all(np.abs(cost[ok] - ce) <= 1e-9 * np.maximum(1.0, np.abs(ce)))
    assert np.abs(u[ok] - fx["exp_u"][ok]).max() <= 1e-6
    assert np.abs(x[ok] - fx["exp_x"][ok]).max() <= 1e-6
    assert np.abs(xf[ok] - fx["exp_xf"][ok]).max() <= 1e-6
    assert np.abs(xb[ok] - fx["exp_xb"][ok]).max() <= 1e-9
    # the bits the switching rule reads: bit-exact
    assert np.array_equal(edge[ok].astype(np.int64), fx["exp_edge"][ok])
    assert (fx["exp_edge"][ok] != 0).mean() > 0.2  # the fixture exercises active region edges


@pytest.fixture(scope="module")
def hostref():
    from hvp import _abi

    subprocess.run(["make", "-s", "-C", PKG, "lib/libhvp_hostref.so"], check=True)
    return ctypes.CDLL(_abi.HOSTREF_PATH)


@pytest.mark.parametrize("N", [5, 10])
def test_gadmm_local_problem_host_build_matches_oracle(hostref, N):
    from hvp import _abi
    from hvp.gadmm import gadmm_problem

    fx = load(f"gadmm_local_N{N}.npz")
    prob = gadmm_problem(N, float(fx["rho"]))
    S = (_abi.HvpSystem * 1)(_system())
    B = len(fx["roles"])
    u, x, xf, xb = np.zeros((B, N)), np.zeros((B, 2, N + 1)), np.zeros((B, 2, N + 1)), np.zeros((B, 2, N + 1))
    cost, st, edge = np.zeros(B), np.zeros(B, np.int32), np.zeros(B, np.uint32)
    f = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    seq = np.ascontiguousarray(fx["seq"].astype(np.int8))
    rc = hostref.hvp_hostref_gadmm_solve(ctypes.byref(prob), S, B, f(np.zeros(B, np.int32)),
                                         f(np.ascontiguousarray(fx["roles"])), f(np.ascontiguousarray(fx["params"])),
                                         f(seq), f(u), f(x), f(xf), f(xb), f(cost), f(st), f(edge))
    assert rc == 0
    _check_local(fx, u, x, xf, xb, cost, st, edge)


def test_oracle_coordinator_is_deterministic_against_its_fixture():
    fx = load("gadmm_steps_n4_N5.npz")
    N, n = int(fx["N"]), int(fx["n"])
    co = O.GAdmmCoordinator([O.gear_pwa_system(800.0)] * n, O.Cfg(), N, admm_iters=int(fx["iters"]))
    co.set_leader_traj(leader_window(N, 0))
    u, c, runs = co.control(fx["states"][0])
    assert np.array_equal(u, fx["exp_u"][0]) and c == fx["exp_cost"][0]
    assert runs[0][2]["rounds"] == fx["exp_rounds"][0][0] and runs[0][2]["rounds"] > 1  # switching happened


def test_switching_rule_moves_across_the_active_edge():
    sysd = O.gear_pwa_system(800.0)
    co = O.GAdmmCoordinator([sysd], O.Cfg(), 4)
    lo, hi = O.region_bands(sysd)
    sig = np.array([2, 2, 2, 2])
    # step 1: upper edge of region 2 -> region 3; step 2: lower edge -> region 1; step 3 untouched
    out = co.switch(0, sig, (1 << (2 * 0 + 1)) | (1 << (2 * 1)))
    assert out.tolist() == [2, 3, 1, 2]
    assert hi[2] == lo[3] and lo[2] == hi[1]


def test_shard_range_partitions_the_chain():
    from hvp.gadmm import shard_range

    for n, w in ((20, 8), (10, 4), (7, 3), (4, 2)):
        blocks = [shard_range(n, r, w) for r in range(w)]
        assert blocks[0][0] == 0 and sum(m for _, m in blocks) == n
        assert all(blocks[r][0] + blocks[r][1] == blocks[r + 1][0] for r in range(w - 1))
        assert min(m for _, m in blocks) >= n // w


def _halo_worker(rank, world, port, P, n, N, q):
    import torch
    import torch.distributed as dist

    from hvp.gadmm import HaloExchange

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(5)
        full = [torch.randn((P * n, 2, N + 1), generator=g, dtype=torch.float64) for _ in range(3)]
        ex = HaloExchange(P, n, N, rank, world)
        mine = [torch.full_like(full[0], float("nan")) for _ in range(3)]
        own = (torch.arange(P)[:, None] * n + torch.arange(ex.lo, ex.hi)[None, :]).reshape(-1)
        for a, b in zip(mine, full):
            a[own] = b[own]
        ex(*mine)
        st = torch.full((P,), 1, dtype=torch.int32)
        st[rank % P] |= 2  # a failure on this rank
        st[(rank + 1) % P] |= 4
        ex.reduce_flags(st)
        cost = torch.full((P,), float(rank + 1), dtype=torch.float64)
        ex.reduce_cost(cost)
        # halo slots the consensus step of [lo, hi) reads
        need = {0: [ex.lo - 1, ex.hi], 1: [ex.hi, ex.hi + 1], 2: [ex.lo - 2, ex.lo - 1]}
        ok = True
        for k, vs in need.items():
            for v in vs:
                if 0 <= v < n:
                    idx = torch.arange(P) * n + v
                    ok &= bool(torch.equal(mine[k][idx], full[k][idx]))
        q.put((rank, ok, st.tolist(), cost.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 5), (3, 7)])
def test_halo_exchange_gloo(world, n):
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    P, N = 3, 4
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, P, n, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    for rank, ok, st, cost in res:
        assert ok, rank
        failed = {r % P for r in range(world)}
        changed = {(r + 1) % P for r in range(world)}
        for p in range(P):
            assert bool(st[p] & 2) == (p in failed) and bool(st[p] & 1) == (p not in failed)
            assert bool(st[p] & 4) == (p in changed)
        assert cost == [float(sum(range(1, world + 1)))] * P


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("N", [5, 10])
def test_gadmm_local_problem_on_gpu(gpu_available, N):
    import torch

    from hvp import _abi
    from hvp.gadmm import gadmm_problem
    from hvp.solver import BatchSolver

    fx = load(f"gadmm_local_N{N}.npz")
    B = len(fx["roles"])
    solver = BatchSolver(gadmm_problem(N, float(fx["rho"])), [_system()])
    dev = torch.device("cuda", 0)
    t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
    sysi, roles = t(np.zeros(B), torch.int32), t(fx["roles"], torch.int32)
    params, seq = t(fx["params"], torch.float64), t(fx["seq"], torch.int8)
    state = torch.ones(B, dtype=torch.int32, device=dev)
    u = torch.zeros((B, N), dtype=torch.float64, device=dev)
    x, xf, xb = (torch.zeros((B, 2, N + 1), dtype=torch.float64, device=dev) for _ in range(3))
    cost = torch.zeros(B, dtype=torch.float64, device=dev)
    st, edge = torch.zeros(B, dtype=torch.int32, device=dev), torch.zeros(B, dtype=torch.int32, device=dev)
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    # B independent "platoons" of one vehicle each
    rc = solver._lib.hvp_gadmm_solve(solver._h, B, 1, 0, 1, p(sysi), p(roles), p(params), p(seq), p(state), p(u),
                                     p(x), p(xf), p(xb), p(cost), p(st), p(edge), None,
                                     ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    _abi.check(rc, "hvp_gadmm_solve")
    torch.cuda.synchronize()
    h = lambda a: a.cpu().numpy()  # noqa: E731
    _check_local(fx, h(u), h(x), h(xf), h(xb), h(cost), h(st), h(edge).astype(np.uint32))


def _engine(fx, P, exchange=None):
    from hvp.gadmm import GAdmmEngine, gadmm_problem

    n, N = int(fx["n"]), int(fx["N"])
    return GAdmmEngine(gadmm_problem(N, float(fx["rho"])), [_system()] * n, n, P, admm_iters=int(fx["iters"]),
                       max_rounds=int(fx["max_rounds"]), exchange=exchange)


def _check_steps(fx, outs):
    n, N, steps = int(fx["n"]), int(fx["N"]), int(fx["steps"])
    for t, (out, runs) in enumerate(outs):
        rows = np.arange(t, len(fx["states"]), steps)  # fixture order: seed-major, then time step
        u = out["u"].cpu().numpy().reshape(-1, n, N)
        assert np.abs(u - fx["exp_u"][rows]).max() <= 1e-6, t
        c, ce = out["cost"].cpu().numpy(), fx["exp_cost"][rows]
        assert np.all(np.abs(c - ce) <= 1e-8 * np.abs(ce)), (t, c, ce)
        assert np.array_equal(out["warm_start"].cpu().numpy(), fx["exp_warm_start"][rows])
        for w, r in enumerate(runs):
            assert np.array_equal(r["platoon_rounds"].cpu().numpy(), fx["exp_rounds"][rows, w]), (t, w)
            seq = r["seq"].cpu().numpy().reshape(-1, n, N)
            assert np.array_equal(seq, fx["exp_seq"][rows, w]), (t, w)
            rc = r["cost"].cpu().numpy()
            assert np.all(np.abs(rc - fx["exp_run_cost"][rows, w]) <= 1e-8 * np.abs(fx["exp_run_cost"][rows, w]))


def _run_steps(fx, engines):
    """Both fixture time steps for all seeds at once (one platoon per seed) on the engine(s)
    (several = vehicle shards run in lockstep threads)."""
    n, N, steps = int(fx["n"]), int(fx["N"]), int(fx["steps"])
    outs = []
    for t in range(steps):
        rows = np.arange(t, len(fx["states"]), steps)
        res = [None] * len(engines)

        def go(k):
            e = engines[k]
            e.set_leader(leader_window(N, t))
            out = dict(e.control(fx["states"][rows]))
            res[k] = (out, out.pop("runs"))

        th = [threading.Thread(target=go, args=(k,)) for k in range(len(engines))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        outs.append(res)
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gadmm_steps_n4_N5.npz", "gadmm_steps_n3_N10.npz", "gadmm_steps_n20_N10.npz"])
def test_gadmm_engine_matches_oracle_coordinator(gpu_available, name):
    fx = load(name)
    P = len(fx["states"]) // int(fx["steps"])
    outs = _run_steps(fx, [_engine(fx, P)])
    _check_steps(fx, [o[0] for o in outs])


class LocalHalo:
    """Test double of hvp.gadmm.HaloExchange for shards that live in one process (threads on
    one GPU): same interface, the halo copied between the shards' arrays under a barrier."""

    def __init__(self, group: list, rank: int, lo: int, m: int, barrier: threading.Barrier) -> None:
        self.group, self.rank, self.lo, self.m, self.bar = group, rank, lo, m, barrier

    def __call__(self, x, xf, xb) -> None:
        import torch

        torch.cuda.synchronize()
        self.bar.wait()
        me = self.group[self.rank]
        for k, other in enumerate(self.group):
            if k == self.rank:
                continue
            P, n = other.P, other.n
            own = (np.arange(P)[:, None] * n + np.arange(other.lo, other.lo + other.m)[None, :]).reshape(-1)
            for a, b in ((me.x, other.x), (me.xf, other.xf), (me.xb, other.xb)):
                a[own] = b[own]
        torch.cuda.synchronize()
        self.bar.wait()

    def _combine(self, t, fn):
        import torch

        torch.cuda.synchronize()
        self.bar.wait()
        vals = [fn(e) for e in self.group]
        self.bar.wait()
        return vals

    def reduce_flags(self, state) -> None:
        from hvp import _abi

        vals = self._combine(state, lambda e: e.state.clone())
        f = (sum(((v & _abi.GADMM_FAILED) != 0).int() for v in vals) > 0).int()
        c = (sum(((v & _abi.GADMM_CHANGED) != 0).int() for v in vals) > 0).int()
        self.bar.wait()
        state |= f * _abi.GADMM_FAILED + c * _abi.GADMM_CHANGED
        state &= ~(f * _abi.GADMM_LIVE)

    def reduce_cost(self, cost) -> None:
        me = self.group[self.rank]
        me._partial = cost.clone()
        vals = self._combine(cost, lambda e: e._partial)
        cost.copy_(sum(vals))


@pytest.mark.gpu
@pytest.mark.parametrize("name,world", [("gadmm_steps_n4_N5.npz", 2), ("gadmm_steps_n20_N10.npz", 8)])
def test_gadmm_vehicle_sharded_engine_matches(gpu_available, name, world):
    """The vehicle-sharded engine (halo exchange per ADMM iteration) against the oracle
    coordinator: 2 shards at n = 4, and configs[3]'s layout -- n = 20 over 8 shards (blocks of
    2-3 vehicles) -- as lockstep threads on one GPU."""
    from hvp.gadmm import GAdmmEngine, gadmm_problem, shard_range

    fx = load(name)
    n, N = int(fx["n"]), int(fx["N"])
    P = len(fx["states"]) // int(fx["steps"])
    bar = threading.Barrier(world)
    group: list = []
    for r in range(world):
        lo, m = shard_range(n, r, world)
        group.append(GAdmmEngine(gadmm_problem(N, 0.5), [_system()] * n, n, P, admm_iters=int(fx["iters"]),
                                 max_rounds=int(fx["max_rounds"]), exchange=LocalHalo(group, r, lo, m, bar)))
    outs = _run_steps(fx, group)
    # the leader's shard reports the winner's u for its vehicles; stitch the shards' u together
    for t, res in enumerate(outs):
        u = np.concatenate([o[0]["u"].cpu().numpy().reshape(P, -1, N) for o in res], axis=1)
        rows = np.arange(t, len(fx["states"]), int(fx["steps"]))
        assert np.abs(u - fx["exp_u"][rows]).max() <= 1e-6
        for o in res:
            c = o[0]["cost"].cpu().numpy()
            assert np.all(np.abs(c - fx["exp_cost"][rows]) <= 1e-8 * np.abs(fx["exp_cost"][rows]))


@pytest.mark.gpu
def test_gadmm_warm_start_keeps_the_answers(gpu_available, monkeypatch):
    """Every local QP starts from the previous ADMM iteration's hinge states, active set and
    factors (hvp_coop.h warm_start); the cold start (HVP_GADMM_WARM=0) reaches the same optima:
    sequences, rounds and warm-start choices identical, controls to 1e-9, costs to 1e-10."""
    fx = load("gadmm_steps_n20_N10.npz")
    P = len(fx["states"]) // int(fx["steps"])
    warm = _run_steps(fx, [_engine(fx, P)])
    monkeypatch.setenv("HVP_GADMM_WARM", "0")
    cold = _run_steps(fx, [_engine(fx, P)])
    for ((wo, wr),), ((co, cr),) in zip(warm, cold):
        assert np.abs(wo["u"].cpu().numpy() - co["u"].cpu().numpy()).max() <= 1e-9
        wc, cc = wo["cost"].cpu().numpy(), co["cost"].cpu().numpy()
        assert np.all(np.abs(wc - cc) <= 1e-10 * np.abs(cc))
        assert np.array_equal(wo["warm_start"].cpu().numpy(), co["warm_start"].cpu().numpy())
        for a, b in zip(wr, cr):
            assert np.array_equal(a["seq"].cpu().numpy(), b["seq"].cpu().numpy())
            assert np.array_equal(a["platoon_rounds"].cpu().numpy(), b["platoon_rounds"].cpu().numpy())


def _gadmm_local_call(solver, N, sysi, roles, params, seq):
    """One hvp_gadmm_solve of B one-vehicle "platoons" on `solver`'s handle; host arrays out."""
    import torch

    from hvp import _abi

    dev = torch.device("cuda", 0)
    B = len(roles)
    t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)  # noqa: E731
    sysi, roles, params, seq = (t(sysi, torch.int32), t(roles, torch.int32), t(params, torch.float64),
                                t(seq, torch.int8))
    state = torch.ones(B, dtype=torch.int32, device=dev)
    u = torch.zeros((B, N), dtype=torch.float64, device=dev)
    x, xf, xb = (torch.zeros((B, 2, N + 1), dtype=torch.float64, device=dev) for _ in range(3))
    cost = torch.zeros(B, dtype=torch.float64, device=dev)
    st, edge = torch.zeros(B, dtype=torch.int32, device=dev), torch.zeros(B, dtype=torch.int32, device=dev)
    p = lambda a: ctypes.c_void_p(a.data_ptr())  # noqa: E731
    rc = solver._lib.hvp_gadmm_solve(solver._h, B, 1, 0, 1, p(sysi), p(roles), p(params), p(seq), p(state), p(u),
                                     p(x), p(xf), p(xb), p(cost), p(st), p(edge), None,
                                     ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    _abi.check(rc, "hvp_gadmm_solve")
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in dict(u=u, x=x, xf=xf, xb=xb, cost=cost, status=st, edge=edge).items()}


@pytest.mark.gpu
def test_gadmm_warm_records_never_start_another_qp(gpu_available):
    """a handle's warm-start records (hvp_coop.h WarmQp) are keyed by region code,
    hinge states AND (system index, role bits), so calling hvp_gadmm_solve again on the same
    handle with another batch -- rows permuted, systems swapped -- gives the answers of a fresh
    handle (cold start), never a solve from another QP's factors."""
    from hvp import tables
    from hvp.gadmm import gadmm_problem
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    N = 10
    fx = load(f"gadmm_local_N{N}.npz")
    B = len(fx["roles"])
    heavy = PwaGearVehicle(950)
    systems = [_system(), tables.system_from_dict(heavy.get_discrete_system(1), tables.gears_of(heavy))]
    prob = gadmm_problem(N, float(fx["rho"]))
    solver = BatchSolver(prob, systems)
    first = _gadmm_local_call(solver, N, np.zeros(B), fx["roles"], fx["params"], fx["seq"])
    _check_local(fx, first["u"], first["x"], first["xf"], first["xb"], first["cost"], first["status"],
                 first["edge"].astype(np.uint32))
    rng = np.random.default_rng(7)
    perm = rng.permutation(B)
    sys2 = (np.arange(B) % 2).astype(np.int32)
    args = (sys2, fx["roles"][perm], fx["params"][perm], fx["seq"][perm])
    again = _gadmm_local_call(solver, N, *args)
    fresh = _gadmm_local_call(BatchSolver(prob, systems), N, *args)
    assert np.array_equal(again["status"], fresh["status"])
    ok = fresh["status"] == 0
    # the heavy vehicle under the light one's traced sequences: some of those QPs are infeasible
    # (MI355X r04h: 87 % solved), the same ones for both handles
    assert ok.mean() > 0.5
    assert np.abs(again["u"][ok] - fresh["u"][ok]).max() <= 1e-9
    assert np.abs(again["x"][ok] - fresh["x"][ok]).max() <= 1e-7
    c, cf = again["cost"][ok], fresh["cost"][ok]
    assert np.all(np.abs(c - cf) <= 1e-10 * np.maximum(1.0, np.abs(cf)))
    assert np.array_equal(again["edge"][ok], fresh["edge"][ok])


@pytest.mark.gpu
@pytest.mark.parametrize("N", [5, 10])
def test_gadmm_local_problem_ipm_fallback(gpu_available, monkeypatch, N):
    """Switching-ADMM local QPs whose active-set solve fails go to k_gadmm_ipm (the interior point
    inside the hinge-state iteration, hvp_admm.h solve_admm_ipm) instead of failing their
    platoon.  Forced with HVP_LEAF_GI_CAP=2: the traced local problems still give the oracle's
    u, trajectories, copies, costs and the switching rule's edge bits (fleet_g_admm.py:162,195-205
    gets them from qpOASES)."""
    from hvp.gadmm import gadmm_problem
    from hvp.solver import BatchSolver

    monkeypatch.setenv("HVP_LEAF_GI_CAP", "2")
    fx = load(f"gadmm_local_N{N}.npz")
    B = len(fx["roles"])
    solver = BatchSolver(gadmm_problem(N, float(fx["rho"])), [_system()])
    r = _gadmm_local_call(solver, N, np.zeros(B), fx["roles"], fx["params"], fx["seq"])
    assert solver.stats().n_fallback > 0
    _check_local(fx, r["u"], r["x"], r["xf"], r["xb"], r["cost"], r["status"], r["edge"].astype(np.uint32))


@pytest.mark.gpu
def test_gadmm_engine_ipm_fallback(gpu_available, monkeypatch):
    """configs[3] at its own size (n = 20, N = 10, 100 ADMM iterations, 2 seeds x 2 steps) with the
    local QPs forced through the interior-point fallback (HVP_LEAF_GI_CAP=2: two active-set
    steps, then k_gadmm_ipm): the fallback polishes the interior point's active set into the
    exact optimum and multipliers (hvp_gi.h gi_polish), so no platoon fails and every warm start's
    sequences, rounds, costs and the winner's controls are the oracle coordinator's -- the same
    bar as the unforced engine (test_gadmm_engine_matches_oracle_coordinator).  Round 4's fallback
    (interior-point multipliers against kEdgeMultTol, hinge states classified at its approximate
    optimum) failed every platoon of this run on MI355X (r04i); the host replay of the same
    forcing, test_gadmm_forced_fallback_host_replay_matches_oracle, pins the algorithm on CPU."""
    monkeypatch.setenv("HVP_LEAF_GI_CAP", "2")
    fx = load("gadmm_steps_n20_N10.npz")
    P = len(fx["states"]) // int(fx["steps"])
    eng = _engine(fx, P)
    outs = _run_steps(fx, [eng])
    for out, runs in (o[0] for o in outs):
        for r in runs:
            assert not r["failed"].cpu().numpy().any()
    _check_steps(fx, [o[0] for o in outs])
    assert eng.solver.stats().n_fallback > 0


def test_gadmm_forced_fallback_host_replay_matches_oracle():
    """The oracle coordinator (oracle.py GAdmmCoordinator) on the product's local-QP algorithm
    built for the host with every local QP through the fallback as HVP_LEAF_GI_CAP=2 forces it on
    the device (two active-set steps, then hvp_admm.h solve_admm_ipm: interior point + active-set
    polish): configs[3]'s first two coordinator calls (34,000 local QPs, both warm starts at
    t = 1) give the fixture's controls, costs, sequences and rounds.  Without the polish, call 0
    failed a local QP and call 1 moved u by 0.19 (tests/gadmm_replay.py, mode 2)."""
    from gadmm_replay import replay

    subprocess.run(["make", "-s", "-C", PKG, "lib/libhvp_hostref.so"], check=True)
    assert replay(2, 2, verbose=False) == 0
