"""Regression test of the branch-and-bound workspace overflow path (the memory fault fixed in
705c8ac: overflowed reservations left uninitialised node slots that the next kernels swept).

A workspace far too small for the batch (hvp_reserve with a tiny capacity) must (1) report
HVP_OVERFLOW for the instances whose children do not fit -- never a truncated answer, never a
fault -- and (2) with ``retry_overflow`` re-solve exactly those instances alone, giving the same
regions, costs and controls as a solver with the default workspace, which the parity tests pin
against the oracle.  Covered at configs[1] (N = 5, lane kernels) and at N = 10 (16-lane groups).
"""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _solver(N):
    from hvp import tables
    from hvp.models import PwaGearVehicle
    from hvp.solver import BatchSolver

    veh = PwaGearVehicle(800)
    return BatchSolver(tables.problem(N), [tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh))])


@pytest.mark.parametrize("n,N,S,per", [(10, 5, 512, 2), (10, 10, 128, 3)])
def test_overflow_is_reported_and_retried(gpu_available, n, N, S, per):
    import torch

    import bench
    from hvp import _abi

    params, roles = bench.make_inputs(range(S), n, N)
    dev = torch.device("cuda", 0)
    tp, tr = torch.from_numpy(params).to(dev), torch.from_numpy(roles).to(dev)
    ts = torch.zeros(len(roles), dtype=torch.int32, device=dev)
    B = len(roles)

    ref = _solver(N).solve_device(ts, tr, tp, retry_overflow=True)
    torch.cuda.synchronize()
    assert (ref["status"] == _abi.OPTIMAL).all()

    tiny = _solver(N)
    tiny.reserve(B, per * B)  # `per` nodes per instance per level: the wide levels cannot fit
    raw = tiny.solve_device(ts, tr, tp)
    torch.cuda.synchronize()
    st = raw["status"].cpu().numpy()
    over = st == _abi.OVERFLOW
    assert over.any(), "the tiny workspace must overflow"
    # every other instance is complete and equal to the reference (an overflow never truncates
    # another instance's search)
    ok = ~over
    assert (st[ok] == _abi.OPTIMAL).all()
    assert torch.equal(raw["region"][torch.from_numpy(ok).to(dev)], ref["region"][torch.from_numpy(ok).to(dev)])

    out = tiny.solve_device(ts, tr, tp, retry_overflow=True)
    torch.cuda.synchronize()
    assert (out["status"] == _abi.OPTIMAL).all()
    assert torch.equal(out["region"], ref["region"])
    assert torch.equal(out["gear"], ref["gear"])
    rel = ((out["cost"] - ref["cost"]).abs() / ref["cost"].abs().clamp(min=1.0)).max().item()
    assert rel <= 1e-12
    assert (out["u"] - ref["u"]).abs().max().item() <= 1e-9
    assert torch.equal(out["nodes"], ref["nodes"])  # the re-solve explores the same tree


def test_overflow_host_path(gpu_available):
    """The host-array path (MpcMld.solve_mpc's batch form) retries overflowed instances too."""
    import bench
    from hvp import _abi

    n, N, S = 10, 5, 64
    params, roles = bench.make_inputs(range(S), n, N)
    B = len(roles)
    ref = _solver(N).solve(np.zeros(B, np.int32), roles, params)
    tiny = _solver(N)
    tiny.reserve(B, 2 * B)
    out = tiny.solve(np.zeros(B, np.int32), roles, params)
    assert (out.status == _abi.OPTIMAL).all()
    assert (out.region == ref.region).all()
    assert np.abs(out.cost - ref.cost).max() <= 1e-12 * np.abs(ref.cost).max()


@pytest.mark.parametrize("buckets", [2, 4])
def test_full_bucket_spills_into_free_segment(gpu_available, monkeypatch, buckets):
    """A level bucket that outgrows its segment (capacity / buckets) spills into another bucket's
    free segment (hvp_lane.h bnb_put_children) instead of reporting HVP_OVERFLOW.  At the smallest
    capacity at which ONE list per level fits (HVP_SPLIT_LEVELS=1, found by bisection), plus a few
    slots for the reservations that straddle a segment end, the bucketed lists fit too: children
    spill (n_spilled > 0), no instance overflows, and the answers and trees equal the default
    solve's (the bucket only orders the refill kernel's claims)."""
    import torch

    import bench
    from hvp import _abi

    n, N, S = 10, 5, 512
    params, roles = bench.make_inputs(range(S), n, N)
    dev = torch.device("cuda", 0)
    tp, tr = torch.from_numpy(params).to(dev), torch.from_numpy(roles).to(dev)
    ts = torch.zeros(len(roles), dtype=torch.int32, device=dev)
    B = len(roles)

    ref = _solver(N).solve_device(ts, tr, tp, retry_overflow=True)
    torch.cuda.synchronize()
    assert (ref["status"] == _abi.OPTIMAL).all()

    def solve(cap):  # a fresh handle per capacity (hvp_reserve only ever grows a workspace)
        s = _solver(N)
        s.reserve(B, cap)
        out = s.solve_device(ts, tr, tp)
        torch.cuda.synchronize()
        return out, s

    monkeypatch.setenv("HVP_SPLIT_LEVELS", "1")
    lo, hi = B, 16 * B
    assert not (solve(hi)[0]["status"] == _abi.OVERFLOW).any()
    while hi - lo > 64:
        mid = (lo + hi) // 2
        if (solve(mid)[0]["status"] == _abi.OVERFLOW).any():
            lo = mid
        else:
            hi = mid
    monkeypatch.setenv("HVP_SPLIT_LEVELS", str(buckets))
    cap = hi + 64 * buckets  # a straddling reservation leaves < 16 dead slots per bucket and attempt
    out, s = solve(cap)
    st = s.stats()
    assert st.n_spilled > 0, "the bucketed levels must have needed the spill at this capacity"
    assert (out["status"] == _abi.OPTIMAL).all()
    assert torch.equal(out["region"], ref["region"])
    assert torch.equal(out["gear"], ref["gear"])
    assert torch.equal(out["nodes"], ref["nodes"])
    assert (out["cost"] - ref["cost"]).abs().max().item() <= 1e-12 * ref["cost"].abs().max().item()
