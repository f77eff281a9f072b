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
