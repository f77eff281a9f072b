"""Device plant step: the batched counterpart of ``PlatoonEnv.step`` (env.py:126-212) for P
platoons, through ``hvp_env_step_batch`` (csrc/hvp_env.hip).  Together with the solvers it keeps
a closed loop (solve -> plant step -> solve) in HBM.  The stage-cost weights, spacing and d_safe
are the handle's controller constants (the env's Q_x, Q_u, Q_du and d_safe equal Params'
defaults, env.py:18-24)."""

from __future__ import annotations

import ctypes

from . import _abi


class DeviceEnv:
    def __init__(self, solver, masses, leader_index: int = 0, real_vehicle_as_reference: bool = False,
                 ts: float = 1.0) -> None:
        """solver: a BatchSolver / CentSolver (its handle's constants); masses (P, n) CUDA float64."""
        import torch

        if leader_index != 0 and real_vehicle_as_reference:
            raise NotImplementedError("Not implemented for real vehicle with leader not 0.")
        if not masses.is_cuda or masses.dtype != torch.float64 or masses.dim() != 2:
            raise ValueError("masses must be a (P, n) CUDA float64 tensor")
        self._solver = solver
        self.masses = masses.contiguous()
        self.P, self.n = int(masses.shape[0]), int(masses.shape[1])
        self.leader_index = leader_index
        self.rvar = bool(real_vehicle_as_reference)
        self.ts = float(ts)

    def step(self, x, u, leader_state, u_prev=None, gear=None, stream=None) -> dict:
        """x (P, 2n) float64 advanced in place; u (P, n); leader_state (P, 2); gear (P, n) int8 or
        None (the PWA-gear model's gear of each velocity).  Returns cost, viol, status (P,)."""
        import torch

        P, n = self.P, self.n
        for name, t, shape in (("x", x, (P, 2 * n)), ("u", u, (P, n)), ("leader_state", leader_state, (P, 2))):
            if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous() or tuple(t.shape) != shape:
                raise ValueError(f"{name} must be a contiguous CUDA float64 {shape} tensor")
        up = u if u_prev is None else u_prev
        dev = x.device
        out = {"cost": torch.empty(P, dtype=torch.float64, device=dev),
               "viol": torch.empty(P, dtype=torch.int32, device=dev),
               "status": torch.empty(P, dtype=torch.int32, device=dev)}
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        rc = self._solver._lib.hvp_env_step_batch(
            self._solver._h, P, n, ptr(self.masses), ptr(x), ptr(u), ptr(gear), ptr(up), ptr(leader_state),
            self.leader_index, 1 if self.rvar else 0, self.ts, ptr(out["cost"]), ptr(out["viol"]), ptr(out["status"]),
            ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_env_step_batch")
        return out
