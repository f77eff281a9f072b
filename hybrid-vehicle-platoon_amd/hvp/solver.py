"""Batched local-MIQP solver: the Python face of libhvpsolve.so (include/hvp.h).

:class:`BatchSolver` owns one ``hvp_handle`` (the compiled problem: horizon, weights, the
vehicles' PWA tables) and solves any number of instances per call:

* ``solve_device(...)`` takes torch tensors already on the GPU (zero-copy device pointers, the
  throughput path: bench.py, batched coordinators), asynchronous on the current torch stream;
* ``solve(...)`` takes numpy arrays (host pointers; one synchronous call, PCIe included) -- the
  path behind the per-agent ``solve_mpc`` drop-in.

There is no CPU fallback: constructing a solver without the HIP library raises.
"""

from __future__ import annotations

import contextlib
import ctypes
from dataclasses import dataclass

import numpy as np

from . import _abi


@dataclass
class BatchResult:
    u: np.ndarray        # (B, N)     control sequence
    x: np.ndarray        # (B, 2, N+1) predicted state trajectory
    region: np.ndarray   # (B, N)     PWA region (= MLD delta) per step, -1 if no solution
    gear: np.ndarray     # (B, N)     gear label implied by the region
    cost: np.ndarray     # (B,)       optimal objective (Gurobi ObjVal equivalent)
    status: np.ndarray   # (B,)       HVP_* status
    nodes: np.ndarray    # (B,)       region sequences solved (Gurobi NodeCount analogue)
    iters: np.ndarray    # (B,)       IPM iterations summed over the sequences


class BatchSolver:
    def __init__(self, problem: _abi.HvpProblem, systems: list[_abi.HvpSystem], device: int = 0,
                 max_batch: int = 0, candidate_capacity: int = 0) -> None:
        self._lib = _abi.load()
        self.N = int(problem.N)
        self.problem = problem
        self.n_systems = len(systems)
        arr = (_abi.HvpSystem * len(systems))(*systems)
        h = ctypes.c_void_p()
        _abi.check(self._lib.hvp_create(ctypes.byref(h), ctypes.byref(problem), arr, len(systems), device), "hvp_create")
        self._h = h
        self.device = device
        if max_batch > 0:
            self.reserve(max_batch, candidate_capacity)

    # -------------------------------------------------------------- lifecycle
    def reserve(self, max_batch: int, candidate_capacity: int = 0) -> None:
        _abi.check(self._lib.hvp_reserve(self._h, int(max_batch), int(candidate_capacity)), "hvp_reserve")

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.hvp_destroy(self._h)
            self._h = None

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    @property
    def params_stride(self) -> int:
        return _abi.params_stride(self.N, int(self.problem.formulation))

    def stats(self) -> _abi.HvpStats:
        s = _abi.HvpStats()
        _abi.check(self._lib.hvp_get_stats(self._h, ctypes.byref(s)), "hvp_get_stats")
        return s

    # -------------------------------------------------------------- host path
    def solve(self, sys_idx, roles, params) -> BatchResult:
        N = self.N
        sys_idx = np.ascontiguousarray(np.asarray(sys_idx, dtype=np.int32).reshape(-1))
        roles = np.ascontiguousarray(np.asarray(roles, dtype=np.int32).reshape(-1))
        params = np.ascontiguousarray(np.asarray(params, dtype=np.float64).reshape(len(roles), -1))
        B = len(roles)
        if params.shape[1] != self.params_stride or len(sys_idx) != B:
            raise ValueError(f"params must be (B, {self.params_stride}) and sys_idx (B,)")
        if B and (sys_idx.min() < 0 or sys_idx.max() >= self.n_systems):
            raise ValueError("system index out of range")
        out = BatchResult(
            u=np.zeros((B, N)), x=np.zeros((B, 2, N + 1)), region=np.zeros((B, N), np.int8),
            gear=np.zeros((B, N), np.int8), cost=np.zeros(B), status=np.zeros(B, np.int32),
            nodes=np.zeros(B, np.int32), iters=np.zeros(B, np.int32),
        )
        if B == 0:
            return out
        self._solve_host(sys_idx, roles, params, out)
        # the search workspace is pooled over the batch with a per-instance share: instances whose
        # search outgrew it (HVP_OVERFLOW, reported, never truncated) are re-solved on their own,
        # where the share is the whole workspace, growing it if needed
        for attempt in range(4):
            over = np.flatnonzero(out.status == _abi.OVERFLOW)
            if not len(over):
                break
            if attempt:
                self.reserve(max(B, 1), 4 * self.stats().capacity)
            sub = BatchResult(**{k: v[over].copy() for k, v in out.__dict__.items()})
            with self._hint_cleared():  # hint rows and node records are indexed by the full batch
                self._solve_host(sys_idx[over], roles[over], np.ascontiguousarray(params[over]), sub)
            for k, v in sub.__dict__.items():
                getattr(out, k)[over] = v
        return out

    def _solve_host(self, sys_idx, roles, params, out: BatchResult) -> None:
        P = lambda a, t: a.ctypes.data_as(ctypes.POINTER(t))  # noqa: E731
        d, i32, i8 = ctypes.c_double, ctypes.c_int32, ctypes.c_int8
        rc = self._lib.hvp_solve_batch_host(
            self._h, len(roles), P(sys_idx, i32), P(roles, i32), P(params, d), P(out.u, d), P(out.x, d),
            P(out.region, i8), P(out.gear, i8), P(out.cost, d), P(out.status, i32), P(out.nodes, i32),
            P(out.iters, i32))
        _abi.check(rc, "hvp_solve_batch_host")

    # -------------------------------------------------------------- device path
    def alloc_outputs(self, B: int, device=None) -> dict:
        import torch

        dev = device or torch.device("cuda", self.device)
        N = self.N
        return {
            "u": torch.empty((B, N), dtype=torch.float64, device=dev),
            "x": torch.empty((B, 2, N + 1), dtype=torch.float64, device=dev),
            "region": torch.empty((B, N), dtype=torch.int8, device=dev),
            "gear": torch.empty((B, N), dtype=torch.int8, device=dev),
            "cost": torch.empty((B,), dtype=torch.float64, device=dev),
            "status": torch.empty((B,), dtype=torch.int32, device=dev),
            "nodes": torch.empty((B,), dtype=torch.int32, device=dev),
            "iters": torch.empty((B,), dtype=torch.int32, device=dev),
        }

    def solve_device(self, sys_idx, roles, params, out: dict | None = None, stream=None,
                     retry_overflow: bool = False) -> dict:
        """Solve of device-resident tensors; returns (and fills) the output dict.

        Asynchronous unless ``retry_overflow``: instances whose search outgrew their share of the
        workspace come back as HVP_OVERFLOW; with ``retry_overflow`` they are gathered on the
        device and re-solved on their own (synchronising once per retry round)."""
        import torch

        out = self._launch(sys_idx, roles, params, out, stream)
        for attempt in range(4 if retry_overflow else 0):
            over = torch.nonzero(out["status"] == _abi.OVERFLOW).reshape(-1)
            if over.numel() == 0:
                break
            if attempt:
                self.reserve(int(roles.shape[0]), 4 * self.stats().capacity)
            with self._hint_cleared():  # the hint rows are indexed by the full batch: not for the subset
                sub = self._launch(sys_idx[over].contiguous(), roles[over].contiguous(), params[over].contiguous(),
                                   None, stream)
            for k, v in sub.items():
                out[k][over] = v
        return out

    def _launch(self, sys_idx, roles, params, out, stream) -> dict:
        import torch

        B = int(roles.shape[0])
        for name, t, dt in (("sys_idx", sys_idx, torch.int32), ("roles", roles, torch.int32),
                            ("params", params, torch.float64)):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous CUDA tensor of dtype {dt}")
        if params.numel() != B * self.params_stride or sys_idx.numel() != B:
            raise ValueError("params must be (B, params_stride), sys_idx (B,)")
        self._check_hint(B)
        out = out or self.alloc_outputs(B, params.device)
        if stream is None:
            stream = torch.cuda.current_stream(params.device)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = self._lib.hvp_solve_batch(
            self._h, B, ptr(sys_idx), ptr(roles), ptr(params), ptr(out["u"]), ptr(out["x"]), ptr(out["region"]),
            ptr(out["gear"]), ptr(out["cost"]), ptr(out["status"]), ptr(out["nodes"]), ptr(out["iters"]),
            ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_solve_batch")
        return out

    # -------------------------------------------------------------- neighbour predictions
    def decent_params_device(self, x, leader_window, x_prev=None, leader_index: int = 0,
                             real_vehicle_as_reference: bool = False, estimator: str = "none",
                             params=None, roles=None, stream=None):
        """hvp_decent_params_batch: the local-MPC parameter blocks and roles of P platoons from
        their measured states x (P, 2n) on the device (observe_states, fleet_decent_mld.py:348-455).
        leader_window (P, 2, N+1).  Returns (params (P*n, stride), roles (P*n,))."""
        import torch

        P, n2 = int(x.shape[0]), int(x.shape[1])
        n = n2 // 2
        est = {"none": 0, "two_point": 1, "sat": 2}[estimator]
        dev = x.device
        for name, t, shape in (("x", x, (P, n2)), ("leader_window", leader_window, (P, 2, self.N + 1))):
            if not t.is_cuda or t.dtype != torch.float64 or not t.is_contiguous() or tuple(t.shape) != shape:
                raise ValueError(f"{name} must be a contiguous CUDA float64 {shape} tensor")
        if params is None:
            params = torch.empty((P * n, self.params_stride), dtype=torch.float64, device=dev)
        if roles is None:
            roles = torch.empty(P * n, dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        rc = self._lib.hvp_decent_params_batch(self._h, P, n, ptr(x), ptr(x_prev), ptr(leader_window),
                                               int(leader_index), 1 if real_vehicle_as_reference else 0, est,
                                               ptr(params), ptr(roles), ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_decent_params_batch")
        return params, roles

    # -------------------------------------------------------------- fixed-control evaluation
    def evaluate_device(self, sys_idx, roles, params, gears, u, stream=None) -> dict:
        """Cost of fixed controls u (B, N) and gear labels (B, N) on the device (hvp_evaluate_batch:
        MpcGear.evaluate_cost, mpcs/mpc_gear.py:137-170).  Returns cost, status, x."""
        import torch

        B = int(roles.shape[0])
        dev = params.device
        for name, t, dt in (("gears", gears, torch.int8), ("u", u, torch.float64)):
            if not t.is_cuda or t.dtype != dt or not t.is_contiguous() or t.numel() != B * self.N:
                raise ValueError(f"{name} must be a contiguous CUDA ({B}, {self.N}) tensor of dtype {dt}")
        out = {"cost": torch.empty(B, dtype=torch.float64, device=dev),
               "status": torch.empty(B, dtype=torch.int32, device=dev),
               "x": torch.empty((B, 2, self.N + 1), dtype=torch.float64, device=dev)}
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = self._lib.hvp_evaluate_batch(self._h, B, ptr(sys_idx), ptr(roles), ptr(params), ptr(gears), ptr(u),
                                          ptr(out["cost"]), ptr(out["status"]), ptr(out["x"]),
                                          ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_evaluate_batch")
        return out

    def evaluate(self, sys_idx, roles, params, gears, u) -> dict:
        """Host-array form of :meth:`evaluate_device` (synchronous)."""
        import torch

        dev = torch.device("cuda", self.device)
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).reshape(-1).to(dev)  # noqa: E731
        B = len(np.asarray(roles).reshape(-1))
        out = self.evaluate_device(t(sys_idx, torch.int32), t(roles, torch.int32),
                                   t(params, torch.float64).reshape(B, -1), t(gears, torch.int8).reshape(B, self.N),
                                   t(u, torch.float64).reshape(B, self.N))
        torch.cuda.synchronize(dev)
        return {k: v.cpu().numpy() for k, v in out.items()}

    # -------------------------------------------------------------- ADMM formulation
    def set_region_hint(self, region) -> None:
        """hvp_set_region_hint: a (B, N) int8 device tensor of region sequences (the "region" output
        of the previous ADMM iteration, or the previous time step's sequences shifted by one step)
        that later solves try as a second initial incumbent -- naive-ADMM solves and decentralised
        solves with N > 8; None clears it.  Only pruning changes, never the answer."""
        import torch

        if region is not None and (not region.is_cuda or region.dtype != torch.int8 or not region.is_contiguous()
                                   or region.dim() != 2 or int(region.shape[1]) != self.N):
            raise ValueError(f"the region hint must be a contiguous CUDA (B, {self.N}) int8 tensor")
        rc = self._lib.hvp_set_region_hint(self._h, ctypes.c_void_p(region.data_ptr() if region is not None else 0))
        _abi.check(rc, "hvp_set_region_hint")
        self._hint = region

    def _check_hint(self, B: int) -> None:
        """The kernels read hint[i * N + k] for every instance i < B."""
        hint = getattr(self, "_hint", None)
        if hint is not None and int(hint.shape[0]) < B:
            raise ValueError(f"the region hint holds {int(hint.shape[0])} rows for a batch of {B}: "
                             "set a matching hint or clear it (set_region_hint(None))")

    @contextlib.contextmanager
    def _hint_cleared(self):
        """For a solve of a subset of the batch: the region hint and the naive-ADMM node records
        (hvp_set_node_records) are indexed by the full batch's positions, so neither is used."""
        hint = getattr(self, "_hint", None)
        if hint is not None:
            self.set_region_hint(None)
        _abi.check(self._lib.hvp_set_node_records(self._h, 0), "hvp_set_node_records")
        try:
            yield
        finally:
            _abi.check(self._lib.hvp_set_node_records(self._h, 1), "hvp_set_node_records")
            if hint is not None:
                self.set_region_hint(hint)

    def solve_admm_device(self, sys_idx, roles, params, out: dict, stream=None, retry_overflow: bool = False) -> dict:
        """hvp_solve_admm_batch on device tensors; ``out`` also needs "x_front", "x_back".
        ``retry_overflow`` as in :meth:`solve_device`."""
        import torch

        self._launch_admm(sys_idx, roles, params, out, stream)
        for attempt in range(4 if retry_overflow else 0):
            over = torch.nonzero(out["status"] == _abi.OVERFLOW).reshape(-1)
            if over.numel() == 0:
                break
            if attempt:
                self.reserve(int(roles.shape[0]), 4 * self.stats().capacity)
            sub = {k: torch.empty_like(v[over]) for k, v in out.items()}
            with self._hint_cleared():  # the hint rows are indexed by the full batch: not for the subset
                self._launch_admm(sys_idx[over].contiguous(), roles[over].contiguous(), params[over].contiguous(),
                                  sub, stream)
            for k, v in sub.items():
                out[k][over] = v
        return out

    def _launch_admm(self, sys_idx, roles, params, out: dict, stream=None) -> dict:
        import torch

        B = int(roles.shape[0])
        if params.numel() != B * self.params_stride:
            raise ValueError("params must be (B, hvp_params_stride_admm)")
        self._check_hint(B)
        if stream is None:
            stream = torch.cuda.current_stream(params.device)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        rc = self._lib.hvp_solve_admm_batch(
            self._h, B, ptr(sys_idx), ptr(roles), ptr(params), ptr(out["u"]), ptr(out["x"]), ptr(out["region"]),
            ptr(out["gear"]), ptr(out["cost"]), ptr(out["status"]), ptr(out["nodes"]), ptr(out["iters"]),
            ptr(out["x_front"]), ptr(out["x_back"]), ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_solve_admm_batch")
        return out

    def admm_update(self, P: int, n: int, x, xf, xb, y_front, y_back, params, z=None, stream=None) -> None:
        """hvp_admm_update: z / y update and next parameter blocks (device tensors, async)."""
        import torch

        if stream is None:
            stream = torch.cuda.current_stream(params.device)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr() if t is not None else 0)  # noqa: E731
        rc = self._lib.hvp_admm_update(self._h, int(P), int(n), ptr(x), ptr(xf), ptr(xb), ptr(y_front), ptr(y_back),
                                       ptr(params), ptr(z), ctypes.c_void_p(stream.cuda_stream))
        _abi.check(rc, "hvp_admm_update")

    def solve_admm(self, sys_idx, roles, params) -> BatchResult:
        """Host-array form of :meth:`solve_admm_device` (synchronous); the result also carries
        x_front / x_back (B, 2, N+1)."""
        import torch

        dev = torch.device("cuda", self.device)
        roles = np.asarray(roles, np.int32).reshape(-1)
        B = len(roles)
        t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a), dtype=dt).to(dev)  # noqa: E731
        out = self.alloc_outputs(B, dev)
        out["x_front"] = torch.zeros((B, 2, self.N + 1), dtype=torch.float64, device=dev)
        out["x_back"] = torch.zeros((B, 2, self.N + 1), dtype=torch.float64, device=dev)
        self.solve_admm_device(t(np.asarray(sys_idx).reshape(-1), torch.int32), t(roles, torch.int32),
                               t(np.asarray(params).reshape(B, -1), torch.float64), out)
        torch.cuda.synchronize(dev)
        h = {k: v.cpu().numpy() for k, v in out.items()}
        res = BatchResult(u=h["u"], x=h["x"], region=h["region"], gear=h["gear"], cost=h["cost"], status=h["status"],
                          nodes=h["nodes"], iters=h["iters"])
        res.x_front, res.x_back = h["x_front"], h["x_back"]
        return res
