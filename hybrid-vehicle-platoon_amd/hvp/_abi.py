"""ctypes mirror of include/hvp.h and the loader of libhvpsolve.so.

The product path has exactly one backend: the HIP library built from csrc/hvp_kernels.hip.
If it is missing, :func:`load` raises -- there is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os

MAX_REGIONS = 16
MAX_N = 16
MAX_N_ENUM = 8
ABI_VERSION = 5

METHOD_AUTO, METHOD_ENUMERATE, METHOD_BNB = 0, 1, 2
FORM_DECENT, FORM_ADMM, FORM_GADMM, FORM_CENT = 0, 1, 2, 3

ROLE_SAFE_FRONT = 1
ROLE_SAFE_BACK = 2
ROLE_TRACK_FRONT = 4
ROLE_TRACK_BACK = 8
ROLE_TRACK_LEADER = 16
ROLE_LEADER_SPACING = 32
ROLE_BACK_COPY = 64

# switching-ADMM platoon state bits (include/hvp.h)
GADMM_LIVE, GADMM_FAILED, GADMM_CHANGED = 1, 2, 4

OPTIMAL, INFEASIBLE, MAXITER, OVERFLOW = 0, 1, 2, 3
STATUS_NAMES = {OPTIMAL: "OPTIMAL", INFEASIBLE: "INFEASIBLE", MAXITER: "MAXITER", OVERFLOW: "OVERFLOW"}

_D8 = ctypes.c_double * MAX_REGIONS


class HvpSystem(ctypes.Structure):
    _fields_ = [
        ("n_regions", ctypes.c_int32),
        ("gear", ctypes.c_int32 * MAX_REGIONS),
        ("pad_", ctypes.c_int32),
        ("ts", ctypes.c_double),
        ("a", _D8),
        ("b", _D8),
        ("c", _D8),
        ("vlo", _D8),
        ("vhi", _D8),
        ("pmin", ctypes.c_double),
        ("pmax", ctypes.c_double),
        ("vmin", ctypes.c_double),
        ("vmax", ctypes.c_double),
        ("umin", ctypes.c_double),
        ("umax", ctypes.c_double),
    ]


class HvpProblem(ctypes.Structure):
    _fields_ = [
        ("N", ctypes.c_int32),
        ("quadratic_cost", ctypes.c_int32),
        ("Qx", ctypes.c_double * 4),
        ("Qu", ctypes.c_double),
        ("Qdu", ctypes.c_double),
        ("w", ctypes.c_double),
        ("a_acc", ctypes.c_double),
        ("a_dec", ctypes.c_double),
        ("ts_acc", ctypes.c_double),
        ("d_safe", ctypes.c_double),
        ("accel_tightening", ctypes.c_double),
        ("spacing_d0", ctypes.c_double),
        ("spacing_t0", ctypes.c_double),
        ("max_iter", ctypes.c_int32),
        ("method", ctypes.c_int32),
        ("tol", ctypes.c_double),
        ("formulation", ctypes.c_int32),
        ("pad_", ctypes.c_int32),
        ("rho", ctypes.c_double),
    ]


class HvpStats(ctypes.Structure):
    _fields_ = [
        ("n_instances", ctypes.c_int64),
        ("n_candidates", ctypes.c_int64),
        ("qp_iterations", ctypes.c_int64),
        ("capacity", ctypes.c_int64),
        ("last_ms", ctypes.c_double),
        ("qp_ms", ctypes.c_double),
        ("n_fallback", ctypes.c_int64),
        ("n_failed_bounds", ctypes.c_int64),
        ("n_spilled", ctypes.c_int64),
    ]


def params_stride(N: int, formulation: int = 0) -> int:
    return 2 + {FORM_ADMM: 10, FORM_GADMM: 14}.get(formulation, 6) * (N + 1)


_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(_PKG_ROOT, "lib")
# HVP_LIB: an alternative build of the same library (A/B kernel variants); default the in-tree build
LIB_PATH = os.environ.get("HVP_LIB") or os.path.join(LIB_DIR, "libhvpsolve.so")
HOSTREF_PATH = os.path.join(LIB_DIR, "libhvp_hostref.so")

_lib = None

_P = ctypes.c_void_p
_I32P = ctypes.POINTER(ctypes.c_int32)
_DP = ctypes.POINTER(ctypes.c_double)
_I8P = ctypes.POINTER(ctypes.c_int8)

# exported symbol -> (argtypes, restype); also the list the CPU tests check
EXPORTS = {
    "hvp_create": ([ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(HvpProblem), ctypes.POINTER(HvpSystem),
                    ctypes.c_int, ctypes.c_int], ctypes.c_int),
    "hvp_reserve": ([_P, ctypes.c_int, ctypes.c_int64], ctypes.c_int),
    "hvp_solve_batch": ([_P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "hvp_solve_batch_host": ([_P, ctypes.c_int, _I32P, _I32P, _DP, _DP, _DP, _I8P, _I8P, _DP, _I32P, _I32P,
                              _I32P], ctypes.c_int),
    "hvp_evaluate_batch": ([_P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P], ctypes.c_int),
    "hvp_solve_admm_batch": ([_P, ctypes.c_int] + [_P] * 14, ctypes.c_int),
    "hvp_set_region_hint": ([_P, _P], ctypes.c_int),
    "hvp_set_node_records": ([_P, ctypes.c_int], ctypes.c_int),
    "hvp_admm_update": ([_P, ctypes.c_int, ctypes.c_int] + [_P] * 8, ctypes.c_int),
    "hvp_gadmm_rollout": ([_P] + [ctypes.c_int] * 4 + [_P, _P, ctypes.c_int] + [_P] * 6, ctypes.c_int),
    "hvp_gadmm_solve": ([_P] + [ctypes.c_int] * 4 + [_P] * 14, ctypes.c_int),
    "hvp_gadmm_update": ([_P] + [ctypes.c_int] * 4 + [_P] * 5 + [ctypes.c_int, _P], ctypes.c_int),
    "hvp_gadmm_switch": ([_P] + [ctypes.c_int] * 4 + [_P] * 5, ctypes.c_int),
    "hvp_cent_solve_batch": ([_P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _P, _P, _P, ctypes.c_int]
                             + [_P] * 9, ctypes.c_int),
    "hvp_env_step_batch": ([_P, ctypes.c_int, ctypes.c_int] + [_P] * 6 + [ctypes.c_int, ctypes.c_int, ctypes.c_double]
                           + [_P] * 4, ctypes.c_int),
    "hvp_decent_params_batch": ([_P, ctypes.c_int, ctypes.c_int, _P, _P, _P, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 _P, _P, _P], ctypes.c_int),
    "hvp_sync": ([_P, _P], ctypes.c_int),
    "hvp_get_stats": ([_P, ctypes.POINTER(HvpStats)], ctypes.c_int),
    "hvp_destroy": ([_P], None),
    "hvp_last_error": ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
    "hvp_abi_version": ([], ctypes.c_int),
    "hvp_abi_sizes": ([_I32P], ctypes.c_int),
}


class HvpError(RuntimeError):
    pass


def _init_torch_runtime() -> None:
    """Let torch's HIP runtime claim the devices first.  The library links the system HIP
    runtime; when it touches a device before torch does, torch's own runtime (the device-tensor
    marshalling) finds no GPU.  Without torch or without a GPU this is a no-op."""
    try:
        import torch
    except ImportError:  # pragma: no cover - torch is part of the image
        return
    if torch.cuda.is_available():
        torch.cuda.init()


def load():
    """Load libhvpsolve.so (built by ``make -C hybrid-vehicle-platoon_amd``); raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HvpError(
            f"{LIB_PATH} not found: build the HIP library first (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C hybrid-vehicle-platoon_amd). There is no CPU fallback."
        )
    _init_torch_runtime()
    lib = ctypes.CDLL(LIB_PATH)
    for name, (argt, rest) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = rest
    if lib.hvp_abi_version() != ABI_VERSION:
        raise HvpError(f"libhvpsolve ABI {lib.hvp_abi_version()} != expected {ABI_VERSION}")
    sizes = (ctypes.c_int32 * 3)()
    lib.hvp_abi_sizes(sizes)
    want = (ctypes.sizeof(HvpSystem), ctypes.sizeof(HvpProblem), ctypes.sizeof(HvpStats))
    if tuple(sizes) != want:
        raise HvpError(f"struct layout mismatch: library {tuple(sizes)} vs binding {want}")
    _lib = lib
    return lib


_lib_sha = None


def lib_sha256() -> str:
    """SHA-256 of the library file this process loads (LIB_PATH): the stamp profiles/ summaries
    carry, so a roofline figure is only ever taken from a profile of the same binary."""
    global _lib_sha
    if _lib_sha is None:
        import hashlib

        with open(LIB_PATH, "rb") as f:
            _lib_sha = hashlib.sha256(f.read()).hexdigest()
    return _lib_sha


def last_error() -> str:
    buf = ctypes.create_string_buffer(1024)
    load().hvp_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise HvpError(f"{what} failed ({rc}): {last_error()}")
