"""The C ABI library: builds for gfx950, loads without a GPU and exports every symbol of
include/hvp.h with the struct layouts the ctypes binding assumes (no compute call)."""

from __future__ import annotations

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hybrid-vehicle-platoon_amd")


def header_functions() -> set[str]:
    src = open(os.path.join(ROOT, "include", "hvp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:int|void|const char\s*\*)\s+(hvp_\w+)\s*\(", src, flags=re.M)) - {
        "hvp_params_stride"}


def abi_digest() -> str:
    """SHA-256 over include/hvp.h's declarations with comments and whitespace runs removed: the
    struct definitions, enums, inline helpers and every prototype.  Any change of a field, a
    signature or an export changes it; comment edits do not."""
    import hashlib

    src = open(os.path.join(ROOT, "include", "hvp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    src = src.replace("#define HVP_ABI_VERSION", "#define HVP_ABI_VERSION_")  # the version is the key
    src = re.sub(r"#define HVP_ABI_VERSION_\s+\d+", "", src)
    return hashlib.sha256(" ".join(src.split()).encode()).hexdigest()


# One entry per released ABI version: (sizeof hvp_system, hvp_problem, hvp_stats) and abi_digest().
# A header change without a version bump fails test_abi_change_bumps_the_version; when the change is
# deliberate, bump HVP_ABI_VERSION (include/hvp.h, hvp/_abi.py), add the new entry here and note the
# change in INTEGRATION.md's ABI history.
ABI_MANIFEST = {
    5: ((768, 152, 72), "039ded6e2bca5fd6408117c0885b6e007dedd7d49a60bfa8b8714821c85f9606"),
}


def test_abi_change_bumps_the_version():
    """hvp_stats grew (n_spilled) and hvp_set_node_records was added in round 5
    under ABI 4, so a round-4 caller would have passed a 64-byte hvp_stats that the library
    overran by 8 bytes.  The layout and the declarations are pinned per version."""
    import ctypes

    from hvp import _abi

    lib = _abi.load()
    assert lib.hvp_abi_version() == _abi.ABI_VERSION
    sizes = (ctypes.c_int32 * 3)()
    lib.hvp_abi_sizes(sizes)
    assert _abi.ABI_VERSION in ABI_MANIFEST, "a new ABI version needs its ABI_MANIFEST entry"
    want_sizes, want_digest = ABI_MANIFEST[_abi.ABI_VERSION]
    assert tuple(sizes) == want_sizes, ("struct sizes changed: bump HVP_ABI_VERSION", tuple(sizes))
    assert abi_digest() == want_digest, ("include/hvp.h declarations changed: bump HVP_ABI_VERSION",
                                         abi_digest())
    for old in ABI_MANIFEST:
        if old != _abi.ABI_VERSION:
            assert ABI_MANIFEST[old][1] != want_digest, f"ABI {_abi.ABI_VERSION} equals ABI {old}"


def test_library_builds_and_exports_the_header():
    from hvp import _abi

    subprocess.run(["make", "-s", "-C", PKG, "lib/libhvpsolve.so"], check=True)  # no-op when up to date
    lib = _abi.load()  # checks ABI version and struct sizes
    funcs = header_functions()
    assert funcs == set(_abi.EXPORTS), funcs ^ set(_abi.EXPORTS)
    for f in funcs:
        assert hasattr(lib, f), f
    nm = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    for f in funcs:
        assert re.search(rf"\bT {f}\b", nm), f


def test_code_object_targets_gfx950():
    from hvp import _abi

    # the fat binary embeds the amdgcn code object; its target id names the architecture
    assert b"amdgcn-amd-amdhsa--gfx950" in open(_abi.LIB_PATH, "rb").read()


def test_invalid_arguments_fail_loudly_without_touching_the_gpu():
    import ctypes

    from hvp import _abi, tables
    from hvp.models import PwaGearVehicle

    lib = _abi.load()
    h = ctypes.c_void_p()
    veh = PwaGearVehicle(800)
    sysv = (_abi.HvpSystem * 1)(tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh)))
    bad = tables.problem(17)  # beyond HVP_MAX_N
    assert lib.hvp_create(ctypes.byref(h), ctypes.byref(bad), sysv, 1, 0) == -3
    assert "horizon" in _abi.last_error()
    enum12 = tables.problem(12, method=_abi.METHOD_ENUMERATE)  # enumeration stops at HVP_MAX_N_ENUM
    assert lib.hvp_create(ctypes.byref(h), ctypes.byref(enum12), sysv, 1, 0) == -3
    assert "enumeration" in _abi.last_error()
    badm = tables.problem(5, method=7)
    assert lib.hvp_create(ctypes.byref(h), ctypes.byref(badm), sysv, 1, 0) == -1
    # min_1_norm runs for the decentralised formulation at every horizon (enumeration up to
    # HVP_MAX_N_ENUM, branch and bound beyond): accepted (on a CPU-only host the device step fails)
    for l1 in (tables.problem(10, quadratic_cost=False), tables.problem(16, quadratic_cost=False),
               tables.problem(5, quadratic_cost=False, method=_abi.METHOD_BNB)):
        rc = lib.hvp_create(ctypes.byref(h), ctypes.byref(l1), sysv, 1, 0)
        assert rc in (0, -2), (rc, _abi.last_error())
        if rc == 0:
            lib.hvp_destroy(h)
    from hvp.admm import admm_problem

    l1a = admm_problem(5, 0.5, quadratic_cost=False)  # naive-ADMM min_1_norm: accepted (round 6)
    rc = lib.hvp_create(ctypes.byref(h), ctypes.byref(l1a), sysv, 1, 0)
    assert rc in (0, -2), (rc, _abi.last_error())
    if rc == 0:
        lib.hvp_destroy(h)
    badq = tables.problem(5)
    badq.quadratic_cost = 2
    assert lib.hvp_create(ctypes.byref(h), ctypes.byref(badq), sysv, 1, 0) == -1


def test_min_1_norm_acceptance_matches_integration_doc():
    """INTEGRATION.md section 1 states which problems take quadratic_cost = 0 (min_1_norm,
    fleet_decent_mld.py:73-76, fleet_naive_admm.py:74-77, mpcs/cent_mld.py:58-61): HVP_FORM_DECENT
    at every N <= 16, HVP_FORM_ADMM and HVP_FORM_CENT are accepted, the switching-ADMM form returns
    HVP_E_UNSUPPORTED.  hvp_create validates before it touches a device, so on a CPU-only host an
    accepted problem fails at the device step (HVP_E_HIP = -2) and a rejected one with
    HVP_E_UNSUPPORTED (-3)."""
    import ctypes

    from hvp import _abi, tables
    from hvp.admm import admm_problem
    from hvp.cent import cent_problem
    from hvp.gadmm import gadmm_problem
    from hvp.models import PwaGearVehicle

    lib = _abi.load()
    h = ctypes.c_void_p()
    veh = PwaGearVehicle(800)
    sysv = (_abi.HvpSystem * 1)(tables.system_from_dict(veh.get_discrete_system(1), tables.gears_of(veh)))

    def rc(p):
        r = lib.hvp_create(ctypes.byref(h), ctypes.byref(p), sysv, 1, 0)
        if r == 0:
            lib.hvp_destroy(h)
        return r

    for p in (tables.problem(10, quadratic_cost=False), cent_problem(5, quadratic_cost=False),
              cent_problem(5, quadratic_cost=False, exhaustive=True), admm_problem(10, 0.5, quadratic_cost=False),
              admm_problem(5, 0.5, quadratic_cost=False)):
        assert rc(p) in (0, -2), _abi.last_error()
    g = gadmm_problem(10)
    g.quadratic_cost = 0
    assert rc(g) == -3
    assert "min_1_norm" in _abi.last_error()
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    assert "HVP_FORM_CENT` accepts it" in doc and "solved by enumeration with" not in doc
    assert "`HVP_FORM_ADMM` accepts it" in doc and "`HVP_FORM_GADMM` with `quadratic_cost = 0` returns" in doc


def test_no_device_function_clobbers_its_return_address():
    """Round 4's k_bnb_ipm<10> hang, root-caused in round 5 (tests/codeobj_audit.py, DESIGN.md
    section 4): ROCm 7.2's branch relaxation routes out-of-range branches of a non-kernel function
    through s[30:31], its return address, so the function never returns.  No function of the
    built library may carry such a branch (the product force-inlines its solvers; the hung build's
    Solver<9>/<10>::solve are caught by the same check, profiles/r05e_codeobj_audit.txt)."""
    import shutil

    from codeobj_audit import OBJDUMP, audit

    from hvp import _abi

    if not os.path.exists(_abi.LIB_PATH) or not shutil.which(OBJDUMP):
        pytest.skip("needs the built library and llvm-objdump")
    n, bad = audit(_abi.LIB_PATH)
    assert n >= 18  # the 18 translation units' gfx950 code objects
    assert not bad, bad
