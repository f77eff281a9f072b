"""Audit of the product library's gfx950 machine code for the compiler bug behind round 4's hang.

ROCm 7.2's LLVM AMDGPU backend (clang 22.0.0git roc-7.2.0) relaxes a branch that is out of the
+-128 KB range of s_branch / s_cbranch into ``s_getpc_b64 s[30:31]; s_add_u32 s30, ...;
s_addc_u32 s31, ...; s_setpc_b64 s[30:31]``.  In a kernel s[30:31] is an ordinary register pair;
in a NON-kernel function it holds the return address (AMDGPU calling convention), which the
expansion overwrites without saving: the function's final ``s_setpc_b64 s[30:31]`` then jumps to
the last long-branch target instead of the caller and the wave loops inside the function for
ever.  Round 4's outlined ``Solver<10>::solve`` (204 KB: every IPM fallback kernel of one
translation unit called it) was such a function -- k_bnb_ipm<10> never returned on MI355X
(profiles/r05e_hang_markers.txt: every working lane passed the solver's converged return, none
reached the instruction after the call).  The product force-inlines the solvers
(hvp_ipm.h HVP_FORCEINLINE); this audit checks the built library for any function that still
carries such a branch.

Test infrastructure (tests/test_abi.py) and a command-line tool:

    python tests/codeobj_audit.py hybrid-vehicle-platoon_amd/lib/libhvpsolve.so
"""

from __future__ import annotations

import concurrent.futures as cf
import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def device_code_objects(path: str) -> list[bytes]:
    """Every amdgcn code object in the clang offload bundles embedded in a HIP shared library."""
    data = open(path, "rb").read()
    objs, pos = [], 0
    while True:
        i = data.find(_MAGIC, pos)
        if i < 0:
            return objs
        n = struct.unpack_from("<Q", data, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "amdgcn" in triple and size:
                objs.append(data[i + off:i + off + size])
        pos = i + 1


def _kernels(syms: str) -> set[str]:
    """Kernel entry symbols of a code object: the names that have a ``<name>.kd`` descriptor."""
    out = set()
    for line in syms.splitlines():
        name = line.split()[-1] if line.strip() else ""
        if name.endswith(".kd"):
            out.add(name[:-3])
    return out


def _scan(code: bytes) -> dict:
    """{function: (long branches through s[30:31], s_setpc_b64 s[30:31])} of one code object's
    NON-kernel functions (in a kernel s[30:31] is an ordinary register pair, so a kernel's long
    branch through it is harmless and not reported)."""
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(code)
        f.flush()
        dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], capture_output=True, text=True,
                             check=True).stdout
        kernels = _kernels(subprocess.run([OBJDUMP, "--syms", f.name], capture_output=True, text=True,
                                          check=True).stdout)
    cur, funcs = None, {}
    for line in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", line)
        if m:
            cur = m.group(1)
            funcs[cur] = [0, 0]
        elif cur is not None:
            if "s_getpc_b64 s[30:31]" in line:
                funcs[cur][0] += 1
            elif "s_setpc_b64 s[30:31]" in line:
                funcs[cur][1] += 1
    return {k: tuple(v) for k, v in funcs.items() if v[0] and k not in kernels}


def audit(path: str) -> tuple[int, dict]:
    """(number of device code objects, {function: counts} of the functions whose long branches go
    through the return-address registers)."""
    objs = device_code_objects(path)
    bad = {}
    with cf.ThreadPoolExecutor(min(8, os.cpu_count() or 1)) as ex:
        for found in ex.map(_scan, objs):
            bad.update(found)
    return len(objs), bad


if __name__ == "__main__":
    n, bad = audit(sys.argv[1])
    print(f"{n} device code objects")
    for name, (g, s) in sorted(bad.items()):
        print(f"{name}: {g} long branches through s[30:31], {s} s_setpc_b64 s[30:31]")
    print("functions clobbering the return address:", len(bad))
    sys.exit(1 if bad else 0)
