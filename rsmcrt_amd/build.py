"""Build the HIP engine library in-tree: rsmcrt_amd/libsmcrt.so (gfx950).

Plain hipcc, no torch extension machinery: every source compiles to an object in parallel and
one link makes the C-ABI shared object (include/smcrt.h) that Fortran/C/Python can bind.
Objects are kept in rsmcrt_amd/.objs/<arch>-<flags hash>/ (git-ignored) and rebuilt only when
their source or a header it includes (found by scanning `#include "..."` lines) is newer.
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import glob
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB = os.path.join(PKG, "libsmcrt.so")
SOURCES = [os.path.join(PKG, "csrc", f) for f in ("smcrt.hip", "writers.cpp", "frontend.cpp", "sources.cpp", "png.cpp", "escape.cpp", "inverse.cpp", "spectral.cpp", "multi.hip", "cull.cpp")]
# the transport kernel instantiations: kinst.hip once per (LDS faces, grid mode), kernel_ptrs.h
KINST = os.path.join(PKG, "csrc", "kinst.hip")
# Part 1 (the plain ws_kernel, M1's lean path) schedules with the AMDGPU register-pressure
# trackers: M1 259.0/260.2 vs 257.8/257.3 M photons/s same box, while the XF ws_kernel (M3)
# lost 1.7 % with them (profiles/r06_s7/ab_sched_strategy.txt), so part 0 keeps the default.
PLAIN_WS_FLAGS = ("-mllvm", "--amdgpu-use-amdgpu-trackers")
UNITS = [(src, ()) for src in SOURCES] + [
    (KINST, (f"-DKI_F={f}", f"-DKI_G={g}", f"-DKI_P={p}") + (PLAIN_WS_FLAGS if p else ()))
    for f in (0, 1) for g in (0, 1, 2) for p in (0, 1)]
DEPS = SOURCES + [KINST] + sorted(glob.glob(os.path.join(PKG, "csrc", "*.h"))) + [os.path.join(ROOT, "include", "smcrt.h")]
ARCH = os.environ.get("SMCRT_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: no fused multiply-add, so fp64 trajectories are bit-identical to the
# CPU restatement (oracle/), which is compiled the same way.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         f"--offload-arch={ARCH}", "-Wall"]
# objects are cached per target and flag set, so a change of either never links stale objects
OBJDIR = os.path.join(PKG, ".objs", ARCH + "-" + hashlib.sha256(" ".join(FLAGS).encode()).hexdigest()[:12])
_INC = re.compile(r'^\s*#\s*include\s+"([^"]+)"', re.M)


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def includes(path: str, seen=None) -> set:
    """The file and every local header it includes, transitively."""
    seen = set() if seen is None else seen
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    with open(path, errors="replace") as f:
        for name in _INC.findall(f.read()):
            includes(os.path.join(os.path.dirname(path), name), seen)
    return seen


def _obj(src: str, defs=(), variant: str = "") -> str:
    tag = "".join("." + d.lstrip("-D").replace("=", "") for d in defs) + ("." + variant if variant else "")
    return os.path.join(OBJDIR, os.path.basename(src) + tag + ".o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def _compile_and_link(out: str, extra=(), variant: str = "", force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJDIR, exist_ok=True)
    # a variant's flags reach every unit (its objects are tagged with the variant's name)
    var = [bool(variant) for _ in UNITS]
    objs = [_obj(src, defs, variant if var[i] else "") for i, (src, defs) in enumerate(UNITS)]
    todo = [i for i, (src, _) in enumerate(UNITS) if (force and (var[i] or not variant)) or _stale(objs[i], includes(src))]

    def compile_one(i: int) -> None:
        src, defs = UNITS[i]
        cmd = [hipcc(), *FLAGS, *(extra if var[i] else ()), *defs, "-c", "-o", objs[i] + ".tmp", src]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(objs[i] + ".tmp", objs[i])

    jobs = max(1, min(len(UNITS), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1)))
    # the largest units first (smcrt.hip and the transport instantiations)
    todo.sort(key=lambda i: (UNITS[i][0] != KINST, not UNITS[i][0].endswith("smcrt.hip")))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, todo))
    cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp", *objs, "-lz", "-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    return _compile_and_link(LIB, force=force, verbose=verbose)


def build_variant(name: str, flags: str, outdir: str = os.path.join(ROOT, "tools", "diag_libs"),
                  verbose: bool = False) -> str:
    """A compile-time variant of the library (extra -D flags) as outdir/libsmcrt_<name>.so, for
    A/B and diagnostic runs; its objects are cached under .objs/ with the variant's name."""
    os.makedirs(outdir, exist_ok=True)
    # (always recompiled: the same name may carry other flags than last time)
    return _compile_and_link(os.path.join(outdir, f"libsmcrt_{name}.so"), tuple(flags.split()), variant=name,
                             force=True, verbose=verbose)


if __name__ == "__main__":
    # python -m rsmcrt_amd.build [--force] | --variant NAME "FLAGS" [NAME2 "FLAGS2" ...]
    if "--variant" in sys.argv:
        a = sys.argv[sys.argv.index("--variant") + 1:]
        for k in range(0, len(a) - 1, 2):
            print(build_variant(a[k], a[k + 1], verbose=True))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
