"""Build the HIP engine library in-tree: rsmcrt_amd/libsmcrt.so (gfx950).

Plain hipcc, no torch extension machinery: every source compiles to an object in parallel and
one link makes the C-ABI shared object (include/smcrt.h) that Fortran/C/Python can bind.
Objects are kept in rsmcrt_amd/.objs/ (git-ignored) and rebuilt only when their source or a
header it includes (found by scanning `#include "..."` lines) is newer.
"""
from __future__ import annotations

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
OBJDIR = os.path.join(PKG, ".objs")
SOURCES = [os.path.join(PKG, "csrc", f) for f in ("smcrt.hip", "writers.cpp", "frontend.cpp", "sources.cpp", "png.cpp", "escape.cpp", "inverse.cpp", "multi.hip", "cull.cpp")]
DEPS = SOURCES + sorted(glob.glob(os.path.join(PKG, "csrc", "*.h"))) + [os.path.join(ROOT, "include", "smcrt.h")]
ARCH = os.environ.get("SMCRT_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: no fused multiply-add, so fp64 trajectories are bit-identical to the
# CPU restatement (oracle/), which is compiled the same way.
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         f"--offload-arch={ARCH}", "-Wall"]
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


def _obj(src: str, extra_flags=()) -> str:
    tag = "" if not extra_flags else "." + str(abs(hash(tuple(extra_flags))) % 10**8)
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


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    os.makedirs(OBJDIR, exist_ok=True)
    objs = [_obj(src) for src in SOURCES]
    todo = [i for i, src in enumerate(SOURCES) if force or _stale(objs[i], includes(src))]

    def compile_one(i: int) -> None:
        cmd = [hipcc(), *FLAGS, "-c", "-o", objs[i] + ".tmp", SOURCES[i]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(objs[i] + ".tmp", objs[i])

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, todo))
    cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", LIB + ".tmp", *objs, "-lz", "-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
