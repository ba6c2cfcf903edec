"""rsmcrt_amd — MI355X-native photon-packet Monte Carlo engine for signedMCRT's hot path.

The compute path is the HIP library rsmcrt_amd/libsmcrt.so (C ABI: include/smcrt.h).
Importing this package does not load it; `rsmcrt_amd.engine` does, and fails loudly if it
is missing or no GPU is present.
"""
import os

# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (default 4), read once
# when the HIP runtime starts. A scene uses up to four launch streams, its own stream and a
# fold stream, and torch has its own: with four queues, overlapped launches that share a queue
# run one after the other (a kernel trace shows two launch streams on one queue). Eight
# measured +16-19 % on the tail-bound scenes (M5, profiles/r03_s3/hwq_ab.txt and
# profiles/r04_s3/hwq_ab.txt) and no change on M1. The GPU boxes export the HIP default (4)
# explicitly, so a value below 8 is raised to 8 (a caller's setting of 8 or more wins); it only
# takes effect if nothing has started the HIP runtime yet (C/Fortran callers export it
# themselves).
MIN_HW_QUEUES = 8
MAX_HW_QUEUES = 32  # the GPU pool refuses more; HIP itself allows no more than the hardware has


def _raise_hw_queues(env=os.environ, want=MIN_HW_QUEUES, log=None):
    """Set GPU_MAX_HW_QUEUES to at least `want` and at most MAX_HW_QUEUES. A value that does not
    parse counts as unset; an explicit value that is changed is reported through `log` (stderr
    by default). Returns the value left in env."""
    raw = env.get("GPU_MAX_HW_QUEUES")
    try:
        cur = int(raw) if raw not in (None, "") else 0
    except ValueError:
        cur = 0
    new = min(max(cur, want), MAX_HW_QUEUES)
    if raw is not None and raw != "" and str(new) != raw.strip():
        msg = f"[rsmcrt_amd] GPU_MAX_HW_QUEUES={raw!r} -> {new} (at least {want}, at most {MAX_HW_QUEUES})"
        if log is None:
            import sys
            print(msg, file=sys.stderr)
        else:
            log(msg)
    env["GPU_MAX_HW_QUEUES"] = str(new)
    return new


_raise_hw_queues()

from . import abi, builders, scene  # noqa: E402,F401

__all__ = ["abi", "builders", "scene"]
