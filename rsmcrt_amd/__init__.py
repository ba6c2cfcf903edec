"""rsmcrt_amd — MI355X-native photon-packet Monte Carlo engine for signedMCRT's hot path.

The compute path is the HIP library rsmcrt_amd/libsmcrt.so (C ABI: include/smcrt.h).
Importing this package does not load it; `rsmcrt_amd.engine` does, and fails loudly if it
is missing or no GPU is present.
"""
import os

# HIP maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues (default 4), read once
# when the HIP runtime starts. A scene uses up to four launch streams, its own stream and a
# fold stream, and torch has its own: with four queues, overlapped launches that share a queue
# run one after the other. Eight measured +16-19 % on the tail-bound scenes (M4, M5) and no
# change on M1 (profiles/r03_s3/hwq_ab.txt). setdefault: a caller's own setting wins, and it
# only takes effect if nothing has started the HIP runtime yet (C/Fortran callers export it
# themselves).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

from . import abi, builders, scene  # noqa: E402,F401

__all__ = ["abi", "builders", "scene"]
