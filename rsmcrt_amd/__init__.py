"""rsmcrt_amd — MI355X-native photon-packet Monte Carlo engine for signedMCRT's hot path.

The compute path is the HIP library rsmcrt_amd/libsmcrt.so (C ABI: include/smcrt.h).
Importing this package does not load it; `rsmcrt_amd.engine` does, and fails loudly if it
is missing or no GPU is present.
"""
from . import abi, builders, scene  # noqa: F401

__all__ = ["abi", "builders", "scene"]
