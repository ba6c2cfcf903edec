"""Photon sharding across ranks.

The reference splits `do j = 1, nphotons` statically over OpenMP threads
(kernelsMod.f90:1859) and would reduce the tallies to rank 0 with MPI
(kernelsMod.f90:2353-2357). Here every rank runs disjoint photon-index ranges and, since a
photon's random stream is keyed by its global index, the union over ranks is exactly the
single-GPU job. The only exchange is one sum of the tally buffers at the end.
"""
from __future__ import annotations


def first_photon(step: int, rank: int, world: int, batch: int, base: int = 0) -> int:
    """First global photon index of (step, rank): steps interleave ranks, [.., +batch)."""
    return base + (step * world + rank) * batch


def reduce_tallies(tensors, dist, group=None) -> None:
    """Sum tally buffers over ranks in place with ONE collective: the tensors are packed into
    one fp64 buffer (integer counters travel as doubles, exact below 2^53), all-reduced, and
    copied back. On GPUs the engine's own smcrt_reduce_device_tallies does the same inside
    libsmcrt over RCCL; this torch form serves gloo (CPU) process groups."""
    import torch
    flat = [t.reshape(-1) for t in tensors]
    buf = torch.cat([f.to(torch.float64) for f in flat])
    dist.all_reduce(buf, group=group)
    at = 0
    for f in flat:
        n = f.numel()
        f.copy_(buf[at:at + n].to(f.dtype))
        at += n
