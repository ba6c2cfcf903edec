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
    """Sum tally buffers over ranks in place (RCCL over xGMI on GPUs, gloo on CPU)."""
    for t in tensors:
        dist.all_reduce(t, group=group)
