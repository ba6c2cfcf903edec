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
    """Sum tally buffers over ranks in place: the floating-point tensors are packed into one
    fp64 buffer and the integer ones (counters) into one int64 buffer, one all-reduce each,
    then copied back. Every tensor must be contiguous (it is reduced through a view). On GPUs
    the engine's own smcrt_reduce_device_tallies does the same inside libsmcrt over RCCL;
    this torch form serves gloo (CPU) process groups."""
    import torch
    for t in tensors:
        if not t.is_contiguous():
            raise ValueError("reduce_tallies needs contiguous tensors (a copy would not reach the caller)")
    for is_float, dtype in ((True, torch.float64), (False, torch.int64)):
        part = [t.view(-1) for t in tensors if t.is_floating_point() == is_float]
        if not part:
            continue
        buf = torch.cat([f.to(dtype) for f in part])
        dist.all_reduce(buf, group=group)
        at = 0
        for f in part:
            n = f.numel()
            f.copy_(buf[at:at + n].to(f.dtype))
            at += n
