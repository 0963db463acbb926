"""Multi-GPU frame assembly: one process per GPU, one collective.

The reference renders one frame with T threads, thread i taking rows i, i+T, ...
(raytracer.cpp:352-360).  Across GPUs the frame is split the same way at stripe
granularity (stripes.py): every rank renders its round-robin row stripes into a
contiguous slab in its own HBM, with no exchange during the render (the scene
is replicated, read-only).  The only data-path collective is the final gather
of the slabs to rank 0 (torch.distributed over RCCL / xGMI on MI355X, gloo on
CPU in the tests), followed by one rank-0 pass that restores row order.

These helpers take torch tensors and an `unshuffle` callable so that the same
code drives the device path (bench.py: RCCL + rt_unshuffle_stripes kernel) and
the CPU tests (gloo + numpy).
"""
from __future__ import annotations

from typing import Callable, Optional

from . import stripes


def slab_shape(width: int, height: int, stripe_rows: int, nranks: int) -> tuple[int, int, int]:
    return (stripes.slab_rows(height, stripe_rows, nranks), width, 3)


def gather_slabs(slab, gbuf=None, dst: int = 0):
    """Gather every rank's (slab_rows, W, 3) uint8 slab into dst's gbuf
    (nranks, slab_rows, W, 3).  One collective; a no-op for a single rank.
    Returns gbuf on dst (allocated if None), None elsewhere."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        if gbuf is None:
            gbuf = slab.unsqueeze(0).clone()
        else:
            gbuf[0].copy_(slab)
        return gbuf
    world, rank = dist.get_world_size(), dist.get_rank()
    if rank == dst and gbuf is None:
        gbuf = torch.empty((world,) + tuple(slab.shape), dtype=slab.dtype, device=slab.device)
    dist.gather(slab, gather_list=[gbuf[i] for i in range(world)] if rank == dst else None, dst=dst)
    return gbuf if rank == dst else None


def assemble_frame(slab, height: int, stripe_rows: int,
                   unshuffle: Optional[Callable] = None, gbuf=None, image=None, dst: int = 0):
    """Gather + un-interleave.  `unshuffle(gbuf, image)` writes row order into
    image (device kernel); default: the numpy restatement (stripes.unshuffle).
    Returns the (height, W, 3) frame on dst, None elsewhere."""
    g = gather_slabs(slab, gbuf, dst)
    if g is None:
        return None
    if unshuffle is not None:
        unshuffle(g, image)
        return image
    import torch

    out = stripes.unshuffle(g.cpu().numpy(), height, stripe_rows)
    return torch.from_numpy(out)
