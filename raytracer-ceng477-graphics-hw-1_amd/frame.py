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


def assemble_frames(slabs, height: int, stripe_rows: int,
                    unshuffle: Optional[Callable] = None, gbuf=None, images=None, dst: int = 0):
    """A frame batch (rt_render_frames_device): every rank's (F, slab_rows, W, 3)
    slabs -> F frames on dst, with ONE gather for the whole batch (bigger xGMI
    messages than F gathers).  images: F (H, W, 3) device outputs for
    `unshuffle`.  Returns the list of frames on dst, None elsewhere."""
    import torch

    g = gather_slabs(slabs, gbuf, dst)            # (nranks, F, slab_rows, W, 3)
    if g is None:
        return None
    per = g.transpose(0, 1).contiguous()          # (F, nranks, slab_rows, W, 3): frame-major
    out = []
    for f in range(per.shape[0]):
        if unshuffle is not None:
            unshuffle(per[f], images[f])
            out.append(images[f])
        else:
            out.append(torch.from_numpy(stripes.unshuffle(per[f].cpu().numpy(), height, stripe_rows)))
    return out


# ---------------------------------------------------------------------------
# Multi-camera batching across GPUs (raytracer.cpp:505-519
# renders the scene's cameras one after another): camera i is rendered by rank
# i mod N (each rank batches its cameras, rt_render_cameras_device), and rank 0
# receives every image with ONE gather of fixed-size packed buffers.
# ---------------------------------------------------------------------------
def camera_ranks(ncams: int, nranks: int) -> list[int]:
    """Owner rank of each camera (round-robin, like the stripes)."""
    return [i % nranks for i in range(ncams)]


def _packed_bytes(sizes, nranks: int) -> int:
    own = camera_ranks(len(sizes), nranks)
    per = [0] * nranks
    for i, (h, w) in enumerate(sizes):
        per[own[i]] += h * w * 3
    return max(per + [1])


def gather_camera_images(local: dict, sizes: list, dst: int = 0, device=None):
    """local: {camera index: (H, W, 3) uint8 tensor} rendered by this rank (its
    cameras per camera_ranks); sizes: [(H, W)] of every camera.  Returns the
    list of all images (index order) on dst, None elsewhere.  One collective."""
    import torch
    import torch.distributed as dist

    dist_on = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    world = dist.get_world_size() if dist_on else 1
    rank = dist.get_rank() if dist_on else 0
    own = camera_ranks(len(sizes), world)
    cap = _packed_bytes(sizes, world)
    dev = device if device is not None else (next(iter(local.values())).device if local else "cpu")
    buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
    off = 0
    for i, (h, w) in enumerate(sizes):
        if own[i] == rank:
            n = h * w * 3
            buf[off:off + n].copy_(local[i].reshape(-1))
            off += n
    if not dist_on:
        allb = [buf]
    else:
        allb = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
        dist.gather(buf, gather_list=allb, dst=dst)
        if rank != dst:
            return None
    out, offs = [], [0] * world
    for i, (h, w) in enumerate(sizes):
        r, n = own[i], h * w * 3
        out.append(allb[r][offs[r]:offs[r] + n].reshape(h, w, 3))
        offs[r] += n
    return out
