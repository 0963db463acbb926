"""Row-stripe partition of a frame over ranks (host-side mirror of the kernel mapping).

The reference splits a frame over threads row-interleaved: thread i renders rows
i, i+T, i+2T, ... (raytracer.cpp:352-360).  Across GPUs the same idea is used at
stripe granularity (better locality per wave tile): output rows are cut into
stripes of `stripe_rows` rows, stripe s belongs to rank s % nranks, and each
rank packs its stripes contiguously into a slab of `slab_rows` rows (equal for
all ranks so the slabs can be gathered with one collective).  Rank 0 then
un-interleaves the gathered slabs (rt_unshuffle_stripes on device; `unshuffle`
below is the numpy equivalent used by the CPU tests).
"""
from __future__ import annotations

import numpy as np

DEFAULT_STRIPE_ROWS = 8


def slab_rows(height: int, stripe_rows: int, nranks: int) -> int:
    stripes = -(-height // stripe_rows)
    return -(-stripes // nranks) * stripe_rows


def rank_rows(height: int, stripe_rows: int, nranks: int, rank: int) -> np.ndarray:
    """Global output row for every slab row of `rank` (-1 = padding)."""
    n = slab_rows(height, stripe_rows, nranks)
    lr = np.arange(n)
    g = ((lr // stripe_rows) * nranks + rank) * stripe_rows + lr % stripe_rows
    return np.where(g < height, g, -1)


def unshuffle(slabs: np.ndarray, height: int, stripe_rows: int) -> np.ndarray:
    """slabs: (nranks, slab_rows, W, 3) -> (height, W, 3)."""
    nranks = slabs.shape[0]
    y = np.arange(height)
    stripe = y // stripe_rows
    owner = stripe % nranks
    lrow = (stripe // nranks) * stripe_rows + y % stripe_rows
    return slabs[owner, lrow]
