"""CPU: the lone frame's mixed deal of phase-A units (pathchain.hip rank_units / mix_sample) deals every
sample of the launch exactly once.  A sample dealt twice would still give the reference's image (the same
chain, recorded twice), so the GPU parity tests cannot see it; this restates the device index arithmetic
(the kUidMix codes, the group table ugrp, the 64-sample wave chunks) and checks the permutation for
random cost classes, every group size and the grid / rounds limits.
"""
from __future__ import annotations

import random

import pytest

K_UID_MIX = 0x80000000
K_MIX_ROUNDS = 12          # pathchain.hip kMixRounds


def rank_units(classes: list[int], mix_cls: int, grid: int) -> tuple[list[int], list[int], int, int]:
    """pathchain.hip rank_units: heaviest class first (each class in unit order here), then the mixed deal."""
    units = len(classes)
    order = sorted(range(units), key=lambda u: (classes[u], u))
    nhot = sum(1 for c in classes if c < (mix_cls & 0xff))
    lg = (mix_cls >> 8) & 3
    if lg == 0:
        lg = 3
        while lg > 1 and (nhot << lg) > grid:
            lg -= 1
    nhot = min(nhot, grid >> lg)
    if nhot == 0 or (nhot << lg) > units or units > K_MIX_ROUNDS * grid:
        lg, nhot = 0, 0
    g1 = (1 << lg) - 1
    nlight = nhot * g1
    uorder = [-1] * units
    ugrp = [-1] * units
    for pos, u in enumerate(order):
        if pos < nhot:
            ugrp[pos << lg] = u
        elif pos >= units - nlight:
            q = units - 1 - pos
            g = q // g1
            ugrp[(g << lg) + 1 + (q - g * g1)] = u
        else:
            uorder[pos + nlight] = u
    for v in range(nhot << lg):
        uorder[v] = K_UID_MIX | lg << 28 | (v & ((1 << lg) - 1)) << 24 | v >> lg
    return uorder, ugrp, nhot, lg


def mix_sample(ugrp: list[int], code: int, o: int) -> int:
    """pathchain.hip mix_sample (a ranked frame: the group table)."""
    lg, sub, g = (code >> 28) & 3, (code >> 24) & 7, code & 0xFFFFFF
    h = 64 >> lg
    vv = (sub << 8) | o
    w, l = vv >> 6, vv & 63
    c = w * (64 - h) + (l - h)
    slot = 0 if l < h else 1 + (c >> 8)
    off = w * h + l if l < h else c & 255
    return ugrp[(g << lg) + slot] * 256 + off


def dealt(uorder: list[int], ugrp: list[int]) -> list[int]:
    out = []
    for code in uorder:
        for o in range(256):
            out.append(mix_sample(ugrp, code, o) if code & K_UID_MIX else code * 256 + o)
    return out


@pytest.mark.parametrize("units,grid", [(8100, 1280), (4096, 1280), (1000, 1280), (32400, 1280), (17, 4)])
@pytest.mark.parametrize("mix_cls", [0, 5, 5 | 1 << 8, 5 | 2 << 8, 6 | 3 << 8, 1 | 3 << 8])
def test_mixed_deal_is_a_permutation(units, grid, mix_cls):
    rng = random.Random(units * 31 + mix_cls)
    classes = [rng.choice([0, 1, 2, 3, 4, 4, 5, 5, 5]) if rng.random() < 0.1 else 6 for _ in range(units)]
    uorder, ugrp, nhot, lg = rank_units(classes, mix_cls, grid)
    if units > K_MIX_ROUNDS * grid:            # beyond kMixRounds units per workgroup: heaviest first only
        assert nhot == 0 and sorted(uorder) == list(range(units))
        return
    assert sorted(dealt(uorder, ugrp)) == list(range(units * 256))


def test_hot_rows_per_wave_chunk():
    """Each 64-sample wave chunk of a group holds 64 / G samples of the hot unit: whole 8-pixel rows."""
    units, grid = 8100, 1280
    classes = [0 if u % 97 == 0 else 6 for u in range(units)]
    uorder, ugrp, nhot, lg = rank_units(classes, 5 | 1 << 8, grid)
    assert nhot > 0 and lg == 1
    hot = set(ugrp[g << lg] for g in range(nhot))
    for vu in range(nhot << lg):
        samples = [mix_sample(ugrp, uorder[vu], o) for o in range(256)]
        for w in range(4):
            chunk = samples[64 * w:64 * (w + 1)]
            hs = [s for s in chunk if s // 256 in hot]
            assert len(hs) == 32
            assert all(s % 8 == 0 for s in hs[::8]) and len({s // 8 for s in hs}) == 4   # 4 rows of 8
