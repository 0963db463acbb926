"""GPU: the specular power term (raytracer.cpp:414, `pow(max(0, n.h), phong)`,
the C library's double pow converted to float) as the shading kernels evaluate
it (phong_pow.hpp: integer fast path + double-double fallback), against
glibc's pow on this host (Python's math.pow), bit for bit.

Cases: the exponents {3, 50, 100, 2.5} and others over random bases, bases
whose power is exactly a float rounding midpoint (the fallback's hardest
inputs: odd mantissas m with m^p of 25 significant bits, perfect squares for
p = 2.5 / 0.5), and the C library's special cases.  The host restatement of
the same code is checked against glibc on ~2 M more cases by
tests/test_host.py::test_phong_pow_matches_glibc_pow.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cases() -> tuple[np.ndarray, np.ndarray]:
    rng = np.random.default_rng(414)
    bs, ps = [], []
    for p in [1, 2, 3, 5, 10, 50, 64, 100, 128, 4096, 4097, 2.5, 0.5, 1.5, 7.25, 33.3, 0.1, -2, -2.5, 2.0 ** 25]:
        b = np.concatenate([rng.random(20000), rng.random(5000) * 4.0, 1.0 + (rng.random(5000) - 0.5) * 2.0 ** -10])
        bs.append(b.astype(np.float32))
        ps.append(np.full(b.size, p, np.float32))
    for p, lo, hi in [(2, 4097, 5792), (3, 257, 322), (5, 29, 31)]:       # exact float midpoints
        m = np.arange(lo | 1, hi + 1, 2, dtype=np.float64)
        for e in range(-20, 9):
            bs.append((m * 2.0 ** (e - 12)).astype(np.float32))
            ps.append(np.full(m.size, p, np.float32))
    m = np.arange(1, 4098, 2, dtype=np.float64)
    for e in range(-6, 4):                                                 # perfect squares: exact roots
        for p in (2.5, 0.5, 1.5):
            bs.append((m * m * 2.0 ** (2 * e)).astype(np.float32))
            ps.append(np.full(m.size, p, np.float32))
    sp = np.array([0.0, -0.0, 1.0, -1.0, 2.0, -2.0, 0.5, -0.5, np.inf, -np.inf, np.nan, 2.0 ** -149, 3.0],
                  np.float32)
    bs.append(np.repeat(sp, sp.size))
    ps.append(np.tile(sp, sp.size))
    return np.concatenate(bs), np.concatenate(ps)


def _glibc(b: np.ndarray, p: np.ndarray) -> np.ndarray:
    """(float)pow((double)b, (double)p) with the C library's pow (numpy's float64
    power calls libm's pow), spot-checked against math.pow on regular inputs."""
    with np.errstate(all="ignore"):
        out = np.power(b.astype(np.float64), p.astype(np.float64)).astype(np.float32)
    for i in range(0, b.size, 997):
        x, y = float(b[i]), float(p[i])
        if x > 0 and math.isfinite(x) and math.isfinite(y):
            try:
                with np.errstate(over="ignore"):
                    v = np.float32(math.pow(x, y))
            except OverflowError:
                v = np.float32(np.inf)
            assert v.view(np.uint32) == out[i].view(np.uint32), (x, y)
    return out


def test_device_phong_pow_matches_glibc(pkg):
    b, p = _cases()
    got = pkg.phong_pow(b, p)
    want = _glibc(b, p)
    both_nan = np.isnan(got) & np.isnan(want)
    bad = ~both_nan & (got.view(np.uint32) != want.view(np.uint32))
    idx = np.flatnonzero(bad)[:10]
    assert not bad.any(), [(float(b[i]).hex(), float(p[i]), float(got[i]).hex(), float(want[i]).hex()) for i in idx]
    assert b.size > 500_000
