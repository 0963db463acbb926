"""GPU: the triangle test's Cramer quotients (rt_device.hpp cramer_div3, through rt_cramer_div).

The reference divides three determinants by detA in float (raytracer.cpp:147, 154, 161).  The
device takes one f32 reciprocal, refines it in double and rounds n * r to float, falling back to
IEEE divisions outside the range its exactness argument covers.  Every quotient must equal
numpy's float32 division (IEEE, correctly rounded) bit for bit: random operands over the whole
exponent range, quotients built within a few ulps of rounding midpoints, exactly representable
quotients, and the special cases (zeros of both signs, infinities, NaN, subnormal and huge
denominators, overflowing and underflowing quotients).  The host-side property check with a
perturbed reciprocal is tests/test_host.py::test_cramer_shared_reciprocal_is_correctly_rounded.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _rand(rng, n, emin, emax):
    m = 1.0 + rng.integers(0, 1 << 23, n) * 2.0 ** -23
    v = np.ldexp(m, rng.integers(emin, emax + 1, n)).astype(np.float32)
    return np.where(rng.integers(0, 2, n) == 1, -v, v).astype(np.float32)


def _cases(n=400_000, seed=20261017):
    rng = np.random.default_rng(seed)
    dens, nums = [], []
    # random over the exponent range
    dens.append(_rand(rng, n, -60, 60)); nums.append(_rand(rng, 3 * n, -149, 127).reshape(n, 3))
    dens.append(_rand(rng, n, -149, 127)); nums.append(_rand(rng, 3 * n, -60, 60).reshape(n, 3))
    # near rounding midpoints and exact quotients: q0 on the grid, num = RN(target * den), nudged
    for half in (True, False):
        d = _rand(rng, n, -40, 40)
        q0 = _rand(rng, 3 * n, -40, 40).reshape(n, 3).astype(np.float64)
        ulp = np.ldexp(1.0, np.frexp(q0)[1] - 24)
        tgt = q0 + np.copysign(ulp / 2, q0) if half else q0
        v = (tgt * d[:, None].astype(np.float64)).astype(np.float32)
        nudge = rng.integers(-2, 3, v.shape)
        for k in range(2):
            up, dn = nudge > k, nudge < -k
            v = np.where(up, np.nextafter(v, np.float32(np.inf)), np.where(dn, np.nextafter(v, np.float32(-np.inf)), v))
        dens.append(d); nums.append(v.astype(np.float32))
    # special values
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 2.0 ** -126, 2.0 ** -100, 2.0 ** -101,
                   2.0 ** 100, 2.0 ** 101, 3.4e38, -3.4e38, 1.0, -1.0, 3.0, 1e-30, 7e37], dtype=np.float32)
    dd, nn = np.meshgrid(sp, sp, indexing="ij")
    dens.append(dd.ravel()); nums.append(np.stack([nn.ravel(), -nn.ravel(), nn.ravel() * np.float32(3)], 1))
    return np.concatenate(dens), np.concatenate(nums).astype(np.float32)


def test_cramer_quotients_bit_exact(pkg, torch_cuda):
    den, num = _cases()
    with np.errstate(all="ignore"):
        ref = num / den[:, None]
    got = pkg.cramer_div(den, num)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
    bad = np.argwhere(~same)
    assert bad.size == 0, [(float(den[i]), float(num[i, j]), float(ref[i, j]), float(got[i, j])) for i, j in bad[:5]]
