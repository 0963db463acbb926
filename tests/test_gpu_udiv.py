"""GPU: the shadow walkers' division by a wave-uniform divisor (pathchain.hip UDiv, through rt_udiv).

occlude_queue_body divides task indices by the chunk size and owner ids by the light count with
a reciprocal held in a scalar register (the compiler's own 32-bit expansion, which otherwise left
the reciprocals in VGPRs that k_occlude spilled).  Checked bit-exact against integer floor
division over the whole 32-bit range: the extremes, multiples of each divisor and their
neighbours (every quotient boundary the corrections handle), and random values.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _values(d_list, rng):
    v = [0, 1, 2, 3, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF]
    for d in d_list:
        for m in (1, 2, 3, 1000, (0xFFFFFFFF // d) - 1, 0xFFFFFFFF // d):
            x = m * d
            v += [x - 1, x, x + 1]
    v = [x & 0xFFFFFFFF for x in v if 0 <= x]
    v = np.array(v, dtype=np.uint64)
    r = rng.integers(0, 2**32, size=200_000, dtype=np.uint64)
    small = rng.integers(0, 2**20, size=50_000, dtype=np.uint64)
    return np.concatenate([v, r, small]).astype(np.uint32)


def test_udiv_exact(pkg, torch_cuda):
    rng = np.random.default_rng(11)
    d = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 16, 31, 100, 127, 128, 255, 256, 1000, 4096, 65535, 65536,
         65537, 1 << 20, 1000003, 0x7FFFFFFF, 0x80000000, 0x80000001, 0xFFFFFFFE, 0xFFFFFFFF]
    d += [int(x) for x in rng.integers(1, 2**32, size=24, dtype=np.uint64)]
    d += [int(x) for x in rng.integers(1, 2**12, size=24, dtype=np.uint64)]
    dd = np.array(d, dtype=np.uint32)
    v = _values(d, rng)
    q = pkg.udiv(v, dd)
    ref = v[None, :].astype(np.uint64) // dd[:, None].astype(np.uint64)
    bad = np.nonzero(q.astype(np.uint64) != ref)
    assert bad[0].size == 0, [(int(dd[j]), int(v[i]), int(q[j, i]), int(ref[j, i])) for j, i in zip(*bad)][:10]


def test_udiv_errors(pkg, torch_cuda):
    with pytest.raises(Exception):
        pkg.udiv(np.array([5], np.uint32), np.array([0], np.uint32))
