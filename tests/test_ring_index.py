"""Flat ring tiles (csrc/foto_spectral.hip ring_divmod, ring_ok): the per-lane row / plane
index of an element comes from an fp32 reciprocal estimate with one correction each way.
Restated in numpy (float32 products and truncation as on the GPU) and checked against exact
integer division over the range ring_ok admits (element index < 2^30, quotient < 2^21)."""
import numpy as np


def ring_divmod(e, n):
    inv = np.float32(1.0) / np.float32(n)
    q = (e.astype(np.float32) * inv).astype(np.int64)
    r = e - q * n
    q = np.where(r < 0, q - 1, np.where(r >= n, q + 1, q))
    return q, e - q * n


def test_ring_divmod_exact():
    rng = np.random.default_rng(0)
    for n in list(range(2, 2400, 38)) + [64, 146, 194, 380, 388, 420, 480, 584, 640, 1024, 2302]:
        top = min((1 << 30) - 1, n * (1 << 21) - 1)
        k = np.arange(1, 3000, dtype=np.int64)
        e = np.concatenate([rng.integers(0, top, 20000), k * n - 1, k * n, top - k])
        e = e[(e >= 0) & (e <= top)]
        q, r = ring_divmod(e, n)
        assert np.array_equal(q, e // n) and np.array_equal(r, e % n), n


def test_flat_tile_pairs_stay_in_a_row():
    # a lane's two elements (e, e + 1), e even, share a row whenever Nx is even
    for nx in (146, 420, 584, 64):
        e = np.arange(0, 40 * nx, 2)
        q0, _ = ring_divmod(e, nx)
        q1, _ = ring_divmod(e + 1, nx)
        assert np.array_equal(q0, q1)
