"""Synthetic inputs for the FOTO hot path.

The reference ships no data (Middlebury is downloaded by ``run.sh:9``, which needs
network), so parity cases and the benchmark use deterministic synthetic pairs:

* ``translating_gaussian`` -- the S-metric / C1 / C4 family: an unnormalised
  Gaussian bump of width sigma = min(Nx, Ny)/8 centred at (0.45 Nx, 0.5 Ny) in
  frame 0 and at (0.55 Nx, 0.5 Ny) in frame 1.  No RNG.
* ``sinusoid_pair`` -- the GN (C3) stand-in: f1 = 0.5 + 0.4 sin(x/7) cos(y/5),
  f2 the same pattern shifted by (1.3, 0.4) pixels.
* ``textured_pair`` -- seeded random texture, low-pass filtered, shifted with a
  sub-pixel offset (a harder FOTO case for parity tests).

All return flat, row-major float64 arrays of length Nx*Ny, the layout
``utils.openGrayscaleImage`` produces (reference ``utils.py:39-42``).
"""
import numpy as np


def translating_gaussian(Nx, Ny, sigma=None, shift=0.10):
    sigma = float(min(Nx, Ny)) / 8.0 if sigma is None else float(sigma)
    x = np.arange(Nx, dtype=np.float64)[None, :]
    y = np.arange(Ny, dtype=np.float64)[:, None]
    cy = 0.5 * Ny
    c0 = (0.5 - shift / 2.0) * Nx
    c1 = (0.5 + shift / 2.0) * Nx
    f0 = np.exp(-((x - c0) ** 2 + (y - cy) ** 2) / (2.0 * sigma * sigma))
    f1 = np.exp(-((x - c1) ** 2 + (y - cy) ** 2) / (2.0 * sigma * sigma))
    return f0.ravel().copy(), f1.ravel().copy()


def sinusoid_pair(w, h, dx=1.3, dy=0.4):
    x = np.arange(w, dtype=np.float64)[None, :]
    y = np.arange(h, dtype=np.float64)[:, None]
    f1 = 0.5 + 0.4 * np.sin(x / 7.0) * np.cos(y / 5.0)
    f2 = 0.5 + 0.4 * np.sin((x - dx) / 7.0) * np.cos((y - dy) / 5.0)
    return f1.ravel().copy(), f2.ravel().copy()


def textured_pair(w, h, seed=0, dx=2.5, dy=1.0, smooth=2):
    """Random texture (box-blurred ``smooth`` times), rescaled to [0.05, 0.95] and
    moved by (dx, dy) pixels with bilinear interpolation and edge clamping."""
    rng = np.random.default_rng(seed)
    f = rng.random((h, w))
    for _ in range(smooth):
        p = np.pad(f, 1, mode="edge")
        f = (p[:-2, :-2] + p[:-2, 1:-1] + p[:-2, 2:] + p[1:-1, :-2] + p[1:-1, 1:-1]
             + p[1:-1, 2:] + p[2:, :-2] + p[2:, 1:-1] + p[2:, 2:]) / 9.0
    f = (f - f.min()) / max(f.max() - f.min(), 1e-300)
    f = 0.05 + 0.9 * f
    yy, xx = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    xs = np.clip(xx - dx, 0, w - 1)
    ys = np.clip(yy - dy, 0, h - 1)
    x0 = np.minimum(np.floor(xs).astype(np.int64), w - 2)
    y0 = np.minimum(np.floor(ys).astype(np.int64), h - 2)
    ax = xs - x0
    ay = ys - y0
    g = ((1 - ay) * (1 - ax) * f[y0, x0] + (1 - ay) * ax * f[y0, x0 + 1]
         + ay * (1 - ax) * f[y0 + 1, x0] + ay * ax * f[y0 + 1, x0 + 1])
    return f.ravel().copy(), g.ravel().copy()
