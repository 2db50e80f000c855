"""Drop-in for the reference's ``utils.py``.

Hot path (GPU, libfoto.so):
  opticalflow_from_benamoubrenier  utils.py:148-183 -> foto_flow_from_phi (one thread per
                                   pixel walks the Nt-1 trajectory steps, then m = -div_D)
Evaluation (GPU):
  apply_opticalflow -> foto_warp, EE / AE -> foto_flow_errors, IE -> foto_intensity_error
Host utilities (image and .flo IO):
  openGrayscaleImage, reconstructTrajectory (single start point), openFlo, saveFlo --
  same semantics and quirks as utils.py:25-292.
"""
import os
import threading
import math  # noqa: F401  (kept for API parity with the reference module)

import numpy as np
from PIL import Image

from foto import evaluate as _ev
from foto import ops as _ops


_frames = {}   # (path, mtime_ns, size) -> (f, w, h): the last few decoded frames
_frames_lock = threading.Lock()   # run.py decodes the next sequence's frames on a pool thread


def openGrayscaleImage(inputPathname):
    """8-bit grayscale -> flat float64 in [0, 1], width, height (utils.py:25-42).  A batch
    worker opens each frame three times (diff, GN, FOTO); the last 4 decodes are kept, keyed
    by path, modification time and size, and handed out as copies."""
    try:
        st = os.stat(inputPathname)
        key = (os.path.abspath(inputPathname), st.st_mtime_ns, st.st_size)
    except (OSError, TypeError):   # file objects and the like: no caching
        key = None
    with _frames_lock:
        hit = _frames.get(key) if key else None
    if hit is None:
        f = np.asarray(Image.open(inputPathname).convert("L"))
        h, w = f.shape
        hit = (f.reshape(-1) / 255, w, h)
        if key:
            with _frames_lock:
                _frames[key] = hit
                while len(_frames) > 4:
                    del _frames[next(iter(_frames))]
    return hit[0].copy(), hit[1], hit[2]


def reconstructTrajectory(xStart, yStart, u, v, Nx, Ny, Nt):
    """One particle through the (Nt x Nx*Ny) velocity slabs u, v with clamped bilinear
    interpolation (utils.py:44-99).  Host helper for a single start point; the solver
    integrates all pixels on the GPU (opticalflow_from_benamoubrenier)."""
    x, y = xStart, yStart
    for n in range(Nt - 1):
        tx = max(0, min(Nx - 2, int(x)))
        ty = max(0, min(Ny - 2, int(y)))
        dX, dY = x - tx, y - ty
        w1, w2, w3, w4 = (1 - dY) * (1 - dX), dX * (1 - dY), dY * dX, (1 - dX) * dY
        a, b = ty * Nx + tx, (ty + 1) * Nx + tx
        x += w1 * u[n, a] + w2 * u[n, a + 1] + w3 * u[n, b + 1] + w4 * u[n, b]
        y += w1 * v[n, a] + w2 * v[n, a + 1] + w3 * v[n, b + 1] + w4 * v[n, b]
    return [x - xStart, y - yStart]


def opticalflow_from_benamoubrenier(phi, Nt, Nx, Ny, grad=None, div=None):
    """(u, v, m) from the space-time potential phi (utils.py:148-183), on the GPU.
    ``grad``/``div`` are accepted for signature parity; the kernels implement the
    reference's operators.grad(bc='N') and operators.div(bc='D')."""
    return _ops.flow_from_phi(phi, Nt, Nx, Ny)


def apply_opticalflow(f1, u, v, w, h, m=np.array([None])):
    """Backward bilinear warp of (1+m) f1 by (u, v) (utils.py:186-248) on the GPU
    (foto_warp; bit-identical to the reference).  Reference behaviour kept: with numpy 2
    ``np.array([None]).all()`` is False, so ``m.all() != None`` holds for every m and the
    reference evaluates ``(1 + m) * f1`` -- a TypeError for the default m, as here."""
    if m.all() != None:  # noqa: E711
        1 + m  # noqa: B018  -- the reference's (1 + m) * f1: raises for the default np.array([None])
        return _ev.warp(f1, u, v, w, h, m)
    return _ev.warp(f1, u, v, w, h, None)


def openFlo(pathname):
    """Middlebury .flo reader -> (w, h, u, v) (utils.py:250-271)."""
    with open(pathname, "rb") as f:
        magic = np.fromfile(f, np.float32, count=1)[0]
        if 202021.25 != magic:
            print("Magic number incorrect. Invalid .flo file")
        w = np.fromfile(f, np.int32, count=1)[0]
        h = np.fromfile(f, np.int32, count=1)[0]
        data = np.fromfile(f, np.float32)
    data = data.reshape(h, w, 2)
    return w, h, data[..., 0].flatten(), data[..., 1].flatten()


def saveFlo(w, h, u, v, pathname):
    """Middlebury .flo writer: float32 magic, int32 w, h, interleaved float32 (u, v)
    (utils.py:273-292)."""
    with open(pathname, "wb") as f:
        np.array([202021.25], dtype=np.float32).tofile(f)
        np.array([w, h], dtype=np.int32).tofile(f)
        np.stack([np.asarray(u, dtype=np.float64), np.asarray(v, dtype=np.float64)], axis=1).astype(np.float32).tofile(f)


def EE(w, h, u, v, uGT, vGT):
    """Average endpoint error and its std over pixels with EE <= 50 (utils.py:294-315), GPU."""
    return _ev.flow_errors(u, v, uGT, vGT, w, h)[0:2]


def AE(w, h, u, v, uGT, vGT):
    """Average angular error (radians) and std, NaNs ignored (utils.py:317-338), GPU."""
    return _ev.flow_errors(u, v, uGT, vGT, w, h)[2:4]


def IE(w, h, I, IGT):
    """RMS intensity error on the 0..255 scale (utils.py:340-354), GPU."""
    return _ev.intensity_error(I, IGT, w, h)
