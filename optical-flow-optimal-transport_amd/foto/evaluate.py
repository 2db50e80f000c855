"""GPU evaluation helpers: the backward warp and the flow / intensity
error metrics of the reference's utils.py, through libfoto's C ABI.

warp            utils.apply_opticalflow (utils.py:186-248)  bit-identical
flow_errors     utils.EE + utils.AE     (utils.py:294-338)  up to summation order
intensity_error utils.IE                (utils.py:340-354)  up to summation order
"""
import numpy as np

from ._lib import check, dptr, f64, lib


def warp(f1, u, v, w, h, m=None):
    """(1 + m) f1 (or f1 if m is None) warped backwards by (u, v)."""
    n = w * h
    f = f64(f1, n, "f1")
    uu, vv = f64(u, n, "u"), f64(v, n, "v")
    mm = None if m is None else f64(np.broadcast_to(np.asarray(m, dtype=np.float64), (n,)), n, "m")
    out = np.empty(n)
    check(lib().foto_warp(dptr(f), dptr(uu), dptr(vv), dptr(mm) if mm is not None else None, w, h, dptr(out)))
    return out


def flow_errors(u, v, uGT, vGT, w, h):
    """(AEE, SDEE, AAE, SDAE): endpoint error <= 50 and non-NaN angular error (radians)."""
    n = w * h
    a = [f64(np.asarray(x, dtype=np.float64)[:n], n, name) for x, name in ((u, "u"), (v, "v"), (uGT, "uGT"), (vGT, "vGT"))]
    out = np.empty(4)
    check(lib().foto_flow_errors(*(dptr(x) for x in a), w, h, dptr(out)))
    return tuple(float(x) for x in out)


def intensity_error(I, IGT, w, h):
    """RMS of 255 I - 255 IGT."""
    n = w * h
    a, b = f64(I, n, "I"), f64(IGT, n, "IGT")
    out = np.empty(1)
    check(lib().foto_intensity_error(dptr(a), dptr(b), w, h, dptr(out)))
    return float(out[0])
