"""Gennert-Negahdaripour baseline on the GPU (classical.py:25-130 semantics)."""
import ctypes

import numpy as np

from ._lib import check, dptr, f64, lib

GN_RTOL = 1e-10      # PCG relative residual; matches SuperLU's spsolve to ~1e-8
GN_MAXITER = 200000


def apply(f1, f2, w, h, alpha, lam, x):
    n = w * h
    a, b, xx = f64(f1, n, "f1"), f64(f2, n, "f2"), f64(x, 3 * n, "x")
    y = np.empty(3 * n)
    check(lib().foto_gn_apply(dptr(a), dptr(b), w, h, float(alpha), float(lam), dptr(xx), dptr(y)))
    return y


def rhs(f1, f2, w, h):
    n = w * h
    a, b = f64(f1, n, "f1"), f64(f2, n, "f2")
    out = np.empty(3 * n)
    check(lib().foto_gn_rhs(dptr(a), dptr(b), w, h, dptr(out)))
    return out


def solve(f1, f2, w, h, alpha, lam, rtol=GN_RTOL, maxiter=GN_MAXITER):
    """Returns (u, v, m, info, iterations)."""
    n = w * h
    a, b = f64(f1, n, "f1"), f64(f2, n, "f2")
    u, v, m = np.empty(n), np.empty(n), np.empty(n)
    its = ctypes.c_int(0)
    info = check(lib().foto_gn_solve(dptr(a), dptr(b), w, h, float(alpha), float(lam), float(rtol), int(maxiter),
                                     dptr(u), dptr(v), dptr(m), ctypes.byref(its)))
    return u, v, m, info, its.value
