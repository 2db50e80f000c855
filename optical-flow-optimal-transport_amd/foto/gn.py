"""Gennert-Negahdaripour baseline on the GPU (classical.py:25-130 semantics)."""
import collections
import os
import ctypes
import sys

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


def _outputs(n):
    """u, v, m as three views of one array: at 640x480 one 7.4 MB allocation, which numpy backs
    with transparent huge pages (it advises them from 4 MB), so copying the solution out faults
    in a few 2 MB pages instead of ~1800 4 KB ones (0.4-0.9 ms of a 4.4 ms solve, FOTO_GN_TRACE)."""
    out = np.empty(3 * n)
    return out[:n], out[n:2 * n], out[2 * n:]


def solve(f1, f2, w, h, alpha, lam, rtol=GN_RTOL, maxiter=GN_MAXITER):
    """Returns (u, v, m, info, iterations)."""
    n = w * h
    a, b = f64(f1, n, "f1"), f64(f2, n, "f2")
    u, v, m = _outputs(n)
    its = ctypes.c_int(0)
    info = check(lib().foto_gn_solve(dptr(a), dptr(b), w, h, float(alpha), float(lam), float(rtol), int(maxiter),
                                     dptr(u), dptr(v), dptr(m), ctypes.byref(its)))
    return u, v, m, info, its.value


def solve_ex(f1, f2, w, h, alpha, lam, rtol=GN_RTOL, maxiter=GN_MAXITER):
    """foto_gn_solve_ex (include/foto.h): solve() with the per-solve report -- returns
    (u, v, m, stats) with stats = {iterations, info, plan_reused, levels, ms_setup, ms_pcg,
    ms_total, alg_bytes_per_iter}."""
    from ._lib import GNStats
    n = w * h
    a, b = f64(f1, n, "f1"), f64(f2, n, "f2")
    u, v, m = _outputs(n)
    st = GNStats()
    check(lib().foto_gn_solve_ex(dptr(a), dptr(b), w, h, float(alpha), float(lam), float(rtol), int(maxiter),
                                 dptr(u), dptr(v), dptr(m), ctypes.byref(st)))
    return u, v, m, {f: getattr(st, f) for f, _ in GNStats._fields_}


class Plan:
    """A reusable GN solver for one (w, h, alpha, lambda): classical.GLLOpticalFlow after
    setAlpha/setLambda (classical.py:25-66).  Buffers, the multigrid hierarchy and the replayed
    PCG graph are made once; solve(f1, f2) is one process() (classical.py:68-130)."""

    def __init__(self, w, h, alpha, lam, rtol=GN_RTOL, maxiter=GN_MAXITER):
        self.w, self.h, self.alpha, self.lam = int(w), int(h), float(alpha), float(lam)
        self._p = ctypes.c_void_p()
        check(lib().foto_gn_plan_create(self.w, self.h, self.alpha, self.lam, float(rtol), int(maxiter),
                                        ctypes.byref(self._p)))

    def solve(self, f1, f2):
        """Returns (u, v, m, info, iterations), like solve()."""
        n = self.w * self.h
        a, b = f64(f1, n, "f1"), f64(f2, n, "f2")
        u, v, m = _outputs(n)
        its = ctypes.c_int(0)
        info = check(lib().foto_gn_plan_solve(self._p, dptr(a), dptr(b), dptr(u), dptr(v), dptr(m),
                                              ctypes.byref(its)))
        return u, v, m, info, its.value

    def timing(self):
        """{ms_setup, ms_pcg, iterations, launched} of the last solve (device events)."""
        out = np.zeros(4)
        check(lib().foto_gn_plan_timing(self._p, dptr(out)))
        return {"ms_setup": float(out[0]), "ms_pcg": float(out[1]), "iterations": int(out[2]),
                "launched": int(out[3])}

    def close(self):
        if self._p:
            lib().foto_gn_plan_destroy(self._p)
            self._p = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        # at interpreter shutdown the HIP runtime may already be torn down: leave the plan
        # to process exit (foto_capi.cpp's cached plan does the same)
        if sys.is_finalizing():
            return
        try:
            self.close()
        except Exception:
            pass


PLAN_CACHE_SIZE = 4
_plans = collections.OrderedDict()


def cached_plan(w, h, alpha, lam, rtol=GN_RTOL, maxiter=GN_MAXITER):
    """A process-wide Plan for (w, h, alpha, lambda, rtol, maxiter), shared by every
    GLLOpticalFlow instance (least recently used of PLAN_CACHE_SIZE dropped): a batch of frames
    of one size -- run.sh's per-sequence GN runs -- makes its buffers, multigrid hierarchy and
    graph once, and instances that come and go do not each hold device memory."""
    key = (int(w), int(h), float(alpha), float(lam), float(rtol), int(maxiter))
    env = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("FOTO_GN")))   # read at plan build
    p = _plans.pop(key + (env,), None)
    if p is None:
        p = Plan(*key)
        while len(_plans) >= PLAN_CACHE_SIZE:
            _plans.popitem(last=False)[1].close()
    _plans[key + (env,)] = p
    return p


def clear_plan_cache():
    while _plans:
        _plans.popitem()[1].close()
