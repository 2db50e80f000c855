"""Matrix-free GPU applications of the reference operators (libfoto per-op entry points).

Each function equals ``operators.<builder>(...) @ x`` of the reference (h = 1), computed
by one HIP kernel (operators.py line numbers in include/foto.h).
"""
import ctypes

import numpy as np

from ._lib import check, dptr, f64, lib


def grad_st(phi, Nt, Nx, Ny):
    N = Nt * Nx * Ny
    x = f64(phi, N, "phi")
    out = np.empty(3 * N)
    check(lib().foto_grad_st(dptr(x), Nt, Nx, Ny, dptr(out)))
    return out


def div_st(w, Nt, Nx, Ny):
    N = Nt * Nx * Ny
    x = f64(w, 3 * N, "w")
    out = np.empty(N)
    check(lib().foto_div_st(dptr(x), Nt, Nx, Ny, dptr(out)))
    return out


def laplacian_st(p, Nt, Nx, Ny):
    N = Nt * Nx * Ny
    x = f64(p, N, "p")
    out = np.empty(N)
    check(lib().foto_laplacian_st(dptr(x), Nt, Nx, Ny, dptr(out)))
    return out


def apply_A(p, Nt, Nx, Ny, r, eps):
    """(-r L_st + r eps I) @ p  (benamou_brenier.py:202-203)."""
    N = Nt * Nx * Ny
    x = f64(p, N, "p")
    out = np.empty(N)
    check(lib().foto_apply_A(dptr(x), Nt, Nx, Ny, float(r), float(eps), dptr(out)))
    return out


def grad2(f, Nx, Ny, bc="N"):
    x = f64(f, Nx * Ny, "f")
    out = np.empty(2 * Nx * Ny)
    check(lib().foto_grad2(dptr(x), Nx, Ny, _bc(bc), dptr(out)))
    return out


def div2(uv, Nx, Ny, bc="D"):
    x = f64(uv, 2 * Nx * Ny, "uv")
    out = np.empty(Nx * Ny)
    check(lib().foto_div2(dptr(x), Nx, Ny, _bc(bc), dptr(out)))
    return out


def grad2_forward(f, Nx, Ny):
    x = f64(f, Nx * Ny, "f")
    out = np.empty(2 * Nx * Ny)
    check(lib().foto_grad2_forward(dptr(x), Nx, Ny, dptr(out)))
    return out


def stepB(p, M):
    """benamou_brenier.stepB: projection onto {a + |b|^2/2 <= 0} of 3 SoA fields of length M."""
    x = f64(p, 3 * M, "p")
    out = np.empty(3 * M)
    check(lib().foto_stepB(dptr(x), ctypes.c_int64(M), dptr(out)))
    return out


def bb_rhs(mu, q, rho0, rhoT, r, Nt, Nx, Ny):
    """F = div_st(mu - r q) + temporal BC correction (benamou_brenier.py:64-82)."""
    N = Nt * Nx * Ny
    a, b = f64(mu, 3 * N, "mu"), f64(q, 3 * N, "q")
    r0, rT = f64(rho0, Nx * Ny, "rho0"), f64(rhoT, Nx * Ny, "rhoT")
    out = np.empty(N)
    check(lib().foto_bb_rhs(dptr(a), dptr(b), dptr(r0), dptr(rT), Nt, Nx, Ny, float(r), dptr(out)))
    return out


def cg(b, Nt, Nx, Ny, r, eps, rtol=1e-6, maxiter=1000, mode=0):
    """scipy cg on A = -r L_st + r eps I from x0 = 0.  Returns (x, info, iterations)."""
    N = Nt * Nx * Ny
    x_in = f64(b, N, "b")
    x = np.empty(N)
    its = ctypes.c_int(0)
    info = check(lib().foto_cg(dptr(x_in), Nt, Nx, Ny, float(r), float(eps), float(rtol), int(maxiter), int(mode),
                               dptr(x), ctypes.byref(its)))
    return x, info, its.value


def flow_from_phi(phi, Nt, Nx, Ny):
    """utils.opticalflow_from_benamoubrenier (grad bc 'N', div bc 'D')."""
    x = f64(phi, Nt * Nx * Ny, "phi")
    u, v, m = np.empty(Nx * Ny), np.empty(Nx * Ny), np.empty(Nx * Ny)
    check(lib().foto_flow_from_phi(dptr(x), Nt, Nx, Ny, dptr(u), dptr(v), dptr(m)))
    return u, v, m


def _bc(bc):
    if bc not in ("N", "D"):
        raise NotImplementedError("These boundary conditions are not implemented")
    return bc.encode()


def dct(x, axis_len, inner=1, inverse=False, path=0):
    """Orthonormal DCT-II (DCT-III if inverse) along the middle axis of a C-order
    [outer][axis_len][inner] array on the GPU (foto_dct; path 0 auto, 1 FFT, 2 GEMM)."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64)).reshape(-1)
    outer = a.size // (axis_len * inner)
    assert outer * axis_len * inner == a.size
    out = np.empty_like(a)
    check(lib().foto_dct(dptr(a), outer, axis_len, inner, int(bool(inverse)), int(path), dptr(out)))
    return out
