"""Drop-in for the reference's ``benamou_brenier.py`` -- the FOTO solver on an MI355X.

``solve`` keeps the signature, defaults, stdout and return value of the reference
(benamou_brenier.py:151-271); the whole outer loop (RHS, Poisson CG, projection, multiplier
update, criterion) and the flow extraction run in libfoto.so (HIP, gfx950).  The Poisson CG
is selected by ``cg_mode`` (env FOTO_CG_MODE): 3 = CG on the Gauss-compressed spectral
measure of the right-hand side (csrc/foto_gauss.inc), 2 = s-step CG in the DCT-II eigenbasis
of A, 1 = one-pass CG in that basis, 0 = 7-point stencil CG, -1 = auto (default: 0 on grids of
at most 2^18 voxels -- config 1 and the golden grids, where it rounds like the reference's
matvec -- and 3 above).  All follow scipy's CG recurrence and stopping rule.  Modes 0, 2 and 3 run time-sharded over GPUs; mode 1 is
single-GPU only (include/foto.h).
"""
import os

import numpy as np

from foto import bb as _bb
from foto import ops as _ops


def _default_mode():
    return int(os.environ.get("FOTO_CG_MODE", "-1"))


def solve_benamou_brenier_step(mu, q, rho0, rhoT, r, A, div, Nt, Nx, Ny, dt, dx, dy):
    """stepA (benamou_brenier.py:26-91): F = div(mu - r q) + temporal BC correction, then
    phi = cg(A, F, rtol=1e-6, maxiter=1000).  ``A`` must be the reference's
    -r*laplacian_st + r*eps*I and ``div`` its div_st (h = 1): eps is read off A's diagonal
    and the operators are applied matrix-free on the GPU."""
    if (dt, dx, dy) != (1, 1, 1):
        raise NotImplementedError("the GPU path implements the reference's dt = dx = dy = 1")
    N = Nt * Nx * Ny
    if A.shape != (N, N):
        raise NotImplementedError(f"A has shape {A.shape}, expected ({N}, {N})")
    d0 = float(A.diagonal()[0])          # corner voxel: r * (3 + eps)
    eps = d0 / r - 3.0
    # A must be exactly the operator the GPU applies: compare on random vectors (any other
    # matrix -- a different stencil, a changed entry anywhere -- fails with probability 1) and
    # the stored entries against the 7-point pattern (every voxel: itself + its neighbours)
    rng = np.random.default_rng(12345)
    for _ in range(2):
        x = rng.standard_normal(N)
        if not np.allclose(A @ x, _ops.apply_A(x, Nt, Nx, Ny, r, eps), rtol=1e-12, atol=1e-12 * abs(r)):
            raise NotImplementedError("A is not -r*laplacian_st + r*eps*I on this grid")
    edges = (Nt - 1) * Nx * Ny + Nt * (Nx - 1) * Ny + Nt * Nx * (Ny - 1)
    if hasattr(A, "count_nonzero") and A.count_nonzero() > N + 2 * edges:
        raise NotImplementedError("A has entries outside the 7-point space-time stencil")
    F = _ops.bb_rhs(mu, q, rho0, rhoT, r, Nt, Nx, Ny)
    u, info, _ = _ops.cg(F, Nt, Nx, Ny, r, eps, rtol=1e-6, maxiter=1000, mode=_default_mode())
    if info > 0:
        print(f"WARNING: CG did not converge in {info} iterations.")
    elif info < 0:
        raise RuntimeError("CG solver failed due to illegal input or breakdown.")
    return u


def stepB(p, Nt, Nx, Ny):
    """Pointwise projection of (alpha, beta1, beta2) onto {a + |b|^2/2 <= 0}
    (benamou_brenier.py:93-149), one HIP thread per voxel."""
    return _ops.stepB(p, Nt * Nx * Ny)


def solve(rho0, rhoT, Nt, Nx, Ny, r=1, convergence_tol=0.3, reg_epsilon=1e-3, max_it=100, **opts):
    """Benamou-Brenier optical flow: returns (u, v, m) as the reference does.
    Extra keyword options go to foto.bb.BBSolver (device, cg_mode, ...)."""
    opts.setdefault("cg_mode", _default_mode())
    return _bb.solve(rho0, rhoT, Nt, Nx, Ny, r=r, convergence_tol=convergence_tol, reg_epsilon=reg_epsilon,
                     max_it=max_it, **opts)
