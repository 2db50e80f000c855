"""Debug helper: mode-3 CG after maxiter steps vs the oracle on a small grid (GPU)."""
import os
import sys
sys.path[:0] = ['/root/repo', '/root/repo/optical-flow-optimal-transport_amd']
import numpy as np
from foto import ops
from foto.synthetic import translating_gaussian
from oracle import foto_oracle as O

Nt, Nx, Ny = 8, 24, 20
rho0, rhoT = translating_gaussian(Nx, Ny)
N, nxy = Nt * Nx * Ny, Nx * Ny
mu = np.zeros(3 * N)
for n in range(Nt):
    mu[n * nxy:(n + 1) * nxy] = (1 - n / (Nt - 1)) * rho0 + (n / (Nt - 1)) * rhoT
F = O.bb_rhs(mu, np.zeros(3 * N), rho0, rhoT, 1.0, Nt, Ny, Nx)
for mi in (1, 2, 3, 5, 10, 1000):
    xo, io, ko = O.cg(O.assemble_A(1.0, 1e-2, Nt, Ny, Nx).dot, F, maxiter=mi)
    x, info, k = ops.cg(F, Nt, Nx, Ny, 1.0, 1e-2, maxiter=mi, mode=3)
    print(os.environ.get("FOTO_GQ_EXACT"), "maxiter", mi, "k", k, ko, "err", np.abs(x - xo).max() / np.abs(xo).max(), flush=True)
