"""theta-binned Gauss compression with a local variable linear in lam~ (not in theta).

The GPU's k_gq_hist needs one acos per voxel to place it in a theta bin and to get its
theta-linear local variable u.  With u linear in lam~ inside the same theta bins, the bin of a
voxel follows from comparisons against the bin edges cos(pi b / B) (incremental along a row,
whose eigenvalues increase with kx), and u from one subtract and one multiply.  This script
checks on the numpy restatement that the compressed CG keeps its residual norms, iteration
counts and solution as close to the literal diagonal CG as the theta-linear variant does.

usage: python tools/gauss_lin_proto.py Nx Ny Nt eps [outer_iterations]
"""
import sys
sys.path.insert(0, '/root/repo/tools'); sys.path.insert(0, '/root/repo')
sys.path.insert(0, '/root/repo/optical-flow-optimal-transport_amd')
import numpy as np
from scipy import fft
import gautschi_proto as G
from oracle import foto_oracle as O
from foto.synthetic import translating_gaussian

B, M = 256, 8


def edges(B):
    hi = np.cos(np.pi * np.arange(B + 1) / B)   # hi[b] = upper lam~ edge of bin b (decreasing)
    mid = 0.5 * (hi[:-1] + hi[1:])
    hw = 0.5 * (hi[:-1] - hi[1:])
    return hi, mid, hw


def bin_lin(lt, B):
    hi, mid, hw = edges(B)
    # bin b: hi[b+1] < lt <= hi[b]  (searchsorted on the increasing reversed edges)
    b = B - 1 - np.searchsorted(hi[::-1], lt, side='left') + 1
    b = np.clip(b, 0, B - 1)
    # fix-up so that hi[b+1] < lt <= hi[b] except at the clamped ends
    u = (lt - mid[b]) / hw[b]
    return b, u


def gauss_rule(mu, m):
    nu = mu.copy()
    for k in range(1, len(nu)): nu[k] = mu[k] / 2.0 ** (k - 1)
    if nu[0] <= 0: return np.zeros(0), np.zeros(0)
    al, be = G.mod_chebyshev(nu, m)
    n = m
    for k in range(1, m):
        if not (be[k] > 1e-13): n = k; break
    J = np.diag(al[:n]) + np.diag(np.sqrt(be[1:n]), 1) + np.diag(np.sqrt(be[1:n]), -1)
    x, V = np.linalg.eigh(J)
    return x, be[0] * V[0, :] ** 2


def compress(lam, w, c0, c1, lin):
    lt = np.clip((lam - c0) / c1, -1, 1)
    if lin:
        b, u = bin_lin(lt, B)
    else:
        th = np.arccos(lt); h = np.pi / (2 * B)
        b = np.minimum((th / (2 * h)).astype(np.int64), B - 1); u = (th - (2 * b + 1) * h) / h
    mom = np.zeros((B, 2 * M))
    t0 = np.ones_like(u); t1 = u.copy()
    mom[:, 0] = np.bincount(b, w, B); mom[:, 1] = np.bincount(b, w * t1, B)
    for j in range(2, 2 * M):
        t0, t1 = t1, 2 * u * t1 - t0
        mom[:, j] = np.bincount(b, w * t1, B)
    hi, mid, hw = edges(B)
    nodes, wts = [], []
    for k in range(B):
        if mom[k, 0] <= 0: continue
        x, ww = gauss_rule(mom[k], M)
        if lin:
            lk = mid[k] + hw[k] * x
        else:
            h = np.pi / (2 * B); lk = np.cos((2 * k + 1) * h + x * h)
        nodes.append(c0 + c1 * lk); wts.append(ww)
    return np.concatenate(nodes), np.concatenate(wts)


def cg_coeffs(nodes, wts, rtol, maxiter=2000):
    r = np.ones_like(nodes); p = None
    bn2 = wts.sum(); al = []; be = []; rho_prev = None; rn = []
    for k in range(maxiter):
        rho = (wts * r * r).sum(); rn.append(np.sqrt(rho))
        if np.sqrt(rho) < rtol * np.sqrt(bn2): return np.array(al), np.array(be), k, np.array(rn)
        if k == 0: p = r.copy(); be.append(0.0)
        else: b_ = rho / rho_prev; p = r + b_ * p; be.append(b_)
        q = nodes * p; a = rho / (wts * p * q).sum(); al.append(a)
        r = r - a * q; rho_prev = rho
    return np.array(al), np.array(be), maxiter, np.array(rn)


def q_eval(lam, al, be):
    x = np.zeros_like(lam); r = np.ones_like(lam); p = np.zeros_like(lam)
    for k in range(len(al)):
        p = r + be[k] * p; x = x + al[k] * p; r = r - al[k] * lam * p
    return x


def q_table(lam, al, be, c0, c1, n, lin):
    lt = np.clip((lam - c0) / c1, -1, 1)
    hi, mid, hw = edges(B)
    j = np.arange(n); un = np.cos(np.pi * (j + 0.5) / n)
    if lin:
        b, u = bin_lin(lt, B)
        ln = (mid[:, None] + hw[:, None] * un[None, :])
    else:
        th = np.arccos(lt); h = np.pi / (2 * B)
        b = np.minimum((th / (2 * h)).astype(np.int64), B - 1); u = (th - (2 * b + 1) * h) / h
        ln = np.cos((2 * np.arange(B)[:, None] + 1) * h + un[None, :] * h)
    vals = q_eval(c0 + c1 * ln.ravel(), al, be).reshape(B, n)
    T = np.cos(np.outer(np.arange(n), np.pi * (j + 0.5) / n))
    coef = (2.0 / n) * vals @ T.T; coef[:, 0] *= 0.5
    c = coef[b]; b1 = np.zeros_like(u); b2 = np.zeros_like(u)
    for k in range(n - 1, 0, -1):
        b1, b2 = c[:, k] + 2 * u * b1 - b2, b1
    return c[:, 0] + u * b1 - b2


def main():
    Nx, Ny, Nt = (int(a) for a in sys.argv[1:4]); eps = float(sys.argv[4]); r = 1.0
    nouter = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    rho0, rhoT = translating_gaussian(Nx, Ny)
    N, nxy = Nt * Nx * Ny, Nx * Ny
    lam = (r * eps + r * (G.eig1d(Nt)[:, None, None] + G.eig1d(Ny)[None, :, None] + G.eig1d(Nx)[None, None, :])).ravel()
    lmin, lmax = r * eps, r * eps + r * (G.eig1d(Nt)[-1] + G.eig1d(Ny)[-1] + G.eig1d(Nx)[-1])
    c0, c1 = 0.5 * (lmax + lmin), 0.5 * (lmax - lmin)
    A = O.assemble_A(r, eps, Nt, Ny, Nx)
    mu = np.zeros(3 * N); q = np.zeros(3 * N)
    for n in range(Nt): mu[n * nxy:(n + 1) * nxy] = (1 - n / (Nt - 1)) * rho0 + (n / (Nt - 1)) * rhoT
    for it in range(nouter):
        F = O.bb_rhs(mu, q, rho0, rhoT, r, Nt, Ny, Nx)
        phi, info, kref = O.cg(A.dot, F)
        bh = fft.dctn(F.reshape(Nt, Ny, Nx), type=2, norm='ortho').ravel()
        _, _, kd, rnd = cg_coeffs(lam, bh * bh, 1e-6)
        line = f"outer {it}: scipy {kref} diag {kd}"
        for lin in (False, True):
            nodes, wts = compress(lam, bh * bh, c0, c1, lin)
            al, be, kc, rnc = cg_coeffs(nodes, wts, 1e-6)
            mm = min(len(rnd), len(rnc))
            rel = np.abs(rnc[:mm] - rnd[:mm]) / rnd[:mm]
            qn = 24
            xt = q_table(lam, al, be, c0, c1, qn, lin) * bh
            pt = fft.idctn(xt.reshape(Nt, Ny, Nx), type=2, norm='ortho').ravel()
            line += (f" | {'lin' if lin else 'theta'}: K {kc} rn rel max {rel.max():.2e}"
                     f" phi {np.abs(pt - phi).max() / np.abs(phi).max():.2e}")
        print(line, flush=True)
        g = O.grad_st(phi, Nt, Ny, Nx); q = O.stepB(g + (1.0 / r) * mu, N); mu = mu + r * (g - q); mu[:N] = np.maximum(mu[:N], 0)


if __name__ == "__main__":
    main()
