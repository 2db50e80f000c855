"""GN multigrid prototype (numpy/scipy, CPU): the PCG iteration count of the GPU's V-cycle
preconditioner (foto_gn.hip) against variants of it, before any kernel work.

The restatement: levels halve (rounding up) down to <= 1024 cells; level operator
s_l (-Lambda) + B_l per field with s_l = (alpha, alpha, lambda) / 4^l and B_l the pointwise
3 x 3 coupling v v^T (v = (fx, fy, -f2)) averaged over children with the prolongation weights;
bilinear prolongation P (3/4, 1/4 per axis, clamped), restriction P^T / 4; damped (0.8)
block-Jacobi sweeps, the first from zero; 12 sweeps on the coarsest level; CG to rtol 1e-10.
With nu = 1 it reproduces the GPU's counts (34 at 640x480 on the sinusoid pair).  Variants:
nu pre- and post-sweeps on level 0 only (nu0) or on every level (nu).

    python tools/gn_mg_proto.py [w h ...]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "optical-flow-optimal-transport_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from foto.synthetic import sinusoid_pair  # noqa: E402
from oracle import foto_oracle as O  # noqa: E402

OMEGA = 0.8
COARSE = 1024
CSWEEPS = 12


def p1d(nf, nc):
    rows, cols, vals = [], [], []
    for i in range(nf):
        i0 = i >> 1
        i1 = i0 + 1 if (i & 1) else i0 - 1
        i1 = min(max(i1, 0), nc - 1)
        rows += [i, i]
        cols += [i0, i1]
        vals += [0.75, 0.25]
    return sp.csr_matrix((vals, (rows, cols)), shape=(nf, nc))   # duplicates add (clamped: 1.0)


def lap(w, h):
    def l1(n):
        e = np.ones(n)
        m = sp.diags([-e[:-1], 2 * e, -e[:-1]], [-1, 0, 1]).tolil()
        m[0, 0] = 1
        m[n - 1, n - 1] = 1
        return m.tocsr()
    return (sp.kron(sp.identity(h), l1(w)) + sp.kron(l1(h), sp.identity(w))).tocsr()


class Level:
    def __init__(self, w, h, s, B):
        self.w, self.h, self.n = w, h, w * h
        self.s = s
        self.B = B                      # (6, n): xx xy xm yy ym mm
        self.L = lap(w, h)
        c = np.asarray(self.L.diagonal())
        M = np.zeros((self.n, 3, 3))
        b = B
        M[:, 0, 0] = s[0] * c + b[0]; M[:, 0, 1] = b[1]; M[:, 0, 2] = b[2]
        M[:, 1, 0] = b[1]; M[:, 1, 1] = s[1] * c + b[3]; M[:, 1, 2] = b[4]
        M[:, 2, 0] = b[2]; M[:, 2, 1] = b[4]; M[:, 2, 2] = s[2] * c + b[5]
        self.Dinv = np.linalg.inv(M)

    def apply(self, x):
        n, b = self.n, self.B
        u, v, m = x[:n], x[n:2 * n], x[2 * n:]
        yu = self.s[0] * (self.L @ u) + b[0] * u + b[1] * v + b[2] * m
        yv = self.s[1] * (self.L @ v) + b[1] * u + b[3] * v + b[4] * m
        ym = self.s[2] * (self.L @ m) + b[2] * u + b[4] * v + b[5] * m
        return np.concatenate([yu, yv, ym])

    def dinv(self, r):
        n = self.n
        R = np.stack([r[:n], r[n:2 * n], r[2 * n:]], axis=1)
        Z = np.einsum("nij,nj->ni", self.Dinv, R)
        return np.concatenate([Z[:, 0], Z[:, 1], Z[:, 2]])


def hierarchy(fx, fy, f2, w, h, alpha, lam):
    v = np.stack([fx, fy, -f2])
    B = np.stack([v[0] * v[0], v[0] * v[1], v[0] * v[2], v[1] * v[1], v[1] * v[2], v[2] * v[2]])
    levs = [Level(w, h, np.array([alpha, alpha, lam]), B)]
    Ps = []
    while w * h > COARSE:
        wc, hc = (w + 1) // 2, (h + 1) // 2
        P = sp.kron(p1d(h, hc), p1d(w, wc)).tocsr()
        wsum = np.asarray(P.sum(axis=0)).ravel()
        Bc = np.stack([(P.T @ B[k]) / wsum for k in range(6)])
        w, h, B = wc, hc, Bc
        levs.append(Level(w, h, levs[-1].s / 4.0, B))
        Ps.append(P)
    return levs, Ps


def vcycle(levs, Ps, l, f, nu):
    L = levs[l]
    if l == len(levs) - 1:
        z = OMEGA * L.dinv(f)
        for _ in range(CSWEEPS - 1):
            z = z + OMEGA * L.dinv(f - L.apply(z))
        return z
    z = OMEGA * L.dinv(f)
    for _ in range(nu[l] - 1):
        z = z + OMEGA * L.dinv(f - L.apply(z))
    r = f - L.apply(z)
    P = Ps[l]
    n, nc = L.n, levs[l + 1].n
    fc = np.concatenate([(P.T @ r[k * n:(k + 1) * n]) / 4.0 for k in range(3)])
    ec = vcycle(levs, Ps, l + 1, fc, nu)
    z = z + np.concatenate([P @ ec[k * nc:(k + 1) * nc] for k in range(3)])
    for _ in range(nu[l]):
        z = z + OMEGA * L.dinv(f - L.apply(z))
    return z


def pcg(A, b, M, rtol=1e-10, maxiter=500):
    x = np.zeros_like(b)
    r = b.copy()
    z = M(r)
    p = z.copy()
    rz = r @ z
    bn = np.sqrt(b @ b)
    for k in range(maxiter):
        if np.sqrt(r @ r) < rtol * bn:
            return x, k
        q = A(p)
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        z = M(r)
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return x, maxiter


def main():
    a = [int(v) for v in sys.argv[1:]]
    sizes = list(zip(a[::2], a[1::2])) or [(160, 120), (320, 240), (640, 480)]
    alpha, lam = 0.1, 0.2
    for w, h in sizes:
        f1, f2 = sinusoid_pair(w, h)
        fx, fy, ft = O.gn_coeffs(f1, f2, w, h)
        f2 = np.asarray(f2, dtype=np.float64)
        b = np.concatenate([-fx * ft, -fy * ft, f2 * ft])
        levs, Ps = hierarchy(fx, fy, f2, w, h, alpha, lam)
        nl = len(levs)
        A = levs[0].apply
        line = f"{w}x{h} ({nl} levels):"
        for name, nu in (("nu 1", [1] * nl), ("nu0 2", [2] + [1] * (nl - 1)), ("nu 2", [2] * nl),
                         ("nu0 3", [3] + [1] * (nl - 1))):
            _, its = pcg(A, b, lambda r: vcycle(levs, Ps, 0, r, nu))
            line += f"  {name}: {its}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
