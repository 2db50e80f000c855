"""The spectral s-step CG planning rule, restated in numpy, against the reference's goldens.

csrc/foto_spectral.hip runs scipy's CG recurrence (benamou_brenier.py:85 ->
scipy.sparse.linalg.cg) in the DCT eigenbasis, where A = C^T diag(lam) C and every CG
update is pointwise.  One pass applies up to SMAX = 8 iterations whose scalars were planned
from Chebyshev moments of the pass-start state (r_k, p_{k-1}) over an interval adapted to
the residual measure ([lmin, mean + 2 sd]: of b^ of the previous solve for the INIT moments,
the whole spectrum for a run's first solve; of the new residual, projected through the Gram,
after short passes; of the pass-start state otherwise); step i > 0 is taken only
while its two Gram-form inner products have cancellation ratio sum|terms| / |value| <=
S_CLIM = 3e4, and the moments are summed with compensated block reductions (correctly
rounded to ~1 ulp).  This module restates that rule on the CPU (test infrastructure: the
oracle provides the rhs, the goldens the reference's answers) and checks that it keeps
scipy's CG iteration counts and the reference's crit / iterate to the stated bars.  The
GPU kernels are checked against the same goldens in test_gpu_parity.py.
"""
import math
import os
import sys

import numpy as np
import pytest
import scipy.fft as sfft

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import foto_oracle as O  # noqa: E402

SMAX = 8
NMOM = 2 * SMAX
NCO = SMAX + 1
S_CLIM = 3e4
S_KAPPA = 2.0
S_PROJ = (NMOM - 3) // 2   # projected interval after n <= S_PROJ steps


def _lam(Nt, Ny, Nx, r, eps):
    mu = lambda n: 2 - 2 * np.cos(np.pi * np.arange(n) / n)  # noqa: E731
    return (r * eps + r * (mu(Nt)[:, None, None] + mu(Ny)[None, :, None] + mu(Nx)[None, None, :])).ravel()


def _moments(T, w):
    # correctly rounded sums (the GPU's compensated block reductions; math.fsum is exact)
    return np.array([math.fsum(T[m] * w) for m in range(NMOM)])


def _plan(Mrr, Mrq, Mqq, k, rho_prev, atol, c0, c1, maxiter):
    """Next pass's (alphas, betas, converged) from the moments of (r_k, p_{k-1})."""
    fam = (Mrr, Mrq, Mqq)
    H = np.zeros((2 * NCO, 2 * NCO))
    for a in range(2 * NCO):
        for c in range(2 * NCO):
            ia, ic = a % NCO, c % NCO
            if ia + ic < NMOM:
                M = fam[a // NCO + c // NCO]
                H[a, c] = 0.5 * (M[ia + ic] + M[abs(ia - ic)])

    def ip(U, V):
        t = U[:, None] * H * V[None, :]
        s = t.sum()
        return s, (np.abs(t).sum() / abs(s) if s != 0 else np.inf)

    def mul_lam(U):
        Y = np.zeros_like(U)
        for pb in (0, NCO):
            c = U[pb:pb + NCO]
            X = np.zeros(NCO)
            X[1] += c[0]
            for m in range(1, NCO - 1):
                X[m + 1] += 0.5 * c[m]
                X[m - 1] += 0.5 * c[m]
            Y[pb:pb + NCO] = c0 * c + c1 * X
        return Y

    R = np.zeros(2 * NCO); R[0] = 1.0
    P = np.zeros(2 * NCO); P[NCO] = 1.0
    al, be = [], []
    for i in range(SMAX):
        if k + i >= maxiter:
            break
        if i == 0:
            rho = Mrr[0]
        else:
            rho, cr = ip(R, R)
            if not cr <= S_CLIM:
                break
        if rho == 0 or math.sqrt(rho) < atol:
            return al, be, True, rho_prev, None
        beta = 0.0 if k + i == 0 else rho / rho_prev
        Pn = R.copy() if k + i == 0 else beta * P + R
        Q = mul_lam(Pn)
        den, cr = ip(Pn, Q)
        if i > 0 and not cr <= S_CLIM:
            break
        alpha = rho / den
        R = R - alpha * Q
        P = Pn
        rho_prev = rho
        al.append(alpha)
        be.append(beta)
    proj = None
    if 0 < len(al) <= S_PROJ:   # mean / variance of the new residual's measure from the Gram
        LR = mul_lam(R)
        rr_, _ = ip(R, R)
        if rr_ > 0:
            mean = ip(R, LR)[0] / rr_
            proj = (mean, ip(LR, LR)[0] / rr_ - mean * mean)
    return al, be, False, rho_prev, proj


def _interval(mean, var, c0, c1, lmin, lmax):
    """Chebyshev interval [lmin, min(lmax, mean + S_KAPPA sd)] (csrc/foto_spectral.hip)."""
    hi = max(min(lmax, mean + S_KAPPA * math.sqrt(max(var, 0.0))), lmin + 1e-3 * (lmax - lmin))
    return (0.5 * (hi + lmin), 0.5 * (hi - lmin)) if hi == hi else (c0, c1)


def _moment_stats(Mrr, c0, c1):
    """Mean and variance of the measure the rr moments describe (None if empty)."""
    if not Mrr[0] > 0:
        return None
    ex, ex2 = Mrr[1] / Mrr[0], 0.5 * (Mrr[2] + Mrr[0]) / Mrr[0]
    return c0 + c1 * ex, c1 * c1 * (ex2 - ex * ex)


def sstep_cg(b, Nt, Ny, Nx, r, eps, rtol=1e-6, maxiter=1000, stats=None, carry=None):
    """x, info, iterations -- scipy's contract (x0 = 0, M = I).  carry: dict kept across the
    solves of one Benamou-Brenier run (the INIT interval comes from the previous solve's b^)."""
    lam = _lam(Nt, Ny, Nx, r, eps)
    lmin, lmax = lam.min(), lam.max()   # r eps, r eps + r (mu_t + mu_y + mu_x)_max
    c0, c1 = 0.5 * (lmax + lmin), 0.5 * (lmax - lmin)   # the first solve's INIT: the whole spectrum
    if carry is not None and "init" in carry:
        c0, c1 = carry["init"]
    first = True
    bh = sfft.dctn(b.reshape(Nt, Ny, Nx), norm="ortho").ravel()
    rr, q = bh.copy(), np.zeros_like(bh)
    atol = max(0.0, rtol * math.sqrt(math.fsum(bh * bh)))
    k, rho_prev, passes, conv = 0, 0.0, 0, False
    while k < maxiter:
        x = (lam - c0) / c1
        T = np.empty((NMOM, lam.size))
        T[0] = 1.0
        T[1] = x
        for m in range(2, NMOM):
            T[m] = 2 * x * T[m - 1] - T[m - 2]
        Mrr, Mrq, Mqq = _moments(T, rr * rr), _moments(T, rr * q), _moments(T, q * q)
        al, be, conv, rho_prev, proj = _plan(Mrr, Mrq, Mqq, k, rho_prev, atol, c0, c1, maxiter)
        passes += 1
        ms = _moment_stats(Mrr, c0, c1)
        if first and carry is not None and ms is not None:
            carry["init"] = _interval(*ms, c0, c1, lmin, lmax)
        first = False
        if proj is not None:
            c0, c1 = _interval(*proj, c0, c1, lmin, lmax)
        elif ms is not None:
            c0, c1 = _interval(*ms, c0, c1, lmin, lmax)
        for a, bt in zip(al, be):
            p = rr.copy() if k == 0 else bt * q + rr
            rr = rr - a * (lam * p)
            q = p
            k += 1
        if conv or not al:
            break
    if stats is not None:
        stats.setdefault("passes", []).append(passes)
    xh = (bh - rr) / lam
    return sfft.idctn(xh.reshape(Nt, Ny, Nx), norm="ortho").ravel(), (0 if conv else maxiter), k


def test_sstep_plan_cg_cases(gold):
    d = gold("cg.npz")
    for c in range(3):
        Nt, Ny, Nx = (int(s) for s in d[f"c{c}_shape"])
        r, eps = d[f"c{c}_r_eps"]
        x, info, its = sstep_cg(d[f"c{c}_b"], Nt, Ny, Nx, r, eps)
        assert info == 0 and abs(its - int(d[f"c{c}_its"])) <= 1
        ref = d[f"c{c}_x"]
        np.testing.assert_allclose(x, ref, rtol=0, atol=5e-8 * np.abs(ref).max())


@pytest.mark.parametrize("name", ["bb_small.npz", "bb_tex.npz"])
def test_sstep_plan_golden_solves(gold, name, monkeypatch):
    """Whole Benamou-Brenier solves with the planned CG: same outer iterations and CG
    counts (+-1) as the reference, crit within 1e-7 relative, and fewer passes than
    iterations / 3 (the point of the rule)."""
    d = gold(name)
    Nt, Ny, Nx = (int(s) for s in d["shape"])
    r, tol, eps, max_it = d["params"]
    stats = {}
    carry = {}
    monkeypatch.setattr(O, "cg", lambda mv, b, rtol=1e-6, maxiter=1000: sstep_cg(b, Nt, Ny, Nx, r, eps, rtol, maxiter, stats,
                                                                                 carry))
    st = {}
    u, v, m = O.solve(d["rho0"], d["rhoT"], Nt, Nx, Ny, r, tol, eps, int(max_it), log=lambda *a: None, stats=st)
    assert len(st["crit"]) == len(d["crit"])
    assert np.max(np.abs(st["cg_its"] - d["cg_its"])) <= 1
    np.testing.assert_allclose(st["crit"], d["crit"], rtol=1e-7, atol=0)
    for a, b in ((u, d["u"]), (v, d["v"])):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-7)
    assert np.mean(stats["passes"]) < np.mean(st["cg_its"]) / 3
