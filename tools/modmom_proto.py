"""Feasibility check (numpy, CPU): can the node CG's alpha_k, beta_k come from the modified
Chebyshev algorithm instead of a block reduction per step?

The serial chain of the default Poisson solve is scipy's CG recurrence on the spectral measure
sigma = sum b^_i^2 delta(lam_i): ~180 steps, each a block reduction on one CU.
The modified Chebyshev algorithm (Gautschi) gets the Jacobi matrix of sigma from 2n modified
moments nu_l = int pi_l dsigma against a known auxiliary family pi_l -- every step a local
update over l plus a broadcast, no reduction -- and CG's alpha, beta follow from the Jacobi matrix
by its LU recurrence.  It is well conditioned only when the pi_l are nearly orthogonal for sigma.
Candidate auxiliaries here: the previous outer iteration's orthogonal polynomials (the measure
moves little from one outer iteration to the next late in a solve), and the Chebyshev
polynomials of the spectrum's interval (known to fail).

For each outer iteration of a moderate grid (the oracle's loop) this prints how far the
algorithm's alpha, beta drift from the reference CG (long double on the full measure), and
whether the stop index K matches.

    python tools/modmom_proto.py [Nx Ny Nt] [outer iterations]
"""
import os
import sys

import numpy as np
import scipy.fft

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "optical-flow-optimal-transport_amd"))
from oracle import foto_oracle as O  # noqa: E402
from foto.synthetic import translating_gaussian  # noqa: E402

LD = np.longdouble


def spectrum(Nt, Ny, Nx, r, eps):
    mu = lambda n: 2.0 - 2.0 * np.cos(np.pi * np.arange(n) / n)  # noqa: E731
    return r * (eps + mu(Nt)[:, None, None] + mu(Ny)[None, :, None] + mu(Nx)[None, None, :])


def cg_coeffs(lam, w, rtol, kmax, dtype):
    """scipy's CG on diag(lam) with b = sqrt(w) (node form): alpha_k, beta_k (beta_0 = 0), K."""
    lam = lam.astype(dtype)
    r = np.sqrt(w.astype(dtype))
    p = np.zeros_like(r)
    bn2 = (r * r).sum()
    atol2 = (dtype(rtol) * np.sqrt(bn2)) ** 2
    al, be, rho_prev = [], [], None
    rho = bn2
    for k in range(kmax):
        rho = (r * r).sum()
        if rho < atol2:
            return np.array(al, dtype=dtype), np.array(be, dtype=dtype), k, rho
        beta = dtype(0) if k == 0 else rho / rho_prev
        p = r + beta * p
        ap = lam * p
        alpha = rho / (p * ap).sum()
        r = r - alpha * ap
        al.append(alpha)
        be.append(beta)
        rho_prev = rho
    return np.array(al, dtype=dtype), np.array(be, dtype=dtype), kmax, rho


def stieltjes(lam, w, n, dtype=LD):
    """Monic recurrence coefficients (a_k, b_k), k < n, of sum w_i delta(lam_i): the discretized
    Stieltjes procedure in long double (b_0 = total mass)."""
    lam = lam.astype(dtype)
    w = w.astype(dtype)
    a = np.zeros(n, dtype=dtype)
    b = np.zeros(n, dtype=dtype)
    p_prev = np.zeros_like(lam)
    p = np.ones_like(lam)
    nrm_prev = None
    for k in range(n):
        nrm = (w * p * p).sum()
        a[k] = (w * lam * p * p).sum() / nrm
        b[k] = nrm if k == 0 else nrm / nrm_prev
        p_next = (lam - a[k]) * p - (b[k] * p_prev if k > 0 else 0)
        p_prev, p, nrm_prev = p, p_next, nrm
    return a, b


def modified_moments(lam, w, ahat, bhat, L):
    """nu_l = sum w_i pi_l(lam_i), l < L, pi_{l+1} = (t - ahat_l) pi_l - bhat_l pi_{l-1}."""
    pm = np.zeros_like(lam)
    p = np.ones_like(lam)
    nu = np.zeros(L)
    for l in range(L):
        nu[l] = (w * p).sum()
        pn = (lam - ahat[l]) * p - (bhat[l] * pm if l > 0 else 0.0)
        pm, p = p, pn
    return nu


def mod_chebyshev(nu, ahat, bhat, n):
    """Gautschi's modified Chebyshev algorithm: (a_k, b_k), k < n, from nu_0 .. nu_{2n-1}."""
    L = 2 * n
    a = np.zeros(n)
    b = np.zeros(n)
    sig_m = np.zeros(L + 1)              # sigma_{k-2, l}
    sig = np.zeros(L + 1)
    sig[:L] = nu                          # sigma_{0, l}
    a[0] = ahat[0] + nu[1] / nu[0]
    b[0] = nu[0]
    sig_prev = np.zeros(L + 1)            # sigma_{-1, l} = 0
    for k in range(1, n):
        new = np.zeros(L + 1)
        for l in range(k, L - k):
            new[l] = (sig[l + 1] - (a[k - 1] - ahat[l]) * sig[l] - b[k - 1] * sig_prev[l]
                      + (bhat[l] * sig[l - 1] if l >= 1 else 0.0))
        a[k] = ahat[k] + new[k + 1] / new[k] - sig[k] / sig[k - 1]
        b[k] = new[k] / sig[k - 1]
        sig_prev, sig = sig, new
    return a, b


def jacobi_to_cg(a, b, rho0):
    """CG's alpha_k, beta_k (beta_0 = 0) from the monic recurrence of the measure (x0 = 0):
    1/alpha_k = a_k - beta_k / alpha_{k-1}, beta_{k+1} = b_{k+1} alpha_k^2 ... via the LU of J."""
    n = len(a)
    al = np.zeros(n)
    be = np.zeros(n)
    for k in range(n):
        if k == 0:
            al[k] = 1.0 / a[0]
        else:
            be[k] = b[k] * al[k - 1] ** 2 / 1.0   # beta_k = b_k alpha_{k-1}^2 (monic b_k)
            be[k] = b[k] * al[k - 1] * al[k - 1]
            al[k] = 1.0 / (a[k] - be[k] / al[k - 1])
    return al, be


def main():
    a = sys.argv[1:]
    Nx, Ny, Nt = (int(v) for v in a[:3]) if len(a) >= 3 else (96, 80, 16)
    iters = int(a[3]) if len(a) >= 4 else 6
    r, eps = 1.0, 1e-2
    rho0, rhoT = translating_gaussian(Nx, Ny)
    N = Nt * Nx * Ny
    A = O.assemble_A(r, eps, Nt, Ny, Nx)
    lam = spectrum(Nt, Ny, Nx, r, eps).ravel()
    mu = np.zeros(3 * N)
    for n in range(Nt):
        mu[n * Nx * Ny:(n + 1) * Nx * Ny] = (1 - n / (Nt - 1)) * rho0 + (n / (Nt - 1)) * rhoT
    q = np.zeros(3 * N)
    prev = None
    lo, hi = lam.min(), lam.max()
    for it in range(iters):
        F = O.bb_rhs(mu, q, rho0, rhoT, r, Nt, Ny, Nx)
        bh = scipy.fft.dctn(F.reshape(Nt, Ny, Nx), type=2, norm="ortho").ravel()
        w = bh * bh
        alr, ber, K, _ = cg_coeffs(lam, w, 1e-6, 1000, LD)
        al64, be64, K64, _ = cg_coeffs(lam, w, 1e-6, 1000, np.float64)
        d64 = max(np.max(np.abs((al64[:min(K, K64)] - alr[:min(K, K64)]) / alr[:min(K, K64)])), 0)
        line = f"outer {it}: K {K} (float64 {K64}, alpha rel {float(d64):.1e})"
        n = K + 4
        variants = [("cheb", None), ("prev", prev)]
        if prev is not None:
            # what a GPU run has: the previous solve's own n_prev = K_prev + 4 coefficients, then a
            # continuation -- (a) the last coefficient pair repeated, (b) the spectrum's Chebyshev
            # asymptotics (centre, h^2 / 4)
            ap_, bp_ = prev
            npv = prev_k + 4
            c, h = (lo + hi) / 2, (hi - lo) / 2
            a1, b1 = ap_.copy(), bp_.copy()
            a1[npv:], b1[npv:] = ap_[npv - 1], bp_[npv - 1]
            a2, b2 = ap_.copy(), bp_.copy()
            a2[npv:], b2[npv:] = c, h * h / 4
            variants += [("prev+last", (a1, b1)), ("prev+cheb", (a2, b2))]
        for name, aux in variants:
            if name == "prev" and aux is None:
                continue
            if name == "cheb":   # monic Chebyshev of the first kind on [lo, hi]
                c, h = (lo + hi) / 2, (hi - lo) / 2
                ahat = np.full(2 * n + 2, c)
                bhat = np.full(2 * n + 2, h * h / 4)
                bhat[1] = h * h / 2
            else:
                ahat, bhat = aux
            nu = modified_moments(lam, w, ahat, bhat, 2 * n)
            am, bm = mod_chebyshev(nu, ahat, bhat, n)
            alm, bem = jacobi_to_cg(am, bm, w.sum())
            kk = min(K, n)
            err = np.abs((alm[:kk] - alr[:kk].astype(float)) / alr[:kk].astype(float))
            bad = np.argmax(err > 1e-10) if np.any(err > 1e-10) else kk
            line += f" | {name}: alpha rel max {np.nanmax(err):.1e}, first step > 1e-10: {bad}"
        print(line, flush=True)
        # the auxiliary family for the next outer iteration: this measure's orthogonal polynomials
        ap, bp = stieltjes(lam, w, 2 * (K + 40) + 2)
        prev = (ap.astype(float), bp.astype(float))
        prev_k = K
        # the outer iteration (oracle): CG solve, stepB, stepC
        phi, _, _ = O.cg(A.dot, F, rtol=1e-6, maxiter=1000)
        g = O.grad_st(phi, Nt, Ny, Nx)
        q = O.stepB(g + (1.0 / r) * mu, N)
        mu = mu + r * (g - q)
        mu[:N] = np.maximum(mu[:N], 0)


if __name__ == "__main__":
    main()
