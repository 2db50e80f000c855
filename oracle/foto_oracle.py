"""CPU oracle for the FOTO hot path -- TEST INFRASTRUCTURE ONLY.

This module is a clean numpy/scipy restatement of the reference algorithm
(thomasjacumin/optical-flow-optimal-transport, mounted read-only at
/root/reference in the build container).  It is the CHECKER: only tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import it.
The product path (optical-flow-optimal-transport_amd/, libfoto.so) never
imports, links or calls anything here.

Parity pinning: every function below is checked against golden vectors that
tests/golden/make_golden.py produced by importing and running the reference
itself in the build container (tests/test_oracle_golden.py).  Those .npz files
are data only (inputs + reference outputs).

Grid convention (reference ``operators.py:124-126``): voxel k = n*Nx*Ny + j*Nx + i,
n in [0,Nt) time, j in [0,Ny) rows (y), i in [0,Nx) columns (x); 3-field vectors
are SoA [t-part; x-part; y-part].  All arithmetic is float64.

Functions and the reference lines they restate:
  d1_central_weird / grad_st / div_st   operators.py:33-48, 114-142
  d1_lap / apply_laplacian_st / apply_A operators.py:95-110, 144-157; benamou_brenier.py:202-203
  grad2_central / div2_central          operators.py:52-65, 160-169, 182-191
  stepB                                 benamou_brenier.py:93-149 (vectorised)
  cg                                    scipy 1.15 sparse/linalg/_isolve/iterative.py cg (A7)
  bb_rhs / solve_step                   benamou_brenier.py:26-91
  solve                                 benamou_brenier.py:151-271
  flow_from_phi                         utils.py:44-99, 148-183 (vectorised over pixels)
  gn_*                                  classical.py:68-130, operators.py:67-79, 171-180
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla


# ----------------------------------------------------------------------------- 1-D stencils

def d1_central_weird(z, axis, h=1.0):
    """A1: operators.grad_1d_central_weird(n, h, 'N') applied along ``axis``.
    Interior (z[k+1]-z[k-1])/(2h); end rows z1-z0 and z[n-1]-z[n-2] (assigned after
    the /h, operators.py:40-46, so they are not scaled)."""
    z = np.moveaxis(np.asarray(z, dtype=np.float64), axis, 0)
    n = z.shape[0]
    out = np.empty_like(z)
    if n > 2:
        out[1:-1] = (0.5 * (z[2:] - z[:-2])) / h
    out[0] = z[1] - z[0]
    out[-1] = z[-1] - z[-2]
    return np.moveaxis(out, 0, axis)


def d1_central(z, axis, bc, h=1.0):
    """A12: operators.grad_1d_central(n, h, bc).  bc 'N': end rows zero.
    bc 'D': zero extension, out[0] = z1/(2h), out[n-1] = -z[n-2]/(2h)."""
    if bc not in ("N", "D"):
        raise NotImplementedError("These boundary conditions are not implemented")
    z = np.moveaxis(np.asarray(z, dtype=np.float64), axis, 0)
    n = z.shape[0]
    out = np.zeros_like(z)
    if n > 2:
        out[1:-1] = (0.5 * (z[2:] - z[:-2])) / h
    if bc == "D":
        out[0] = (0.5 * z[1]) / h
        out[-1] = (-0.5 * z[-2]) / h
    return np.moveaxis(out, 0, axis)


def d1_lap(z, axis, h=1.0):
    """A2: operators.lap1d(n, h, 'N'): interior z[k-1]-2z[k]+z[k+1], ends z1-z0 and
    z[n-2]-z[n-1], all /h^2."""
    z = np.moveaxis(np.asarray(z, dtype=np.float64), axis, 0)
    out = np.empty_like(z)
    out[1:-1] = z[:-2] - 2.0 * z[1:-1] + z[2:]
    out[0] = z[1] - z[0]
    out[-1] = z[-2] - z[-1]
    return np.moveaxis(out / (h * h), 0, axis)


# ----------------------------------------------------------------------------- space-time operators

def _vol(v, Nt, Ny, Nx):
    return np.asarray(v, dtype=np.float64).reshape(Nt, Ny, Nx)


def grad_st(phi, Nt, Ny, Nx):
    """A3: [D_t phi; D_x phi; D_y phi] (3N)."""
    P = _vol(phi, Nt, Ny, Nx)
    return np.concatenate([d1_central_weird(P, 0).ravel(), d1_central_weird(P, 2).ravel(),
                           d1_central_weird(P, 1).ravel()])


def div_st(w, Nt, Ny, Nx):
    """A4: D_t w_t + D_x w_x + D_y w_y with the SAME D as grad_st (no transpose)."""
    N = Nt * Ny * Nx
    w = np.asarray(w, dtype=np.float64)
    wt, wx, wy = (_vol(w[k * N:(k + 1) * N], Nt, Ny, Nx) for k in range(3))
    return (d1_central_weird(wt, 0) + d1_central_weird(wx, 2) + d1_central_weird(wy, 1)).ravel()


def apply_laplacian_st(p, Nt, Ny, Nx):
    """A5: L = Lt (x) I + I (x) (Ly (x) Ix + Iy (x) Lx), Neumann."""
    P = _vol(p, Nt, Ny, Nx)
    return (d1_lap(P, 0) + d1_lap(P, 1) + d1_lap(P, 2)).ravel()


def apply_A(p, r, eps, Nt, Ny, Nx):
    """A5: A = -r L + r eps I (benamou_brenier.py:202-203)."""
    p = np.asarray(p, dtype=np.float64)
    return -r * apply_laplacian_st(p, Nt, Ny, Nx) + (r * eps) * p


def _lap1d_csr(n):
    main = np.full(n, -2.0)
    main[0] = main[-1] = -1.0
    off = np.ones(n - 1)
    return sp.diags([off, main, off], [-1, 0, 1], shape=(n, n), format="csr")


def assemble_A(r, eps, Nt, Ny, Nx):
    """CSR form of A (used by the CPU baseline so the SpMV is scipy's, as in the reference)."""
    Lt, Ly, Lx = _lap1d_csr(Nt), _lap1d_csr(Ny), _lap1d_csr(Nx)
    It, Iy, Ix = sp.identity(Nt, format="csr"), sp.identity(Ny, format="csr"), sp.identity(Nx, format="csr")
    Lxy = sp.kron(Iy, Lx, format="csr") + sp.kron(Ly, Ix, format="csr")
    L = sp.kron(Lt, sp.identity(Nx * Ny, format="csr"), format="csr") + sp.kron(It, Lxy, format="csr")
    return (-r * L + (r * eps) * sp.identity(Nt * Nx * Ny, format="csr")).tocsr()


# ----------------------------------------------------------------------------- 2-D operators

def grad2_central(f, Nx, Ny, bc="N"):
    """A12: operators.grad(Nx, Ny, 1, 1, bc) @ f -> [G_x f; G_y f]."""
    F = np.asarray(f, dtype=np.float64).reshape(Ny, Nx)
    return np.concatenate([d1_central(F, 1, bc).ravel(), d1_central(F, 0, bc).ravel()])


def div2_central(uv, Nx, Ny, bc="D"):
    """A12: operators.div(Nx, Ny, 1, 1, bc) @ [u; v]."""
    n = Nx * Ny
    U = np.asarray(uv[:n], dtype=np.float64).reshape(Ny, Nx)
    V = np.asarray(uv[n:2 * n], dtype=np.float64).reshape(Ny, Nx)
    return (d1_central(U, 1, bc) + d1_central(V, 0, bc)).ravel()


def grad2_forward(f, Nx, Ny):
    """operators.grad_forward(Nx, Ny, 1, 1, 'N') @ f: forward differences, last row 0."""
    F = np.asarray(f, dtype=np.float64).reshape(Ny, Nx)
    gx = np.zeros_like(F)
    gy = np.zeros_like(F)
    gx[:, :-1] = F[:, 1:] - F[:, :-1]
    gy[:-1, :] = F[1:, :] - F[:-1, :]
    return np.concatenate([gx.ravel(), gy.ravel()])


# ----------------------------------------------------------------------------- stepB

def stepB(p, M):
    """A8: pointwise projection onto K = {a + |b|^2/2 <= 0}, vectorised restatement of
    benamou_brenier.py:118-148 (same formulas, same branch tests, same trig path)."""
    p = np.asarray(p, dtype=np.float64)
    al, b1, b2 = p[:M].copy(), p[M:2 * M].copy(), p[2 * M:3 * M].copy()
    out_a, out_1, out_2 = al.copy(), b1.copy(), b2.copy()
    outside = ~(2 * al + b1 ** 2 + b2 ** 2 <= 0)
    if np.any(outside):
        a = al[outside]
        rho = np.sqrt(b1[outside] ** 2 + b2[outside] ** 2)
        th = np.arctan2(b2[outside], b1[outside])
        card = -32 * (a + 1) ** 3 - 108 * rho ** 2 < 0
        zh = np.empty_like(a)
        aH = np.empty_like(a)
        rH = np.empty_like(a)
        ac, rc = a[card], rho[card]
        S = 1 / 4 * np.sqrt(2) * rc + 1 / 6 * np.sqrt(4 / 3 * ac ** 3 + 4 * ac ** 2 + 9 / 2 * rc ** 2 + 4 * ac + 4 / 3)
        c = np.power(S, 1 / 3)
        z = -1 / 3 * (ac + 1) / c + c
        zh[card] = z
        aH[card] = -z ** 2
        rH[card] = np.sqrt(2) * z
        tr = ~card
        at, rt = a[tr], rho[tr]
        with np.errstate(invalid="ignore"):
            z = 2 * np.sqrt(2 / 3) * np.sqrt(-at - 1) * np.cos(
                1 / 3 * np.arccos(np.power(3 / 2, 3 / 2) * rt / np.power(-at - 1, 3 / 2)))
        zh[tr] = z
        aH[tr] = -0.5 * z ** 2
        rH[tr] = z
        out_a[outside] = aH
        out_1[outside] = rH * np.cos(th)
        out_2[outside] = rH * np.sin(th)
    return np.concatenate([out_a, out_1, out_2])


# ----------------------------------------------------------------------------- CG (A7)

def cg(matvec, b, rtol=1e-6, maxiter=1000):
    """scipy.sparse.linalg.cg (scipy 1.15) restated for x0 = 0, M = I.
    Returns (x, info, iterations).  Stop test ``norm(r) < rtol*norm(b)`` at the top of
    every iteration on the recursive residual; p = r first, then p = beta p + r."""
    b = np.asarray(b, dtype=np.float64)
    bnrm2 = np.linalg.norm(b)
    atol = max(0.0, float(rtol) * float(bnrm2))
    if bnrm2 == 0:
        return b.copy(), 0, 0
    x = np.zeros_like(b)
    r = b.copy()
    p = None
    rho_prev = None
    for it in range(maxiter):
        if np.linalg.norm(r) < atol:
            return x, 0, it
        rho = np.dot(r, r)
        if it > 0:
            p *= rho / rho_prev
            p += r
        else:
            p = r.copy()
        q = matvec(p)
        alpha = rho / np.dot(p, q)
        x += alpha * p
        r -= alpha * q
        rho_prev = rho
    return x, maxiter, maxiter


# ----------------------------------------------------------------------------- BB solver

def bb_rhs(mu, q, rho0, rhoT, r, Nt, Ny, Nx):
    """A6 RHS: F = div_st(mu - r q), then the temporal BC correction (dt = 1)."""
    nxy = Nx * Ny
    F = div_st(mu - r * q, Nt, Ny, Nx)
    F[:nxy] -= rho0 - mu[:nxy] + r * q[:nxy]
    lo = (Nt - 1) * nxy
    F[lo:lo + nxy] += rhoT - mu[lo:lo + nxy] + r * q[lo:lo + nxy]
    return F


def solve_step(mu, q, rho0, rhoT, r, matvec, Nt, Ny, Nx, rtol=1e-6, maxiter=1000):
    """A6: returns (phi, info, cg_iterations)."""
    F = bb_rhs(mu, q, rho0, rhoT, r, Nt, Ny, Nx)
    return cg(matvec, F, rtol=rtol, maxiter=maxiter)


def solve(rho0, rhoT, Nt, Nx, Ny, r=1, convergence_tol=0.3, reg_epsilon=1e-3, max_it=100,
          assembled=True, log=print, stats=None, stop_rules=True):
    """A11: benamou_brenier.solve restated.  Returns (u, v, m); prints the reference's
    per-iteration line ``f"{crit} ({i+1}/{max_it})"``.  ``stats`` (dict) receives
    crit, cg_its and phi.  ``stop_rules=False`` runs exactly max_it iterations (bench)."""
    N = Nt * Nx * Ny
    nxy = Nx * Ny
    rho0 = np.asarray(rho0, dtype=np.float64)
    rhoT = np.asarray(rhoT, dtype=np.float64)
    q = np.zeros(3 * N)
    mu = np.zeros(3 * N)
    for n in range(Nt):
        mu[n * nxy:(n + 1) * nxy] = (1 - n / (Nt - 1)) * rho0 + (n / (Nt - 1)) * rhoT
    if assembled:
        A = assemble_A(r, reg_epsilon, Nt, Ny, Nx)
        matvec = A.dot
    else:
        def matvec(p):
            return apply_A(p, r, reg_epsilon, Nt, Ny, Nx)
    crit = -1
    crits, its = [], []
    phi = None
    for i in range(max_it):
        phi, info, k = solve_step(mu, q, rho0, rhoT, r, matvec, Nt, Ny, Nx)
        its.append(k)
        if info > 0:
            log(f"WARNING: CG did not converge in {info} iterations.")
        g = grad_st(phi, Nt, Ny, Nx)
        q = stepB(g + (1.0 / r) * mu, N)
        mu = mu + r * (g - q)
        mu[:N] = np.maximum(mu[:N], 0)
        gt, gx, gy = g[:N], g[N:2 * N], g[2 * N:]
        res = gt + 0.5 * (gx ** 2 + gy ** 2)
        num = np.sum(mu[:N] * np.abs(res))
        den = np.sum(mu[:N] * (gx ** 2 + gy ** 2))
        prev = crit
        crit = np.sqrt(num / (den + 1e-10))
        crits.append(crit)
        log(str(crit) + " (" + str(i + 1) + "/" + str(max_it) + ")")
        if stop_rules:
            if crit <= convergence_tol:
                break
            if prev >= 0 and np.abs(prev - crit) < 1e-5:
                break
    if stats is not None:
        stats.update(crit=np.array(crits), cg_its=np.array(its), phi=phi, mu=mu, q=q)
    return flow_from_phi(phi, Nt, Nx, Ny)


# ----------------------------------------------------------------------------- flow extraction

def flow_from_phi(phi, Nt, Nx, Ny):
    """A13/A14: utils.opticalflow_from_benamoubrenier with the per-pixel
    reconstructTrajectory loop vectorised over all pixels (same operation order)."""
    nxy = Nx * Ny
    phi = np.asarray(phi, dtype=np.float64)
    un = np.zeros((Nt, nxy))
    vn = np.zeros((Nt, nxy))
    for n in range(Nt - 1):
        g = grad2_central(phi[n * nxy:(n + 1) * nxy], Nx, Ny, "N")
        un[n] = g[:nxy]
        vn[n] = g[nxy:]
    jj, ii = np.meshgrid(np.arange(Ny), np.arange(Nx), indexing="ij")
    x0 = ii.ravel().astype(np.float64)
    y0 = jj.ravel().astype(np.float64)
    x = x0.copy()
    y = y0.copy()
    for n in range(Nt - 1):
        tx = np.clip(np.trunc(x), 0, Nx - 2).astype(np.int64)
        ty = np.clip(np.trunc(y), 0, Ny - 2).astype(np.int64)
        dX = x - tx
        dY = y - ty
        w1 = (1 - dY) * (1 - dX)
        w2 = dX * (1 - dY)
        w3 = dY * dX
        w4 = (1 - dX) * dY
        i00 = ty * Nx + tx
        i01 = i00 + 1
        i11 = (ty + 1) * Nx + tx + 1
        i10 = (ty + 1) * Nx + tx
        u_, v_ = un[n], vn[n]
        x = x + (w1 * u_[i00] + w2 * u_[i01] + w3 * u_[i11] + w4 * u_[i10])
        y = y + (w1 * v_[i00] + w2 * v_[i01] + w3 * v_[i11] + w4 * v_[i10])
    u = x - x0
    v = y - y0
    m = -div2_central(np.concatenate([u, v]), Nx, Ny, "D")
    return u, v, m


# ----------------------------------------------------------------------------- GN baseline

def gn_coeffs(f1, f2, w, h):
    """classical.py:90-100: fx, fy central differences of f2 (zero on the edge
    columns / rows), ft = f2 - f1."""
    F2 = np.asarray(f2, dtype=np.float64).reshape(h, w)
    fx = np.zeros((h, w))
    fy = np.zeros((h, w))
    fx[:, 1:-1] = 0.5 * (F2[:, 2:] - F2[:, :-2])
    fy[1:-1, :] = 0.5 * (F2[2:, :] - F2[:-2, :])
    ft = np.asarray(f2, dtype=np.float64) - np.asarray(f1, dtype=np.float64)
    return fx.ravel(), fy.ravel(), ft


def gn_neg_lap(z, w, h):
    """-Lambda2 z = G^T G z, G = grad_forward (5-point Neumann, classical.py:102-104)."""
    Z = np.asarray(z, dtype=np.float64).reshape(h, w)
    out = np.zeros_like(Z)
    dx = Z[:, 1:] - Z[:, :-1]
    dy = Z[1:, :] - Z[:-1, :]
    out[:, :-1] -= dx
    out[:, 1:] += dx
    out[:-1, :] -= dy
    out[1:, :] += dy
    return out.ravel()


def gn_apply(x, f1, f2, w, h, alpha, lam):
    """Matrix-free A @ x for classical.py:106-108's block system."""
    n = w * h
    fx, fy, _ = gn_coeffs(f1, f2, w, h)
    f2 = np.asarray(f2, dtype=np.float64)
    u, v, m = x[:n], x[n:2 * n], x[2 * n:]
    s = fx * u + fy * v - f2 * m
    yu = alpha * gn_neg_lap(u, w, h) + fx * s
    yv = alpha * gn_neg_lap(v, w, h) + fy * s
    ym = lam * gn_neg_lap(m, w, h) - f2 * s
    return np.concatenate([yu, yv, ym])


def gn_assemble(f1, f2, w, h, alpha, lam):
    """CSR system (A, b) of classical.GLLOpticalFlow.assemble."""
    fx, fy, ft = gn_coeffs(f1, f2, w, h)
    f2 = np.asarray(f2, dtype=np.float64)
    Lx, Ly = _lap1d_csr(w), _lap1d_csr(h)
    lap = sp.kron(sp.identity(h), Lx, format="csr") + sp.kron(Ly, sp.identity(w), format="csr")
    d = sp.diags
    A = sp.bmat([[-alpha * lap + d(fx * fx), d(fx * fy), d(-fx * f2)],
                 [d(fy * fx), -alpha * lap + d(fy * fy), d(-fy * f2)],
                 [d(-f2 * fx), d(-f2 * fy), -lam * lap + d(f2 * f2)]]).tocsr()
    b = np.concatenate([-fx * ft, -fy * ft, f2 * ft])
    return A, b


def gn_solve(f1, f2, w, h, alpha, lam):
    """classical.py:113-130: direct solve (SuperLU), split into u, v, m."""
    A, b = gn_assemble(f1, f2, w, h, alpha, lam)
    x = spla.spsolve(A, b)
    n = w * h
    return x[:n], x[n:2 * n], x[2 * n:]


# ----------------------------------------------------------------------------- evaluation (§8(f) row 1)

def apply_opticalflow(f1, u, v, w, h, m=None):
    """utils.apply_opticalflow (utils.py:186-248) restated over all pixels: backward
    bilinear warp of (1+m) f1 (m None: unscaled); weights from the unclamped fractional
    parts, indices clamped, the +1 neighbour collapsed onto the edge pixel."""
    f1 = np.asarray(f1, dtype=np.float64)
    if m is not None:
        f1 = (1 + np.asarray(m, dtype=np.float64)) * f1
    ii, jj = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    ti = ii.ravel() - np.asarray(v, dtype=np.float64)
    tj = jj.ravel() - np.asarray(u, dtype=np.float64)
    dI = ti - np.trunc(ti)
    dJ = tj - np.trunc(tj)
    w1, w2, w3, w4 = (1 - dI) * (1 - dJ), dJ * (1 - dI), dI * dJ, (1 - dJ) * dI
    ti = np.where(ti >= h, h - 1, ti)
    tj = np.where(tj >= w, w - 1, tj)
    ti = np.where(ti < 0, 0, ti)
    tj = np.where(tj < 0, 0, tj)
    a = ti.astype(np.int64)
    b = tj.astype(np.int64)
    a1 = np.where(a < h - 1, a + 1, a)
    b1 = np.where(b < w - 1, b + 1, b)
    x = w1 * f1[a * w + b]
    x = x + w2 * f1[a * w + b1]
    x = x + w3 * f1[a1 * w + b1]
    x = x + w4 * f1[a1 * w + b]
    return x


def EE(w, h, u, v, uGT, vGT):
    """utils.EE (utils.py:294-315): mean and std of the endpoint error over EE <= 50."""
    e = np.sqrt((u - uGT) ** 2 + (v - vGT) ** 2)[: w * h]
    kept = e[e <= 50]
    mean = np.sum(kept) / len(kept)
    return mean, np.sqrt(np.sum((kept - mean) ** 2) / len(kept))


def AE(w, h, u, v, uGT, vGT):
    """utils.AE (utils.py:317-338): mean and std of the angular error, NaN ignored."""
    a = np.arccos((1.0 + u * uGT + v * vGT) / (np.sqrt(1.0 + u ** 2 + v ** 2) * np.sqrt(1.0 + uGT ** 2 + vGT ** 2)))
    kept = a[: w * h][~np.isnan(a[: w * h])]
    mean = np.sum(kept) / len(kept)
    return mean, np.sqrt(np.sum((kept - mean) ** 2) / len(kept))


def IE(w, h, I, IGT):
    """utils.IE (utils.py:340-354): RMS of 255 I - 255 IGT."""
    return np.sqrt(np.sum((255 * I - 255 * IGT) ** 2) / (w * h))
