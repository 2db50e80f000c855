import sys, time
sys.path.insert(0,'/root/repo/tools'); sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/optical-flow-optimal-transport_amd')
import numpy as np
from scipy import fft
import gautschi_proto as G
from oracle import foto_oracle as O
from foto.synthetic import translating_gaussian

def gauss_from_cheb_moments(mu, m):
    """m-point Gauss rule on [-1,1] for a measure given its Chebyshev moments mu_j = sum w T_j(u), j<2m.
    Returns nodes, weights (possibly fewer nodes if degenerate)."""
    # monic Chebyshev moments: p_0 = 1, p_k = T_k/2^(k-1)
    nu = mu.copy()
    for k in range(1, len(nu)): nu[k] = mu[k] / 2.0**(k-1)
    if nu[0] <= 0: return np.zeros(0), np.zeros(0)
    al, be = G.mod_chebyshev(nu, m)
    # truncate at degeneracy
    n = m
    for k in range(1, m):
        if not (be[k] > 1e-13 * 1.0):   # beta in u-units (interval length 2): tiny means measure has <k+1 points
            n = k; break
    J = np.diag(al[:n]) + np.diag(np.sqrt(be[1:n]), 1) + np.diag(np.sqrt(be[1:n]), -1)
    x, V = np.linalg.eigh(J)
    return x, be[0] * V[0, :]**2

def compress(lam, w, c0, c1, B, m):
    lt = np.clip((lam - c0) / c1, -1, 1)
    th = np.arccos(lt)
    h = np.pi / (2 * B)
    b = np.minimum((th / (2 * h)).astype(np.int64), B - 1)
    u = (th - (2 * b + 1) * h) / h
    # Chebyshev moments per bin
    mom = np.zeros((B, 2 * m))
    t0 = np.ones_like(u); t1 = u.copy()
    mom[:, 0] = np.bincount(b, w, B)
    mom[:, 1] = np.bincount(b, w * t1, B)
    for j in range(2, 2 * m):
        t0, t1 = t1, 2 * u * t1 - t0
        mom[:, j] = np.bincount(b, w * t1, B)
    nodes, wts = [], []
    for k in range(B):
        if mom[k, 0] <= 0: continue
        x, ww = gauss_from_cheb_moments(mom[k], m)
        thk = (2 * k + 1) * h + x * h
        nodes.append(c0 + c1 * np.cos(thk)); wts.append(ww)
    return np.concatenate(nodes), np.concatenate(wts)

def cg_measure(lam, w, rtol, maxiter=2000):
    """CG on the diagonal system (lam, b with b^2 = w): residual norms and step coeffs, using
    vectors in the 'sqrt(w)' representation."""
    b = np.sqrt(w)
    _, k, rn = G.diag_cg(lam, b, rtol, maxiter)
    return k, np.array(rn)

Nx,Ny,Nt,r,eps = [int(a) for a in sys.argv[1:4]] + [1.0, float(sys.argv[4])]
B, m = int(sys.argv[5]), int(sys.argv[6])
rho0,rhoT = translating_gaussian(Nx,Ny)
N,nxy = Nt*Nx*Ny, Nx*Ny
lam=(r*eps+r*(G.eig1d(Nt)[:,None,None]+G.eig1d(Ny)[None,:,None]+G.eig1d(Nx)[None,None,:])).ravel()
lmin,lmax=r*eps,r*eps+r*(G.eig1d(Nt)[-1]+G.eig1d(Ny)[-1]+G.eig1d(Nx)[-1])
c0,c1=0.5*(lmax+lmin),0.5*(lmax-lmin)
A=O.assemble_A(r,eps,Nt,Ny,Nx)
mu=np.zeros(3*N); q=np.zeros(3*N)
for n in range(Nt): mu[n*nxy:(n+1)*nxy]=(1-n/(Nt-1))*rho0+(n/(Nt-1))*rhoT
for it in range(int(sys.argv[7]) if len(sys.argv)>7 else 3):
    F=O.bb_rhs(mu,q,rho0,rhoT,r,Nt,Ny,Nx)
    phi,info,kref=O.cg(A.dot,F)
    bh=fft.dctn(F.reshape(Nt,Ny,Nx),type=2,norm='ortho').ravel()
    t=time.time()
    nodes,wts=compress(lam,bh*bh,c0,c1,B,m)
    kd, rnd = cg_measure(lam, bh*bh, 1e-6)
    kc, rnc = cg_measure(nodes, wts, 1e-6)
    mm=min(len(rnd),len(rnc))
    rel=np.abs(rnc[:mm]-rnd[:mm])/rnd[:mm]
    print(f"outer {it}: scipy {kref} diag {kd} compressed {kc} ({len(nodes)} nodes, min w {wts.min():.1e}); rel diff rn max {rel.max():.2e} at {rel.argmax()}, at end {rel[-1]:.2e}", flush=True)
    g=O.grad_st(phi,Nt,Ny,Nx); q=O.stepB(g+(1.0/r)*mu,N); mu=mu+r*(g-q); mu[:N]=np.maximum(mu[:N],0)

def cg_coeffs(nodes, wts, rtol, maxiter=2000):
    """scalar CG on the compressed measure: alphas, betas, K (scipy's order: p = r + beta p)."""
    r = np.ones_like(nodes); p = None; x = np.zeros_like(nodes)
    bn2 = wts.sum(); al=[]; be=[]; rho_prev=None
    for k in range(maxiter):
        rho = (wts*r*r).sum()
        if np.sqrt(rho) < rtol*np.sqrt(bn2): return np.array(al), np.array(be), k
        if k == 0: p = r.copy(); be.append(0.0)
        else: b_ = rho/rho_prev; p = r + b_*p; be.append(b_)
        q = nodes*p; a = rho/(wts*p*q).sum(); al.append(a)
        r = r - a*q; rho_prev = rho
    return np.array(al), np.array(be), maxiter

def q_eval(lam, al, be):
    x = np.zeros_like(lam); r = np.ones_like(lam); p = np.zeros_like(lam)
    for k in range(len(al)):
        p = r + be[k]*p
        x = x + al[k]*p
        r = r - al[k]*lam*p
    return x

def q_table_eval(lam, al, be, c0, c1, B, n):
    lt = np.clip((lam - c0)/c1, -1, 1); th = np.arccos(lt); h = np.pi/(2*B)
    b = np.minimum((th/(2*h)).astype(np.int64), B-1); u = (th - (2*b+1)*h)/h
    # Chebyshev nodes in u, values of Q at them
    j = np.arange(n); un = np.cos(np.pi*(j+0.5)/n)
    thn = (2*np.arange(B)[:,None]+1)*h + un[None,:]*h
    vals = q_eval(c0 + c1*np.cos(thn).ravel(), al, be).reshape(B, n)
    # Chebyshev coefficients per bin
    T = np.cos(np.outer(np.arange(n), np.pi*(j+0.5)/n))   # T_k(un_j)
    coef = (2.0/n) * vals @ T.T; coef[:,0] *= 0.5
    # Clenshaw
    c = coef[b]; b1 = np.zeros_like(u); b2 = np.zeros_like(u)
    for k in range(n-1, 0, -1):
        b1, b2 = c[:,k] + 2*u*b1 - b2, b1
    return c[:,0] + u*b1 - b2

if __name__ == "__main__" and len(sys.argv) > 8:
    Bq, nq = int(sys.argv[8]), int(sys.argv[9])
    F=O.bb_rhs(mu,q,rho0,rhoT,r,Nt,Ny,Nx)
    phi,info,kref=O.cg(A.dot,F)
    bh=fft.dctn(F.reshape(Nt,Ny,Nx),type=2,norm='ortho').ravel()
    nodes,wts=compress(lam,bh*bh,c0,c1,B,m)
    al,be,K = cg_coeffs(nodes,wts,1e-6)
    xd = q_eval(lam, al, be)*bh
    xt = q_table_eval(lam, al, be, c0, c1, Bq, nq)*bh
    phid = fft.idctn(xd.reshape(Nt,Ny,Nx),type=2,norm='ortho').ravel()
    phit = fft.idctn(xt.reshape(Nt,Ny,Nx),type=2,norm='ortho').ravel()
    print("K", K, "scipy", kref, "table vs direct Q:", np.abs(xt-xd).max()/np.abs(xd).max(),
          "direct vs scipy phi:", np.abs(phid-phi).max()/np.abs(phi).max(), "table vs scipy:", np.abs(phit-phi).max()/np.abs(phi).max())
    res = np.linalg.norm(bh - lam*xt)/np.linalg.norm(bh)
    print("true residual (table)", res)
