# Experiment (CPU, test infrastructure: imports the oracle and the numpy plan restatement).
# usage: python tools/cs_bound_exp.py exact|cs 80x60x32 [limit]
# Pass counts of the s-step plan with the exact |terms| cancellation ratio vs the Cauchy-Schwarz
# bound (|H_ac| <= sqrt(H_aa H_cc)), on the first BB solve of a translating-Gaussian pair.
import sys, math, time
import numpy as np
import os; _R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [os.path.join(_R, "tests"), _R, os.path.join(_R, "optical-flow-optimal-transport_amd")]
import test_sstep_plan as T
from oracle import foto_oracle as O
from foto.synthetic import translating_gaussian
mode = sys.argv[1]; Nx, Ny, Nt = (int(v) for v in sys.argv[2].split("x"))
lim = float(sys.argv[3]) if len(sys.argv) > 3 else T.S_CLIM
T.S_CLIM = lim
orig_plan = T._plan
if mode == "cs":
    src = open(T.__file__).read()
    # rebuild _plan with the bound in ip()
    code = src[src.index("def _plan("):src.index("def _interval(")]
    code = code.replace("""        t = U[:, None] * H * V[None, :]
        s = t.sum()
        return s, (np.abs(t).sum() / abs(s) if s != 0 else np.inf)""",
"""        t = U[:, None] * H * V[None, :]
        s = t.sum()
        d = np.sqrt(np.maximum(np.diag(H), 0.0))
        bound = (np.abs(U) * d).sum() * (np.abs(V) * d).sum()
        return s, (bound / abs(s) if s != 0 else np.inf)""")
    ns = dict(T.__dict__)
    exec(code, ns)
    T._plan = ns["_plan"]
rho0, rhoT = translating_gaussian(Nx, Ny)
N = Nt * Nx * Ny
mu0 = np.concatenate([np.concatenate([(1 - n / (Nt - 1)) * rho0 + (n / (Nt - 1)) * rhoT for n in range(Nt)]), np.zeros(2 * N)])
b = O.bb_rhs(mu0, np.zeros(3 * N), rho0, rhoT, 1.0, Nt, Ny, Nx)
st = {}
t0 = time.time()
x, info, k = T.sstep_cg(b, Nt, Ny, Nx, 1.0, 1e-2, stats=st)
res = np.linalg.norm(b - O.apply_A(x, 1.0, 1e-2, Nt, Ny, Nx)) / np.linalg.norm(b)
print(f"{mode} lim {lim:g} {Nx}x{Ny}x{Nt}: its {k} passes {st['passes']} info {info} true res {res:.3e} ({time.time()-t0:.0f}s)")
