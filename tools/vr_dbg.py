import sys, os
sys.path[:0] = ['/root/repo', '/root/repo/optical-flow-optimal-transport_amd']
import numpy as np
from foto.bb import BBSolver
d = np.load('tests/golden/bb_tex.npz')
Nt, Ny, Nx = (int(s) for s in d["shape"])
r, tol, eps, max_it = d["params"]
for vr in (1, 2, 3):
    for rep in range(2):
        with BBSolver(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, reg_epsilon=eps, virtual_ranks=vr, cg_mode=3) as s:
            s.iterate(int(max_it), tol, True)
            print(os.environ.get("TAG", ""), "vr", vr, "rep", rep, list(s.cg_its), s.stats().get("cg_redo"), flush=True)
