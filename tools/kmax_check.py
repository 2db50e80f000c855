"""Gauss CG at high iteration counts (the solution table's K range): mode 3 against the s-step
CG (mode 2) on the bench grid and a noisy 96x80x16 pair at small reg_epsilon; run with
FOTO_LIB pointing at a build with a larger FOTO_GQ_KMAX to see whether the compressed measure
stays accurate past 512 steps.  Prints K, the redo count, phi and crit differences."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "optical-flow-optimal-transport_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from foto.bb import BBSolver
from foto.synthetic import translating_gaussian
from test_gpu_batch import _pair

cases = [("bench", 32, 640, 480, eps, translating_gaussian(640, 480)) for eps in (1e-3, 1.6e-3, 2.5e-3)]
cases += [("noisy", 16, 96, 80, eps, _pair(96, 80, 2, shift=3)) for eps in (1e-3, 3e-4)]
for name, Nt, Nx, Ny, eps, (r0, r1) in cases:
    out = {}
    for mode in (2, 3):
        with BBSolver(r0, r1, Nt, Nx, Ny, reg_epsilon=eps, cg_mode=mode) as s:
            s.iterate(3, 0.0, False)
            out[mode] = (list(s.cg_its), np.array(s.crit), s.phi(), s.stats()["cg_redo"])
    (k2, c2, p2, _), (k3, c3, p3, rd) = out[2], out[3]
    prel = float(np.abs(p3 - p2).max() / np.abs(p2).max())
    crel = float(np.abs(c3 - c2).max() / np.abs(c2).max())
    print(f"{name} eps {eps}: K s-step {k2} gauss {k3} redo {rd}; phi rel {prel:.2e} crit rel {crel:.2e}")
