#!/usr/bin/env python3
"""Bit-identity of two library builds on the bench grid: run as
    FOTO_LIB=a.so python tools/bitcmp.py save A.npz [Nt Nx Ny iters sharded_W]
    FOTO_LIB=b.so python tools/bitcmp.py save B.npz ...
    python tools/bitcmp.py cmp A.npz B.npz"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "optical-flow-optimal-transport_amd"))
if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in a.files)
    print("bit-identical" if same else "DIFFERENT", {k: float(np.max(np.abs(a[k] - b[k]))) for k in a.files})
    sys.exit(0 if same else 1)
from foto.bb import BBSolver  # noqa: E402
from foto.synthetic import translating_gaussian  # noqa: E402
Nt, Nx, Ny, iters, vr = (int(v) for v in (sys.argv[3:8] + ["32", "640", "480", "6", "1"][len(sys.argv[3:8]):]))
rho0, rhoT = translating_gaussian(Nx, Ny)
with BBSolver(rho0, rhoT, Nt, Nx, Ny, r=1.0, reg_epsilon=1e-2, cg_mode=3, virtual_ranks=vr) as s:
    s.iterate(iters, 0.0, stop_rules=False)
    np.savez(sys.argv[2], cg=np.array(s.cg_its), crit=np.array(s.crit), phi=s.phi())
