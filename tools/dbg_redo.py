import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "optical-flow-optimal-transport_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np
from foto.bb import BBSolver
from test_gpu_batch import _pair
Nt, Nx, Ny = 16, 96, 80
b0, b1 = _pair(Nx, Ny, 2, shift=3)
for pipe in ("1", "0"):
    os.environ["FOTO_PIPE"] = pipe
    for mode in (3, 2):
        with BBSolver(b0, b1, Nt, Nx, Ny, cg_mode=mode) as s:
            s.iterate(6, 0.0, False)
            print("pipe", pipe, "mode", mode, "its", s.cg_its, "info", s.cg_info, "redo", s.stats()["cg_redo"])
for eps in (1e-3, 1e-2):
    with BBSolver(b0, b1, Nt, Nx, Ny, reg_epsilon=eps, cg_mode=3) as s:
        s.iterate(3, 0.0, False)
        print("eps", eps, "its", s.cg_its, "redo", s.stats()["cg_redo"])
