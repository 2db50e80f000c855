#!/usr/bin/env python3
"""Outer iterations/s of the Benamou-Brenier solve on one GPU at the SURVEY.md §8 config sizes
(synthetic translating-Gaussian pairs; r = 1, eps = 1e-2, stop rules off).
usage: python tools/size_sweep.py [NxxNyxNt ...] [--mode=M] [--kernels]"""
import sys
import time

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..",
                                              "optical-flow-optimal-transport_amd"))
from foto.bb import BBSolver  # noqa: E402
from foto.synthetic import translating_gaussian  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
kern = "--kernels" in sys.argv   # also a timed pass with HIP events around every launch
mode = int(next((a.split("=")[1] for a in sys.argv if a.startswith("--mode=")), "3"))
sizes = args or ["64x64x8", "584x388x32", "640x480x32", "1024x1024x64"]
for sz in sizes:
    Nx, Ny, Nt = (int(v) for v in sz.split("x"))
    rho0, rhoT = translating_gaussian(Nx, Ny)
    with BBSolver(rho0, rhoT, Nt, Nx, Ny, r=1.0, reg_epsilon=1e-2, device=0, cg_mode=mode) as s:
        s.iterate(2, 0.0, stop_rules=False)
        s.sync()
        k = 10
        t = time.perf_counter()
        s.iterate(k, 0.0, stop_rules=False)
        s.sync()
        dt = time.perf_counter() - t
        its = s.cg_its[-k:]
        print(f"{sz}: {k / dt:8.2f} outer it/s, {1e3 * dt / k:8.3f} ms/outer, CG its {its}", flush=True)
        if kern:
            s.reset_stats()
            s.set_timing(True)
            s.iterate(k, 0.0, stop_rules=False)
            s.sync()
            s.set_timing(False)
            import ctypes
            from foto import _lib
            n = Nx * Ny * Nt
            us = (ctypes.c_double * 2)()
            if n % 2 == 0 and n * 8 < 2 ** 31 and _lib.lib().foto_stream_probe(n, 10, us) == 0:
                print(f"    stream probe (r, q of this box): {min(us[0], us[1]):8.1f} us = "
                      f"{32 * n / (min(us[0], us[1]) * 1e-6) / 1e9:7.1f} GB/s", flush=True)
            for name, v in s.stats()["kernels"].items():
                n = max(v["n"], 1)
                us = 1e3 * v["ms"] / n
                print(f"    {name:8s} {v['n']:5d} launches  {us:9.1f} us avg  {v['bytes'] / n / (us * 1e-6) / 1e9:8.1f} GB/s "
                      f"(algorithmic)  {v['ms'] / k:7.3f} ms per outer", flush=True)
