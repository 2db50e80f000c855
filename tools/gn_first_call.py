#!/usr/bin/env python3
"""GN plan creation and first solves, timed from Python (first_call_ms studies; set
FOTO_GN_TRACE=1 for the library's per-phase breakdown on stderr).
usage: python tools/gn_first_call.py [W H]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "optical-flow-optimal-transport_amd"))
from foto import gn, _lib  # noqa: E402
from foto.synthetic import sinusoid_pair  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
w, h = (int(args[0]), int(args[1])) if len(args) > 1 else (640, 480)
_lib.device_count()   # HIP initialised outside the timings (bench.py runs the BB solve first)
if "--after-bb" in sys.argv:   # as in bench.py: a BB solve (its context and stream) first
    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian
    r0, r1 = translating_gaussian(64, 48)
    with BBSolver(r0, r1, 8, 64, 48, r=1.0, reg_epsilon=1e-2, device=0) as s:
        s.iterate(2, 0.0, stop_rules=False)
f1, f2 = sinusoid_pair(w, h)
g1, g2 = sinusoid_pair(w, h, dx=0.7, dy=1.1)
for label, a, b in (("first call (plan + solve)", f1, f2), ("same size, new pair", g1, g2), ("repeat", g1, g2)):
    t = time.perf_counter()
    _, _, _, info, its = gn.solve(a, b, w, h, 0.1, 0.2)
    print(f"{label:28s} {1e3 * (time.perf_counter() - t):8.2f} ms  ({its} PCG its)", flush=True)
t = time.perf_counter()
p = gn.Plan(w, h, 0.1, 0.2)
print(f"{'Plan() alone':28s} {1e3 * (time.perf_counter() - t):8.2f} ms", flush=True)
p.close()
