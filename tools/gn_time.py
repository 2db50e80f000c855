"""GN solve timing on the GPU (sinusoid pairs, alpha 0.1, lambda 0.2): one-shot solves, and a
reused plan with its create / solve / destroy times split.  A/B knobs via env (FOTO_GN_MG).
usage: python tools/gn_time.py [w h ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "optical-flow-optimal-transport_amd"))
from foto import gn  # noqa: E402
from foto.synthetic import sinusoid_pair  # noqa: E402

args = [int(a) for a in sys.argv[1:]]
sizes = list(zip(args[::2], args[1::2])) or [(320, 240), (640, 480)]
for (w, h) in sizes:
    f1, f2 = sinusoid_pair(w, h)
    ts = []
    for rep in range(3):
        t = time.perf_counter()
        u, v, m, info, its = gn.solve(f1, f2, w, h, 0.1, 0.2)
        ts.append(time.perf_counter() - t)
    print(f"GN {w}x{h} one-shot: {1e3 * min(ts):.2f} ms (best of 3; {[round(1e3 * x, 2) for x in ts]}), "
          f"{its} PCG its, info {info}", flush=True)
    t0 = time.perf_counter()
    P = gn.Plan(w, h, 0.1, 0.2)
    t1 = time.perf_counter()
    sol = []
    for rep in range(4):
        t = time.perf_counter()
        P.solve(f1, f2)
        sol.append((time.perf_counter() - t, P.timing()))
    t2 = time.perf_counter()
    P.close()
    t3 = time.perf_counter()
    best = min(sol, key=lambda s: s[0])
    print(f"GN {w}x{h} plan: create {1e3 * (t1 - t0):.2f} ms, solve {[round(1e3 * s[0], 2) for s in sol]} ms, "
          f"destroy {1e3 * (t3 - t2):.2f} ms; best solve device {best[1]}, "
          f"{1e3 * best[1]['ms_pcg'] / best[1]['iterations']:.1f} us/it", flush=True)
