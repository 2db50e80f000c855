"""GN solve timing on the GPU (sinusoid pairs, alpha 0.1, lambda 0.2); A/B knobs via env
(FOTO_GN_MG, FOTO_GN_GRAPH).  usage: python tools/gn_time.py"""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..",
                                              "optical-flow-optimal-transport_amd"))
from foto import gn  # noqa: E402
from foto.synthetic import sinusoid_pair  # noqa: E402

for (w, h) in [(320, 240), (640, 480)]:
    f1, f2 = sinusoid_pair(w, h)
    ts = []
    for rep in range(3):
        t = time.perf_counter()
        u, v, m, info, its = gn.solve(f1, f2, w, h, 0.1, 0.2)
        ts.append(time.perf_counter() - t)
    dt = min(ts)
    print(f"GN {w}x{h}: {dt*1e3:.1f} ms (best of 3; {[round(1e3 * x, 1) for x in ts]}), {its} PCG its, info {info}, "
          f"{dt/its*1e6:.1f} us/it", flush=True)
