import sys, time, numpy as np
sys.path.insert(0, '/root/repo/optical-flow-optimal-transport_amd')
from foto import gn
for (w, h) in [(320, 240), (640, 480)]:
    y, x = np.mgrid[0:h, 0:w].astype(float)
    f1 = 0.5 + 0.4 * np.sin(x / 7) * np.cos(y / 5)
    f2 = 0.5 + 0.4 * np.sin((x - 1.3) / 7) * np.cos((y - 0.4) / 5)
    for rep in range(2):
        t = time.perf_counter()
        u, v, m, info, its = gn.solve(f1.ravel(), f2.ravel(), w, h, 0.1, 0.2)
        dt = time.perf_counter() - t
    print(f"GN {w}x{h}: {dt*1e3:.1f} ms, {its} PCG its, info {info}, {dt/its*1e6:.1f} us/it", flush=True)
