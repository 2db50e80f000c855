#!/usr/bin/env python3
"""Compute-only proxy of the multi-GPU strong-scaling curve (communication excluded).

The 640x480x32 bench problem is split into W time slabs / row boxes exactly as W RCCL ranks
would split it, but as W in-process shards on ONE device (virtual ranks: the same kernels,
the same transfer lists, executed as device copies).  Every kernel launch of a shard is that
rank's work on a whole GPU, so the per-launch HIP-event times (foto_bb_set_timing) summed
over one shard are what one rank of a W-GPU run computes per outer iteration.  The device
copies standing in for RCCL are not kernels and are not counted: communication (halo and
moment all-gathers, the slab <-> row-box all-to-alls, RCCL launch latency) is EXCLUDED, so
the curve is an upper bound on what W GPUs can reach.

    python tools/proxy_scaling.py [--worlds 1,2,4,8] [--steps 10] [--warmup 3] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "optical-flow-optimal-transport_amd"))

import numpy as np  # noqa: E402

NX, NY, NT = 640, 480, 32
R, EPS = 1.0, 1e-2


def measure(W, steps, warmup):
    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian
    rho0, rhoT = translating_gaussian(NX, NY)
    with BBSolver(rho0, rhoT, NT, NX, NY, r=R, reg_epsilon=EPS, virtual_ranks=W) as s:
        s.iterate(warmup, 0.0, stop_rules=False)
        s.sync()
        t = time.perf_counter()
        s.iterate(steps, 0.0, stop_rules=False)
        s.sync()
        wall = (time.perf_counter() - t) / steps
        n0 = len(s.cg_its)
        s.reset_stats()
        s.set_timing(True)
        s.iterate(steps, 0.0, stop_rules=False)
        s.sync()
        st = s.stats()
        cg = float(np.mean(s.cg_its[n0:]))
    k = {name: v["ms"] / steps / W for name, v in st["kernels"].items()}     # per rank, per outer iteration
    n = {name: v["n"] / steps / W for name, v in st["kernels"].items()}
    return {"W": W, "rank_ms": sum(k.values()), "kernels_ms": k, "launches": n, "cg_its": cg,
            "one_device_wall_ms": wall * 1e3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = [measure(int(w), args.steps, args.warmup) for w in args.worlds.split(",")]
    base = rows[0]["rank_ms"] * rows[0]["W"]
    lines = [f"# compute-only proxy, {NX}x{NY}x{NT}, r={R}, eps={EPS}: per-rank kernel time of W virtual shards on one",
             "# MI355X (HIP events around every launch); COMMUNICATION EXCLUDED (halo / moment all-gathers,",
             "# slab<->box all-to-alls and RCCL latency are not counted) -> an upper bound for W GPUs.",
             f"# {'W':>2} {'rank ms/it':>10} {'proxy it/s':>10} {'eff':>5} {'CG its':>6} {'cg launches':>13} "
             f"{'cg ms':>8} {'dct ms':>7} {'prox+rhs ms':>11} {'flow/other':>10}"]
    for r in rows:
        k = r["kernels_ms"]
        eff = base / (r["W"] * r["rank_ms"])
        lines.append(f"  {r['W']:>2} {r['rank_ms']:10.3f} {1e3 / r['rank_ms']:10.1f} {eff:5.2f} {r['cg_its']:6.1f} "
                     f"{r['launches'].get('spec_cg', 0):13.1f} {k.get('spec_cg', 0):8.3f} {k.get('dct', 0):7.3f} "
                     f"{k.get('prox', 0) + k.get('rhs', 0):11.3f} {k.get('flow', 0) + k.get('other', 0):10.3f}")
    lines.append("# cg: the CG kernels as timed by the library (mode 3: the Gauss-compressed CG's histogram and "
                 "node solve groups; mode 2: the s-step passes, incl. a deferred solve's no-op margin passes).")
    lines.append("# rank ms/it = what one rank's GPU computes per outer iteration; one_device_wall_ms in the JSON below is")
    lines.append("# the single device running all W shards in turn (not a scaling number).")
    txt = "\n".join(lines)
    print(txt)
    print(json.dumps(rows))
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt + "\n" + json.dumps(rows) + "\n")


if __name__ == "__main__":
    main()
