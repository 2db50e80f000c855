#!/usr/bin/env python3
"""Compute-only proxy of the multi-GPU strong-scaling curve (communication excluded).

A grid (default the 640x480x32 bench problem; --grid c4: BASELINE config 4, 1024x1024x64) is
split into W time slabs / row boxes exactly as W RCCL ranks would split it, but as W in-process shards on ONE device (virtual ranks: the same kernels,
the same transfer lists, executed as device copies).  Every kernel launch of a shard is that
rank's work on a whole GPU, so the per-launch HIP-event times (foto_bb_set_timing) summed
over one shard are what one rank of a W-GPU run computes per outer iteration.  The device
copies standing in for RCCL are not kernels and are not counted: communication (halo and
moment all-gathers, the slab <-> row-box all-to-alls, RCCL launch latency) is EXCLUDED, so
the curve is an upper bound on what W GPUs can reach.

A communication MODEL is printed beside it (not a measurement: the RCCL calls have only run
through the in-process transport): per rank and outer iteration the slab <-> row-box
all-to-alls (each rank sends (W-1)/W of its slab each way, one peer per xGMI link), the
one-plane phi and w_t halos of the fused prox + RHS with deferred slab edges (both
neighbours; FOTO_PR_EDGE=0's recompute would send 2 phi + 3 mu planes), the 32-KB
histogram all-gather and the crit all-gather, at LINK_GBS per direction per link and
LAT_US per RCCL call.

    python tools/proxy_scaling.py [--grid 640,480,32 | c4] [--worlds 1,2,4,8] [--steps 10] [--warmup 3] [--out FILE]
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
LINK_GBS = 64.0   # xGMI, effective GB/s per direction of one link (7 links x ~153 GB/s per GPU, both directions)
LAT_US = 10.0     # per RCCL call (grouped send / recv or all-gather) at these message sizes


def comm_model_us(W):
    """Modelled communication per rank per outer iteration (see the docstring)."""
    if W == 1:
        return 0.0, {}
    nl = -(-NT // W)                          # the largest slab
    plane = NX * NY * 8
    a2a = nl * plane * (W - 1) / W            # bytes one rank sends in one all-to-all
    # W - 1 peers over 7 links (8 GPUs fully connected): a2a spread over min(W - 1, 7) links
    a2a_us = a2a / min(W - 1, 7) / (LINK_GBS * 1e3) + LAT_US
    halo_us = 2 * plane / (LINK_GBS * 1e3) + 2 * LAT_US       # per neighbour: phi, then w_t, one plane each
    gath_us = 2 * LAT_US                                      # histogram (32 KB) + crit all-gathers
    parts = {"alltoall_x2": 2 * a2a_us, "halos": halo_us, "allgathers": gath_us}
    return sum(parts.values()), parts


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
    ap.add_argument("--grid", default="640,480,32", help="Nx,Ny,Nt or c4 (1024,1024,64)")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    global NX, NY, NT
    NX, NY, NT = (1024, 1024, 64) if args.grid == "c4" else (int(v) for v in args.grid.split(","))
    rows = [measure(int(w), args.steps, args.warmup) for w in args.worlds.split(",")]
    base = rows[0]["rank_ms"] * rows[0]["W"]
    lines = [f"# compute-only proxy, {NX}x{NY}x{NT}, r={R}, eps={EPS}: per-rank kernel time of W virtual shards on one",
             "# MI355X (HIP events around every launch); COMMUNICATION EXCLUDED (halo / moment all-gathers,",
             "# slab<->box all-to-alls and RCCL latency are not counted) -> an upper bound for W GPUs.",
             f"# {'W':>2} {'rank ms/it':>10} {'proxy it/s':>10} {'eff':>5} {'CG its':>6} {'cg launches':>13} "
             f"{'cg ms':>8} {'dct ms':>7} {'prox+rhs ms':>11} {'flow/other':>10} {'comm model ms':>13} "
             f"{'model it/s':>10} {'model eff':>9}"]
    for r in rows:
        k = r["kernels_ms"]
        eff = base / (r["W"] * r["rank_ms"])
        cm, parts = comm_model_us(r["W"])
        r["comm_model_us"] = {"total": cm, **parts}
        model_ms = r["rank_ms"] + cm / 1e3
        lines.append(f"  {r['W']:>2} {r['rank_ms']:10.3f} {1e3 / r['rank_ms']:10.1f} {eff:5.2f} {r['cg_its']:6.1f} "
                     f"{r['launches'].get('spec_cg', 0):13.1f} {k.get('spec_cg', 0):8.3f} {k.get('dct', 0):7.3f} "
                     f"{k.get('prox', 0) + k.get('rhs', 0):11.3f} {k.get('flow', 0) + k.get('other', 0):10.3f} "
                     f"{cm / 1e3:13.3f} {1e3 / model_ms:10.1f} {base / (r['W'] * model_ms):9.2f}")
    lines.append(f"# comm model: all-to-all bytes (W-1)/W of the rank's slab each way over min(W-1, 7) xGMI links, "
                 f"halos 2 planes per neighbour (phi, w_t), {LINK_GBS:.0f} GB/s per link direction, {LAT_US:.0f} us per RCCL call "
                 f"(a model, not a measurement; no overlap with compute assumed).")
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
