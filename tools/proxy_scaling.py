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
through the in-process transport).  Per rank and outer iteration (round 5 structure,
foto_bb.cpp sharded_fwd / sharded_inv / prox_rhs):
  * the slab -> box all-to-all, (W-1)/W of the rank's slab, one peer per xGMI link over
    min(W-1, 7) links, in PARTS groups on the communication stream, each sent while the compute
    stream runs the next part's x / y DCTs (dct_slab, measured per rank): a two-stage pipeline
    of PARTS equal parts takes C/P + (P-1) max(C, M)/P + M/P for compute C and transfer M;
  * the box -> slab all-to-all likewise, carrying phi's halo planes (one per side) as well, so
    the inverse x / y DCTs run on nloc + 2 planes (their extra compute is added);
  * the w_t halo of the deferred slab edges: one plane with each neighbour (both at once),
    issued before k_prox_rhs (k_wt_pre) so that only what outlasts the measured prox time is
    exposed (FOTO_WT_OVERLAP=0: all of it; the virtual shards run k_wt_pre, FOTO_WT_PRE=1);
  * the 32-KB histogram all-gather and the crit all-gather;
at LINK_GBS per direction per link and LAT_US per RCCL call.  --no-overlap prints round 4's
model (phi halo a separate plane per neighbour, nothing overlapped) for comparison.

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


def a2a_setup():
    """foto_bb.cpp a2a_parts / a2a_halo defaults (and their environment overrides): two parts and
    phi's halo inside the backward all-to-all for planes of >= 2^19 voxels, else one part and the
    separate halo plane."""
    big = NX * NY >= (1 << 19)
    parts = int(os.environ.get("FOTO_A2A_PARTS", "2" if big else "1"))
    halo = int(os.environ.get("FOTO_A2A_HALO", "1" if big else "0"))
    return max(1, min(8, parts)), halo


def wt_overlap_on(W):
    """foto_bb.cpp wt_overlap: every slab of >= 3 planes, FOTO_WT_OVERLAP not 0."""
    return NT // W >= 3 and os.environ.get("FOTO_WT_OVERLAP", "1") != "0"


def pipe_us(c_us, m_us, parts):
    """A two-stage pipeline (compute then transfer, or transfer then compute) of `parts` equal
    parts: the time beyond the compute alone."""
    p = max(1, parts)
    return c_us / p + (p - 1) * max(c_us, m_us) / p + m_us / p - c_us


def comm_model_us(W, slab_ms=0.0, overlap=True, prox_ms=0.0):
    """Modelled communication time per rank per outer iteration that the compute does not hide
    (see the docstring).  slab_ms: the rank's measured slab-side x / y DCT time (both directions);
    prox_ms: its measured k_wt_pre + k_prox_rhs time (the w_t exchange travels behind it)."""
    if W == 1:
        return 0.0, {}
    nl = -(-NT // W)                          # the largest slab
    plane = NX * NY * 8
    links = min(W - 1, 7)
    bw = LINK_GBS * 1e3                       # bytes per us
    a2a = nl * plane * (W - 1) / W / links / bw
    if not overlap:                           # round 4: no overlap, phi halo its own plane
        parts = {"alltoall_x2": 2 * (a2a + LAT_US), "halos": 2 * (plane / bw + LAT_US), "allgathers": 2 * LAT_US}
        return sum(parts.values()), parts
    P, halo = a2a_setup()
    c = 1e3 * slab_ms / 2                     # x / y DCTs of one direction (measured: incl. the halo
    #                                           planes' inverse DCTs when they are delivered)
    a2a_i = (nl + 2 * halo) * plane * (W - 1) / W / links / bw   # + phi's two halo planes
    # w_t (foto_bb.cpp wt_overlap, slabs of >= 3 planes, FOTO_WT_OVERLAP=0: off) travels while
    # k_prox_rhs runs (the crit all-gather behind it on the communication stream is joined next)
    wt = plane / bw + LAT_US
    if wt_overlap_on(W):
        wt = max(0.0, wt - 1e3 * prox_ms)
    parts = {"alltoall_fwd": pipe_us(c, a2a, P) + P * LAT_US,
             "alltoall_inv": pipe_us(c, a2a_i, P) + P * LAT_US,
             "halo_phi": 0.0 if halo else plane / bw + LAT_US,
             "halo_wt": wt,
             "allgathers": 2 * LAT_US}
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
    ap.add_argument("--no-overlap", action="store_true", help="round 4's communication model")
    args = ap.parse_args()
    global NX, NY, NT
    NX, NY, NT = (1024, 1024, 64) if args.grid == "c4" else (int(v) for v in args.grid.split(","))
    if not args.no_overlap and os.environ.get("FOTO_WT_OVERLAP", "1") != "0":
        os.environ["FOTO_WT_PRE"] = "1"   # the virtual shards run k_wt_pre as the RCCL ranks would
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
        cm, parts = comm_model_us(r["W"], k.get("dct_slab", 0.0), overlap=not args.no_overlap,
                                  prox_ms=k.get("prox", 0.0))
        r["comm_model_us"] = {"total": cm, **parts}
        model_ms = r["rank_ms"] + cm / 1e3
        lines.append(f"  {r['W']:>2} {r['rank_ms']:10.3f} {1e3 / r['rank_ms']:10.1f} {eff:5.2f} {r['cg_its']:6.1f} "
                     f"{r['launches'].get('spec_cg', 0):13.1f} {k.get('spec_cg', 0):8.3f} {k.get('dct', 0) + k.get('dct_slab', 0):7.3f} "
                     f"{k.get('prox', 0) + k.get('rhs', 0):11.3f} {k.get('flow', 0):10.3f} "
                     f"{cm / 1e3:13.3f} {1e3 / model_ms:10.1f} {base / (r['W'] * model_ms):9.2f}")
    if args.no_overlap:
        lines.append(f"# comm model (round 4): all-to-all bytes (W-1)/W of the rank's slab each way over min(W-1, 7) xGMI "
                     f"links, halos 2 planes per neighbour (phi, w_t), {LINK_GBS:.0f} GB/s per link direction, "
                     f"{LAT_US:.0f} us per RCCL call, no overlap (a model, not a measurement).")
    else:
        P, halo = a2a_setup()
        lines.append(f"# comm model (round 5): the all-to-alls in {P} part(s) on the communication stream, pipelined "
                     f"against the slab-side x / y DCTs (dct_slab, measured), phi's halo planes "
                     f"{'inside the backward all-to-all (their inverse DCT is in the measured compute)' if halo else 'as one plane per neighbour'}, "
                     f"w_t one plane per neighbour{' behind k_prox_rhs (k_wt_pre in the measured prox)' if wt_overlap_on(2) else ''}, {LINK_GBS:.0f} GB/s per link direction, {LAT_US:.0f} us per RCCL call "
                     f"(a model, not a measurement).")
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
