#!/usr/bin/env python3
"""C5-shaped batch measurement on synthetic data with known ground truth.

BASELINE config 5 is the whole Middlebury-2 other-data-gray batch streamed across GPUs with an
EPE + iters/s table (run.sh:81-157).  The Middlebury data is not in the image (no network), so
this builds a stand-in batch: textured frames at the Middlebury-2 sequence sizes, frame11 =
frame10 translated by a known sub-pixel (dx, dy), the ground truth written as flow10.flo.  The
real pipeline (run.py: the reference's GN and FOTO parameters, one worker per GPU) processes
it, and the table reports per sequence and algorithm the solve time, AEE / AAE against the
known flow (utils.EE / utils.AE) and IE, plus whole-batch sequences/s.

    python tools/batch_bench.py [--gpus N] [--devices 0,0] [--seqs K] [--out DIR] [--table T.md] [--reuse]

--gpus N starts N run.py workers; --devices maps them to GPUs (run.py --devices: "0,0" puts two
workers on GPU 0).  --table writes the config-5 table (markdown: per sequence and algorithm the
solve time, FOTO's outer iterations and iterations/s, AEE / AAE / IE).  --reuse runs again on
an existing --out (frames and results kept: run.sh's markers make it a no-op).
"""
import re
import argparse
import json
import os
import shutil
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "optical-flow-optimal-transport_amd")
sys.path.insert(0, PKG)

# Middlebury-2 other-data sequence sizes (README.md of the dataset; run.sh:81-157 walks them)
SIZES = [("Dimetrodon", 584, 388), ("Grove2", 640, 480), ("Venus", 420, 380), ("RubberWhale", 584, 388),
         ("Urban2", 640, 480), ("Hydrangea", 584, 388), ("Grove3", 640, 480), ("Urban3", 640, 480)]


def make_pair(w, h, dx, dy, seed):
    from scipy import ndimage
    rng = np.random.default_rng(seed)
    f = ndimage.gaussian_filter(rng.random((h, w)), 3.0)
    f = (f - f.min()) / (f.max() - f.min())
    g = ndimage.shift(f, (dy, dx), order=1, mode="nearest")   # g(x) = f(x - d): flow d
    return np.uint8(np.round(255 * f)), np.uint8(np.round(255 * g))


def sequences_list(k):
    """The first k stand-in sequences: the 8 Middlebury-2 sizes, then again with a suffix (a
    longer batch for steady-state throughput)."""
    return [(name if i < len(SIZES) else f"{name}_{i // len(SIZES)}", w, h)
            for i, (name, w, h) in ((i, SIZES[i % len(SIZES)]) for i in range(k))]


def build(root, k):
    from PIL import Image
    import utils
    frames, gt = os.path.join(root, "frames"), os.path.join(root, "gt")
    for i, (name, w, h) in enumerate(sequences_list(k)):
        dx, dy = 0.6 + 0.25 * i, -0.4 + 0.2 * i
        a, b = make_pair(w, h, dx, dy, i)
        os.makedirs(os.path.join(frames, name), exist_ok=True)
        os.makedirs(os.path.join(gt, name), exist_ok=True)
        Image.fromarray(a, "L").save(os.path.join(frames, name, "frame10.png"))
        Image.fromarray(b, "L").save(os.path.join(frames, name, "frame11.png"))
        utils.saveFlo(w, h, np.full(w * h, dx), np.full(w * h, dy), os.path.join(gt, name, "flow10.flo"))
    return frames, gt


def outer_iterations(log):
    """FOTO's outer iterations of a solve: its log holds one `crit (i/max_it)` line per
    iteration (benamou_brenier.py:252); None for GN (no such lines) or a missing log."""
    if not os.path.isfile(log):
        return None
    n = sum(1 for line in open(log) if re.search(r"\(\d+/\d+\)\s*$", line))
    return n or None


def write_table(path, rows, out):
    """The config-5 table (BASELINE configs[4]: EPE + iters/s per sequence) as markdown."""
    lines = [f"# C5 stand-in: {out['sequences']} sequences, {out['gpus']} worker(s)"
             + (f" on devices {out['devices']}" if out.get("devices") else " (one per GPU)"),
             "",
             f"{out['data']}; run.sh's parameters (GN alpha 0.1 lambda 0.2; FOTO r 1, tol 0.01, eps 1e-2, "
             f"Nt 16, max-it 200, stop rules on).  time = main.py's solver wall clock; AEE / AAE = utils.EE / "
             f"utils.AE against the known translation; IE = utils.IE of the reconstruction.",
             "",
             "| sequence | algo | time s | outer its | iters/s | AEE px | AAE rad | IE |",
             "|---|---|---|---|---|---|---|---|"]
    for r in rows:
        its = r["outer_its"]
        ips = r["iters_per_s"]
        lines.append(f"| {r['sequence']} | {r['algo']} | {r['time']:.3f} | {its if its else '-'} | "
                     f"{f'{ips:.1f}' if ips else '-'} | {r.get('EE-mean', float('nan')):.4f} | "
                     f"{r.get('AE-mean', float('nan')):.4f} | {r['IE']:.4f} |")
    fo = [r for r in rows if r["algo"] == "foto" and r["outer_its"]]
    lines += ["",
              f"Whole batch: {out['sequences']} sequences in {out['wall_s']} s wall ({out['sequences_per_s']} "
              f"sequences/s, interpreter start and HIP init included), slowest worker loop {out['loop_s']} s, "
              f"summed solver time {out['solve_s']} s; mean AEE GN {out['mean_AEE']['gn']:.4f} px, "
              f"FOTO {out['mean_AEE']['foto']:.4f} px"
              + (f"; FOTO {sum(r['outer_its'] for r in fo)} outer iterations in {sum(r['time'] for r in fo):.3f} s "
                 f"of FOTO solves ({sum(r['outer_its'] for r in fo) / sum(r['time'] for r in fo):.1f} iters/s "
                 f"including each solve's setup and flow extraction)." if fo else ".")]
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--seqs", type=int, default=len(SIZES))
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "batch"))
    ap.add_argument("--json", default=None, help="also write the summary line here")
    ap.add_argument("--cprofile", default=None, help="run run.py under cProfile, stats to this file")
    ap.add_argument("--devices", default=None, help="run.py --devices (worker i on device LIST[i mod len])")
    ap.add_argument("--table", default=None, help="write the config-5 EPE + iters/s table (markdown) here")
    ap.add_argument("--reuse", action="store_true", help="keep --out's frames and results (markers: a no-op run)")
    args = ap.parse_args()
    if args.reuse:
        frames, gt = os.path.join(args.out, "frames"), os.path.join(args.out, "gt")
    else:
        shutil.rmtree(args.out, ignore_errors=True)
        frames, gt = build(args.out, args.seqs)
    res = os.path.join(args.out, "results")
    if args.reuse:
        for f in os.listdir(res) if os.path.isdir(res) else []:
            if f.startswith(".worker"):
                os.remove(os.path.join(res, f))
    t, t_wall = time.perf_counter(), time.time()
    run_args = ["run", f"--gpus={args.gpus}", f"--data={os.path.join(args.out, 'nodata')}", f"--results={res}",
                f"--dataset=synthetic={frames}:{gt}"]
    if args.devices:
        run_args.append(f"--devices={args.devices}")
    if args.cprofile:
        # run.py's __main__ leaves through os._exit (no stats would be written): profile run.main in-process
        code = (f"import cProfile, sys; sys.path.insert(0, {PKG!r}); import run; "
                f"cProfile.run({'run.main(%r)' % run_args!r}, {args.cprofile!r})")
        cmd = [sys.executable, "-c", code]
    else:
        cmd = [sys.executable, os.path.join(PKG, "run.py"), *run_args]
    rc = subprocess.run(cmd).returncode
    wall, t_end = time.perf_counter() - t, time.time()
    rows = json.load(open(os.path.join(res, "summary.json")))
    for r in rows:   # FOTO's outer iterations: one stdout line per iteration in its log
        r["outer_its"] = outer_iterations(os.path.join(res, r["dataset"], r["sequence"], f"{r['algo']}.log"))
        r["iters_per_s"] = r["outer_its"] / r["time"] if r["outer_its"] and r["time"] > 0 else None
    print(f"{'sequence':<12} {'algo':<5} {'time s':>7} {'its':>5} {'it/s':>8} {'AEE px':>8} {'AAE rad':>8} {'IE':>8}")
    for r in rows:
        print(f"{r['sequence']:<12} {r['algo']:<5} {r['time']:7.3f} {r['outer_its'] or '':>5} "
              f"{r['iters_per_s'] or float('nan'):8.1f} {r.get('EE-mean', float('nan')):8.4f} "
              f"{r.get('AE-mean', float('nan')):8.4f} {r['IE']:8.4f}")
    solve_s = float(sum(r["time"] for r in rows))
    workers = [json.load(open(os.path.join(res, f))) for f in sorted(os.listdir(res)) if f.startswith(".worker")]
    loop_s = max((x["loop_s"] for x in workers), default=float("nan"))
    # solve_s: the solver wall clocks main.py prints (time), summed over every solve of every
    # worker; loop_s: the slowest worker's whole loop (frame IO, diff / rec / lum / colour PNGs,
    # errors, markers); wall_s: the run.py process tree, interpreter start and HIP init included
    out = {"sequences": args.seqs, "gpus": args.gpus, "wall_s": round(wall, 2), "rc": rc,
           "loop_s": round(loop_s, 3), "solve_s": round(solve_s, 3),
           # process start -> first worker loop, last worker loop end -> process tree exit
           "startup_s": round(min((x["t0_wall"] for x in workers), default=t_wall) - t_wall, 3),
           "teardown_s": round(t_end - max((x["t1_wall"] for x in workers), default=t_end), 3),
           "loop_over_solve": round(loop_s * args.gpus / solve_s, 3) if solve_s else None,
           "wall_over_solve": round(wall * args.gpus / solve_s, 3) if solve_s else None,
           "sequences_per_s": round(args.seqs / wall, 3),
           "mean_AEE": {a: float(np.mean([r["EE-mean"] for r in rows if r["algo"] == a])) for a in ("gn", "foto")},
           "data": "synthetic translations at Middlebury-2 sizes (no Middlebury offline)"}
    out["devices"] = args.devices
    print(json.dumps(out))
    if args.table:
        write_table(args.table, rows, out)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({**out, "rows": rows}, f)
    return rc


if __name__ == "__main__":
    sys.exit(main())
