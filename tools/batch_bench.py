#!/usr/bin/env python3
"""C5-shaped batch measurement on synthetic data with known ground truth.

BASELINE config 5 is the whole Middlebury-2 other-data-gray batch streamed across GPUs with an
EPE + iters/s table (run.sh:81-157).  The Middlebury data is not in the image (no network), so
this builds a stand-in batch: textured frames at the Middlebury-2 sequence sizes, frame11 =
frame10 translated by a known sub-pixel (dx, dy), the ground truth written as flow10.flo.  The
real pipeline (run.py: the reference's GN and FOTO parameters, one worker per GPU) processes
it, and the table reports per sequence and algorithm the solve time, AEE / AAE against the
known flow (utils.EE / utils.AE) and IE, plus whole-batch sequences/s.

    python tools/batch_bench.py [--gpus N] [--seqs K] [--out DIR]
"""
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


def build(root, k):
    from PIL import Image
    import utils
    frames, gt = os.path.join(root, "frames"), os.path.join(root, "gt")
    for i, (name, w, h) in enumerate(SIZES[:k]):
        dx, dy = 0.6 + 0.25 * i, -0.4 + 0.2 * i
        a, b = make_pair(w, h, dx, dy, i)
        os.makedirs(os.path.join(frames, name), exist_ok=True)
        os.makedirs(os.path.join(gt, name), exist_ok=True)
        Image.fromarray(a, "L").save(os.path.join(frames, name, "frame10.png"))
        Image.fromarray(b, "L").save(os.path.join(frames, name, "frame11.png"))
        utils.saveFlo(w, h, np.full(w * h, dx), np.full(w * h, dy), os.path.join(gt, name, "flow10.flo"))
    return frames, gt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--seqs", type=int, default=len(SIZES))
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "batch"))
    ap.add_argument("--json", default=None, help="also write the summary line here")
    ap.add_argument("--cprofile", default=None, help="run run.py under cProfile, stats to this file")
    args = ap.parse_args()
    shutil.rmtree(args.out, ignore_errors=True)
    frames, gt = build(args.out, args.seqs)
    res = os.path.join(args.out, "results")
    t, t_wall = time.perf_counter(), time.time()
    run_args = ["run", f"--gpus={args.gpus}", f"--data={os.path.join(args.out, 'nodata')}", f"--results={res}",
                f"--dataset=synthetic={frames}:{gt}"]
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
    print(f"{'sequence':<12} {'algo':<5} {'time s':>7} {'AEE px':>8} {'AAE rad':>8} {'IE':>8}")
    for r in rows:
        print(f"{r['sequence']:<12} {r['algo']:<5} {r['time']:7.3f} {r.get('EE-mean', float('nan')):8.4f} "
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
    print(json.dumps(out))
    if args.json:
        with open(args.json, "w") as f:
            json.dump({**out, "rows": rows}, f)
    return rc


if __name__ == "__main__":
    sys.exit(main())
