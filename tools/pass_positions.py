#!/usr/bin/env python3
"""Durations of the s-step CG passes (k_spec_s2r) by their position inside each solve, from a
rocprofv3 --kernel-trace CSV.  A solve is a run of consecutive pass dispatches (anything else
-- DCTs, prox -- ends it).  Launches under 25 % of the median are the deferred solve's no-op
margin passes.

usage: tools/pass_positions.py gpurun_out/prof_kt [more dirs]"""
import collections
import csv
import glob
import sys

import numpy as np

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    solves, cur = [], []
    for r in rows:
        name = r["Kernel_Name"]
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_spec_s2r" in name:
            cur.append(dur)
        else:
            if cur:
                solves.append(cur)
            cur = []
    if cur:
        solves.append(cur)
    allp = np.concatenate([np.array(s) for s in solves]) if solves else np.array([])
    med = np.median(allp)
    work = [[x for x in s if x >= 0.25 * med] for s in solves]
    noop = sum(len(s) - len(w) for s, w in zip(solves, work))
    print(f"== {d}: {len(solves)} solves, {len(allp)} pass launches ({noop} no-op, {np.mean([len(w) for w in work]):.1f} "
          f"working per solve), working mean {np.mean(np.concatenate(work)):.2f} us")
    bypos = collections.defaultdict(list)
    for w in work:
        for i, x in enumerate(w):
            bypos[i].append(x)
        if w:
            bypos["last"].append(w[-1])
    for k in list(range(0, 30)) + ["last"]:
        if k in bypos:
            v = np.array(bypos[k])
            print(f"  pass {k!s:>4}: n={len(v):3d} mean {v.mean():7.2f} us  min {v.min():7.2f}  max {v.max():7.2f}")
