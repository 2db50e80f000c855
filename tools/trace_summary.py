#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace CSV, with the gaps between
consecutive dispatches.  usage: tools/trace_summary.py gpurun_out/trace_<name> [...]"""
import csv, glob, sys, collections
import numpy as np

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("foto::", "")
        by[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"== {d}: {len(rows)} dispatches, span {(int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp']))/1e3:.0f} us")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v = np.array(v)
        print(f"  {n:28s} n={len(v):4d} total={v.sum():9.1f} us  mean={v.mean():7.2f}  p10={np.percentile(v,10):7.2f} "
              f"p50={np.median(v):7.2f} p90={np.percentile(v,90):7.2f}")
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
    g = np.array(gaps)
    print(f"  gaps: total {g.sum():.0f} us, median {np.median(g):.2f}, >20us: {int((g > 20).sum())} totalling {g[g > 20].sum():.0f} us")
    # gaps by (previous kernel -> next kernel), the most frequent pairs
    pairs = collections.defaultdict(list)
    short = lambda r: r["Kernel_Name"].split("(")[0].split("<")[0].replace("foto::", "").replace("void ", "")
    for a, b, gp in zip(rows, rows[1:], gaps):
        pairs[(short(a), short(b))].append(gp)
    for (a, b), v in sorted(pairs.items(), key=lambda kv: -len(kv[1]))[:8]:
        v = np.array(v)
        print(f"  gap {a} -> {b}: n={len(v)} median {np.median(v):.2f} us, p10 {np.percentile(v,10):.2f}, p90 {np.percentile(v,90):.2f}")
