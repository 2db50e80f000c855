#!/usr/bin/env python3
"""Per-position kernel times of the GN PCG iteration from a rocprofv3 kernel trace of
tools/gn_time.py: the dispatch sequence between two k_gnp_dir launches is one PCG iteration
(k_gnp_dir, k_gnp_upd, the V-cycle's down legs, coarse solve, up legs); prints the median
duration of each position and the median gap before it, over the iterations of the last solve.
usage: tools/gn_trace.py gpurun_out/<trace dir>"""
import csv, glob, sys
import numpy as np

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("foto::", "").replace("void ", "")
# iterations: runs starting at k_gnp_dir
its, cur = [], None
for a, r in zip([None] + rows[:-1], rows):
    n = name(r)
    if n.startswith("k_gnp_dir"):
        if cur: its.append(cur)
        cur = []
    if cur is not None:
        gap = (int(r["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 if a else 0.0
        cur.append((n, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, gap))
# keep the iterations of the most common length (full V-cycles) from the last 60
L = max(set(len(i) for i in its), key=lambda k: sum(1 for i in its if len(i) == k))
sel = [i for i in its if len(i) == L][-60:]
print(f"{len(sel)} PCG iterations of {L} launches")
tot, gtot = 0.0, 0.0
for p in range(L):
    d = np.median([i[p][1] for i in sel]); g = np.median([i[p][2] for i in sel])
    tot += d; gtot += g
    print(f"  {p:2d} {sel[0][p][0]:28s} {d:7.2f} us  (gap before {g:5.2f})")
span = np.median([sum(x[1] + x[2] for x in i) for i in sel])
print(f"  kernels {tot:.1f} us + gaps {gtot:.1f} us; median iteration span {span:.1f} us")
