#!/usr/bin/env python3
"""Print the bench value and the top kernels of tools/quick_prof.sh's outputs."""
import csv
import json

for ln in open("gpurun_out/bench3.log"):
    if ln.startswith("{"):
        d = json.loads(ln)
        print("value", d["value"], "it/s; roofline", d["roofline"]["kernel"], d["roofline"]["avg_launch_us"], "us")
rows = list(csv.DictReader(open("gpurun_out/prof_g3/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"{r['Name'][:70]:70s} n={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:9.2f}us")
