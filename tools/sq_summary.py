#!/usr/bin/env python3
"""Per-kernel averages of SQ counters from one rocprofv3 --pmc run (counter_collection.csv).

    python3 tools/sq_summary.py DIR [kernel-substring ...]

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md); the
table prints each counter's per-launch average and, when SQ_WAVE_CYCLES is present, each
wait / active bucket as a fraction of it.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    keys = sys.argv[2:]
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value
    names = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if keys and not any(s in k for s in keys):
            continue
        key = (k, r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = 1
    agg = defaultdict(lambda: defaultdict(list))
    for (k, _), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
    for k in names:
        cs = agg[k]
        n = max(len(v) for v in cs.values())
        print(f"{k[:90]}  ({n} launches)")
        wc = sum(cs["SQ_WAVE_CYCLES"]) / n if "SQ_WAVE_CYCLES" in cs else None
        for c in sorted(cs):
            avg = sum(cs[c]) / len(cs[c])
            extra = f"  {avg / wc:6.3f} of WAVE_CYCLES" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print(f"    {c:28s} {avg:16.1f}{extra}")


if __name__ == "__main__":
    main()
