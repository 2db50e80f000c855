#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch):
    python tools/pmc_sq_summary.py DIR [DIR ...]"""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("foto::", "")
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
for k in sorted(tot):
    c = {n: tot[k][n] / cnt[k][n] for n in tot[k]}
    w = c.get("SQ_WAVES", 0) or 1
    print(k)
    print("   " + "  ".join(f"{n.replace('SQ_', '')}={v:.4g}" for n, v in sorted(c.items())))
    print(f"   per wave: VALU {c.get('SQ_INSTS_VALU', 0) / w:.1f}  LDS {c.get('SQ_INSTS_LDS', 0) / w:.1f}  "
          f"VMEM_RD {c.get('SQ_INSTS_VMEM_RD', 0) / w:.1f}  SALU {c.get('SQ_INSTS_SALU', 0) / w:.1f}  "
          f"F64 FMA {c.get('SQ_INSTS_VALU_FMA_F64', 0) / w:.1f}")
