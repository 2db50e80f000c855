#!/usr/bin/env python3
"""k_prox_rhs launch durations from a rocprofv3 kernel trace of `bench.py` WITH its kernel-timing
pass: the first K launches are the timed loop (kernels back to back, no events between them),
the last K the timing pass (a HIP event pair around every launch) that the bench's roofline
uses.  Also the gap from each launch's predecessor.
usage: tools/prox_segments.py run_kernel_trace.csv STEPS WARMUP [loop_trace.json SOURCE]
With the last two arguments it also writes the loop / event averages as JSON (bench.py reads
profiles/prox_loop_trace.json for roofline.loop_trace)."""
import csv
import json
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
K, W = int(sys.argv[2]), int(sys.argv[3])
idx = [i for i, r in enumerate(rows) if "k_prox_rhs" in r["Kernel_Name"]]
dur = [(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e3 for i in idx]
gap = [(int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3 for i in idx]
# launches: warmup W, timed loop K, timing pass K (plus the first iteration's separate RHS)
n = len(dur)
seg = {"warmup": (0, W), "timed loop (no events)": (W, W + K), "timing pass (HIP events)": (n - K, n)}
print(f"k_prox_rhs launches: {n}")
for name, (a, b) in seg.items():
    d, g = dur[a:b], gap[a:b]
    if d:
        print(f"{name:26s}: {len(d)} launches, avg {sum(d) / len(d):7.2f} us (min {min(d):.2f}, max {max(d):.2f}), "
              f"avg gap from the previous kernel {sum(g) / len(g):6.2f} us")
if len(sys.argv) > 5:
    (la, lb), (ea, eb) = seg["timed loop (no events)"], seg["timing pass (HIP events)"]
    json.dump({"loop_avg_us": round(sum(dur[la:lb]) / max(1, lb - la), 2),
               "event_avg_us": round(sum(dur[ea:eb]) / max(1, eb - ea), 2), "source": sys.argv[5]},
              open(sys.argv[4], "w"))
