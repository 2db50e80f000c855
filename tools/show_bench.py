#!/usr/bin/env python3
"""One line per bench JSON file: value, step time and the per-kernel HIP-event averages.
usage: tools/show_bench.py gpurun_out/b1.json [gpurun_out/b2.json ...]"""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f"{path}: unreadable ({e})")
        continue
    k = d.get("kernels", {})
    kern = " ".join(f"{a}={b['avg_us']:.1f}" for a, b in sorted(k.items()))
    roof = d.get("roofline") or {}
    print(f"{path}: {d['value']} it/s, {d['ms_per_step']} ms/step, cg {d.get('cg_iters_per_step')}, "
          f"redo {d.get('cg_redo')}, dom {roof.get('kernel')} {roof.get('avg_launch_us')} us frac {roof.get('frac')} | {kern}")
