#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE / WRITE_SIZE PMC passes) into
profiles/<tag>_*.md / .json, and write profiles/pmc_traffic.json (HBM bytes per launch of
each hot kernel) that bench.py reports as roofline.traffic.

HBM bytes per launch = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes), following
MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE counts 64 B per 128-B request of a
coalesced streaming read (report = 1/2 of the bytes); WRITE_SIZE is exact for streaming
stores.  Our kernels read fp64 with 8-16 B per lane, fully coalesced.

usage: tools/summarize_profile.py --tag r01 --kt gpurun_out/prof_kt --fetch gpurun_out/prof_fetch \
          --write gpurun_out/prof_write [--bench gpurun_out/bench_full.log]
"""
import argparse
import collections
import csv
import json
import os

SHORT = {
    "k_cg_upd": "cg_upd", "k_cg_dir": "cg_dir", "k_prox": "prox", "k_rhs": "rhs", "k_spec": "spec_cg",
    "k_dct": "dct", "k_traj": "flow", "k_gn_pcg_dir": "gn_dir", "k_gn_pcg_upd": "gn_upd",
}


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return name.split("(")[0][:48]


def pmc(dirname, counter):
    agg = collections.defaultdict(list)
    path = os.path.join(dirname, "run_counter_collection.csv")
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}, {k: len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--bench")
    ap.add_argument("--out", default="profiles")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    rows = list(csv.DictReader(open(os.path.join(a.kt, "run_kernel_stats.csv"))))
    lines = [f"# rocprofv3 kernel stats ({a.tag})", "",
             "| kernel | calls | total ms | avg us | min us | max us | % |", "|---|---|---|---|---|---|---|"]
    stats = {}
    for r in rows:
        n = short(r["Name"])
        stats[n] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                    "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["Percentage"])}
        lines.append(f"| {n} | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.2f} | "
                     f"{float(r['AverageNs'])/1e3:.2f} | {float(r['MinNs'])/1e3:.2f} | "
                     f"{float(r['MaxNs'])/1e3:.2f} | {float(r['Percentage']):.2f} |")
    traffic = {}
    if a.fetch and a.write:
        f, nf = pmc(a.fetch, "FETCH_SIZE")
        w, nw = pmc(a.write, "WRITE_SIZE")
        lines += ["", "## HBM traffic per launch (PMC, separate passes)", "",
                  "| kernel | launches | FETCH_SIZE KiB | WRITE_SIZE KiB | HBM MB/launch (2F+W) |",
                  "|---|---|---|---|---|"]
        for k in sorted(set(f) & set(w)):
            hbm = (2 * f[k] + w[k]) * 1024.0
            traffic[k] = {"fetch_kib": f[k], "write_kib": w[k], "hbm_bytes_per_launch": hbm, "launches": nf[k]}
            lines.append(f"| {k} | {nf[k]} | {f[k]:.0f} | {w[k]:.0f} | {hbm/1e6:.1f} |")
    if a.bench and os.path.exists(a.bench):
        for ln in open(a.bench):
            if ln.startswith("{"):
                lines += ["", "## bench line", "", "```", ln.strip(), "```"]
    open(os.path.join(a.out, f"{a.tag}_rocprof_summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump({"kernel_stats": stats, "pmc": traffic}, open(os.path.join(a.out, f"{a.tag}_rocprof.json"), "w"),
              indent=1)
    if traffic:
        json.dump(traffic, open(os.path.join(a.out, "pmc_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
