#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + FETCH_SIZE / WRITE_SIZE PMC passes) into
profiles/<tag>_*.md / .json, and write profiles/pmc_traffic.json (HBM bytes per launch of
each hot kernel) that bench.py reports as roofline.traffic.

HBM bytes per launch = f_load * FETCH_SIZE + f_store * WRITE_SIZE (KiB -> bytes).  The
correction factors come from a calibration run of tools/calib_fetch (known byte counts,
2 GiB streams far beyond the Infinity Cache) under the same two PMC passes.  Measured
(profiles/r01c_*): FETCH_SIZE reports 1/2 of the bytes of a streaming read for 8-B and
16-B loads per lane alike (MI355X_MICROARCH.md HBM section states it for 16 B); WRITE_SIZE
is exact.  Each kernel's factor follows the load width it uses (LOAD_WIDTH below).

usage: tools/summarize_profile.py --tag r01 --kt gpurun_out/prof_kt --fetch gpurun_out/prof_fetch \
          --write gpurun_out/prof_write --calib-fetch gpurun_out/cal_fetch --calib-write gpurun_out/cal_write \
          [--bench gpurun_out/bench_full.log]
"""
import argparse
import collections
import csv
import glob
import json
import os

SHORT = {
    # first match wins: the specific names before their prefixes
    "k_cg_upd": "cg_upd", "k_cg_dir": "cg_dir", "k_prox_rhs": "prox", "k_prox": "prox_sep", "k_rhs": "rhs",
    "k_gq_hist": "gq_hist", "k_gq_reduce": "gq_reduce", "k_gq_perm_reduce": "gq_reduce",
    "k_gq_perm_count": "gq_setup", "k_gq_perm_fill": "gq_setup", "k_gq_perm_scan": "gq_setup",
    "k_gq_exact": "gq_setup", "k_gq_rowmu": "gq_setup", "k_gq_bins": "gq_setup", "k_gq_nodes": "gq_nodes", "k_gq_cgtab": "gq_cg", "k_gq_cg": "gq_cg",
    "k_gq_qtab": "gq_qtab", "k_gq_xhat": "gq_xhat", "k_dct_t_inv_q": "dct_t_q", "k_dct_tp_inv_q": "dct_tp_q",
    "k_dct_tp_fwd_init": "dct_tp_init", "k_dct_tp_inv_xhat": "dct_tp_xhat",
    "k_spec_s2_plan": "spec_plan", "k_spec_s2": "spec_cg", "k_spec_init": "spec_init", "k_spec_xhat": "spec_xhat",
    "k_spec_cg": "spec_cg1", "k_dct_fft_fwd": "dct_fft_fwd", "k_dct_fft_inv": "dct_fft_inv",
    "k_dct_t_fwd_init": "dct_t_init", "k_dct_t_inv_xhat": "dct_t_xhat", "k_dct": "dct_gemm", "k_traj": "flow",
    "k_gn_pcg_dir": "gn_dir", "k_gn_pcg_upd": "gn_upd",
}


# bytes per lane of each hot kernel's streaming loads (csrc/*.hip)
LOAD_WIDTH = {"spec_cg": 16, "spec_cg1": 16, "spec_init": 16, "spec_xhat": 16, "cg_upd": 8, "cg_dir": 8, "prox": 8,
              "prox_sep": 8, "gq_hist": 16, "dct_t_q": 8, "dct_tp_q": 8, "dct_tp_init": 8, "dct_tp_xhat": 8,
              "rhs": 8, "dct_fft_fwd": 8, "dct_fft_inv": 8, "dct_t_init": 8, "dct_t_xhat": 8, "dct_gemm": 8, "flow": 8,
              "gn_dir": 8, "gn_upd": 8}
# kernels of one outer iteration of the default path (profiles' "_step" traffic)
STEP_KERNELS = {"dct_fft_fwd", "dct_fft_inv", "dct_t_init", "dct_t_xhat", "dct_tp_init", "dct_tp_xhat", "dct_gemm",
                "gq_hist", "gq_reduce", "gq_nodes", "gq_cg", "gq_qtab", "gq_xhat", "prox"}
CALIB_BYTES = {"rd8": 2 << 30, "rd16": 2 << 30, "wr8": 1 << 30, "wr16": 1 << 30}


def find_csv(dirname, suffix):
    hits = sorted(glob.glob(os.path.join(dirname, "**", "*" + suffix), recursive=True))
    if not hits:
        raise FileNotFoundError(f"no *{suffix} under {dirname}")
    return hits[0]


def short(name):
    for k, v in SHORT.items():
        if k in name:
            return v
    return name.split("(")[0][:48]


def pmc(dirname, counter):
    """Mean counter value per launch of each kernel.  Launches below 1 % of that kernel's
    median are no-ops (s-step passes launched past the end of a solve exit at once) and are
    left out, so the figure describes a working launch."""
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(find_csv(dirname, "counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            agg[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    out, cnt = {}, {}
    for k, v in agg.items():
        med = sorted(v)[len(v) // 2]
        w = [x for x in v if x >= 0.01 * med] or v
        out[k], cnt[k] = sum(w) / len(w), len(w)
    return out, cnt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--kt", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("--bench")
    ap.add_argument("--out", default="profiles")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    rows = list(csv.DictReader(open(find_csv(a.kt, "kernel_stats.csv"))))
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
    # Working launches from the kernel trace: s-step passes launched past the end of a solve
    # exit at once, and the pass whose plan finds the solve done only joins the ticket; launches
    # under a quarter of the kernel's median are left out (bench.py's HIP-event timing drops
    # the same launches), so "work avg" is comparable with the bench line's avg_launch_us.
    tr = collections.defaultdict(list)
    for r in csv.DictReader(open(find_csv(a.kt, "kernel_trace.csv"))):
        tr[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    lines += ["", "## working launches (kernel trace; launches < 25 % of the median left out)", "",
              "| kernel | working calls | work avg us | other calls | other avg us |", "|---|---|---|---|---|"]
    for n, v in sorted(tr.items(), key=lambda t: -sum(t[1])):
        med = sorted(v)[len(v) // 2]
        wk = [x for x in v if x >= 0.25 * med]
        ot = [x for x in v if x < 0.25 * med]
        stats.setdefault(n, {})["work_avg_us"] = sum(wk) / len(wk)
        stats[n]["work_calls"] = len(wk)
        lines.append(f"| {n} | {len(wk)} | {sum(wk) / len(wk):.2f} | {len(ot)} | "
                     f"{(sum(ot) / len(ot)) if ot else 0.0:.2f} |")
    traffic = {}
    fac_ld, fac_st = {8: 1.0, 16: 2.0}, 1.0   # defaults (guide); replaced by the calibration
    if a.calib_fetch and a.calib_write:
        cf, _ = pmc(a.calib_fetch, "FETCH_SIZE")
        cw, _ = pmc(a.calib_write, "WRITE_SIZE")
        fac_ld = {8: CALIB_BYTES["rd8"] / (cf["rd8"] * 1024.0), 16: CALIB_BYTES["rd16"] / (cf["rd16"] * 1024.0)}
        fac_st = 0.5 * (CALIB_BYTES["wr8"] / (cw["wr8"] * 1024.0) + CALIB_BYTES["wr16"] / (cw["wr16"] * 1024.0))
        lines += ["", "## PMC calibration (tools/calib_fetch, 2 GiB streams)", "",
                  "| access | bytes | counter KiB | bytes / counter byte |", "|---|---|---|---|"]
        for k in ("rd8", "rd16"):
            lines.append(f"| {k} | {CALIB_BYTES[k]} | {cf[k]:.0f} | {CALIB_BYTES[k] / (cf[k] * 1024.0):.3f} |")
        for k in ("wr8", "wr16"):
            lines.append(f"| {k} | {CALIB_BYTES[k]} | {cw[k]:.0f} | {CALIB_BYTES[k] / (cw[k] * 1024.0):.3f} |")
    if a.fetch and a.write:
        f, nf = pmc(a.fetch, "FETCH_SIZE")
        w, nw = pmc(a.write, "WRITE_SIZE")
        lines += ["", "## HBM traffic per launch (PMC, separate passes, calibrated per load width)", "",
                  "| kernel | launches | FETCH_SIZE KiB | WRITE_SIZE KiB | load B/lane | HBM MB/launch |",
                  "|---|---|---|---|---|---|"]
        for k in sorted(set(f) & set(w)):
            lw = LOAD_WIDTH.get(k, 8)
            hbm = (fac_ld[lw] * f[k] + fac_st * w[k]) * 1024.0
            traffic[k] = {"fetch_kib": f[k], "write_kib": w[k], "load_width": lw, "fetch_factor": fac_ld[lw],
                          "store_factor": fac_st, "hbm_bytes_per_launch": hbm, "launches": nf[k]}
            lines.append(f"| {k} | {nf[k]} | {f[k]:.0f} | {w[k]:.0f} | {lw} | {hbm/1e6:.1f} |")
    if a.bench and os.path.exists(a.bench):
        for ln in open(a.bench):
            if ln.startswith("{"):
                lines += ["", "## bench line", "", "```", ln.strip(), "```"]
    open(os.path.join(a.out, f"{a.tag}_rocprof_summary.md"), "w").write("\n".join(lines) + "\n")
    json.dump({"kernel_stats": stats, "pmc": traffic}, open(os.path.join(a.out, f"{a.tag}_rocprof.json"), "w"),
              indent=1)
    if traffic:
        # "_source": the profile these per-launch bytes come from (bench.py quotes it as
        # roofline.traffic_source: the traffic is measured by rocprofv3 PMC passes, not in the
        # bench run itself)
        src = {"_source": f"profiles/{a.tag}_rocprof_summary.md (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, "
                          f"calibrated by tools/calib_fetch)"}
        out = {**src, **traffic}
        # the whole outer iteration (mode 3, one GPU): every kernel launched per outer iteration,
        # summed over the profiled run and divided by the outer iterations (one prox each)
        step_k = [k for k in traffic if k in STEP_KERNELS]
        if "prox" in traffic and traffic["prox"]["launches"] > 0:
            n_outer = traffic["prox"]["launches"]
            tot = sum(traffic[k]["hbm_bytes_per_launch"] * traffic[k]["launches"] for k in step_k)
            out["_step"] = {"hbm_bytes_per_step": tot / n_outer, "outer_iterations": n_outer, "kernels": step_k,
                            "source": src["_source"]}
            lines += ["", f"## HBM traffic per outer iteration: {tot / n_outer / 1e6:.1f} MB "
                          f"({n_outer} outer iterations; kernels {', '.join(step_k)})"]
            open(os.path.join(a.out, f"{a.tag}_rocprof_summary.md"), "w").write("\n".join(lines) + "\n")
        json.dump(out, open(os.path.join(a.out, "pmc_traffic.json"), "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
