#!/usr/bin/env python3
"""FOTO hot-path benchmark: Benamou-Brenier outer iterations/s on the 640x480x32 grid.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cg-mode 0|1|2] [--no-cpu-baseline] [--no-gn]

A "step" is one outer iteration of benamou_brenier.solve (benamou_brenier.py:204-258:
RHS + CG Poisson solve + stepB/stepC + criterion) over the synthetic 640x480x32
translating-Gaussian pair (SURVEY.md §8(d) S-metric; r = 1, eps = 1e-2, run.sh:114
parameters), with every input and all solver state resident in HBM.  The stop rules are
disabled so exactly K steps run.  With N > 1 (torch.distributed.run, one process per GPU)
the time axis is sharded into N slabs with RCCL halo exchange (strong scaling: the same
problem on more GPUs); value = outer iterations of that one problem per second.

At N = 1 the line also carries a "gn" object: the GN baseline (classical.py)
solved on the GPU at 640x480 and 320x240, and the oracle's SuperLU solve of the 320x240 pair on
one host core beside it.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "optical-flow-optimal-transport_amd"))

import numpy as np  # noqa: E402

NX, NY, NT = 640, 480, 32
R, EPS = 1.0, 1e-2
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s (spec)
METRIC = "BB solver iters/sec on 640×480×32 grid"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cg-mode", type=int, default=int(os.environ.get("FOTO_CG_MODE", "2")),
                    help="0 stencil CG, 1 spectral CG (one GPU), 2 spectral s-step CG (default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gn", action="store_true", help="skip the GN (classical.py, config 3) side measurement")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--gn-cpu-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-launch HIP-event pass (roofline fields become null)")
    return ap.parse_args()


def cpu_baseline():
    """The oracle (numpy/scipy restatement, CSR SpMV + scipy-recurrence CG + vectorised
    stepB) timed on the first outer iteration of the same workload.  Run in a child
    process pinned to one BLAS/OpenMP thread (the reference path is single-core)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-only"], env=env,
                         capture_output=True, text=True, timeout=900)
    if out.returncode != 0:
        raise RuntimeError("cpu baseline failed: " + out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def cpu_baseline_child():
    sys.path.insert(0, REPO)
    from oracle import foto_oracle as O
    from foto.synthetic import translating_gaussian
    rho0, rhoT = translating_gaussian(NX, NY)
    t0 = time.perf_counter()
    A = O.assemble_A(R, EPS, NT, NY, NX)   # once per solve, outside the loop (like the GPU context)
    total = time.perf_counter() - t0
    N = NT * NX * NY
    mu = np.zeros(3 * N)
    for n in range(NT):
        mu[n * NX * NY:(n + 1) * NX * NY] = (1 - n / (NT - 1)) * rho0 + (n / (NT - 1)) * rhoT
    t1 = time.perf_counter()
    phi, info, its = O.solve_step(mu, np.zeros(3 * N), rho0, rhoT, R, A.dot, NT, NY, NX)
    g = O.grad_st(phi, NT, NY, NX)
    q = O.stepB(g + (1.0 / R) * mu, N)
    mu = mu + R * (g - q)
    mu[:N] = np.maximum(mu[:N], 0)
    loop = time.perf_counter() - t1
    print(json.dumps({"loop_s": loop, "assemble_s": total, "cg_its": int(its)}))


GN_W, GN_H, GN_ALPHA, GN_LAMBDA = 640, 480, 0.1, 0.2   # config 3 size, run.sh:103 parameters
GN_CPU_W, GN_CPU_H = 320, 240                          # bounded CPU sample (spsolve ~13 s here)


def gn_cpu_child():
    """The oracle's GN solve (classical.py:113-130: SuperLU spsolve) on the CPU sample pair."""
    sys.path.insert(0, REPO)
    from oracle import foto_oracle as O
    from foto.synthetic import sinusoid_pair
    f1, f2 = sinusoid_pair(GN_CPU_W, GN_CPU_H)
    t = time.perf_counter()
    O.gn_solve(f1, f2, GN_CPU_W, GN_CPU_H, GN_ALPHA, GN_LAMBDA)
    print(json.dumps({"solve_s": time.perf_counter() - t}))


def gn_side(with_cpu):
    """GN baseline (SURVEY.md §8(d) config 3 stand-in: sinusoid pair, alpha 0.1, lambda 0.2):
    GPU PCG solve time at 640x480 and at the CPU sample size, the oracle's spsolve beside it."""
    from foto import gn
    from foto.synthetic import sinusoid_pair
    out = {"workload": f"GN classical solve, sinusoid pair, alpha={GN_ALPHA}, lambda={GN_LAMBDA}, "
                       f"CG preconditioned by a symmetric multigrid V-cycle (FOTO_GN_MG=0: block-Jacobi) to rtol {gn.GN_RTOL}"}
    for (w, h) in ((GN_W, GN_H), (GN_CPU_W, GN_CPU_H)):
        f1, f2 = sinusoid_pair(w, h)
        best = None
        for _ in range(2):
            t = time.perf_counter()
            _, _, _, info, its = gn.solve(f1, f2, w, h, GN_ALPHA, GN_LAMBDA)
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        out[f"gpu_{w}x{h}"] = {"solve_ms": round(1e3 * best, 2), "pcg_its": its, "info": info}
    if with_cpu:
        env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
        res = subprocess.run([sys.executable, os.path.abspath(__file__), "--gn-cpu-only"], env=env,
                             capture_output=True, text=True, timeout=600)
        if res.returncode == 0:
            cpu_s = json.loads(res.stdout.strip().splitlines()[-1])["solve_s"]
            gpu_s = out[f"gpu_{GN_CPU_W}x{GN_CPU_H}"]["solve_ms"] / 1e3
            out["cpu_baseline"] = {"value_s": round(cpu_s, 3), "kind": "port", "cores": 1,
                                   "sample": f"oracle spsolve (SuperLU, classical.py:113-130) on the "
                                             f"{GN_CPU_W}x{GN_CPU_H} pair"}
            out["speedup_vs_cpu"] = round(cpu_s / gpu_s, 1)
    return out


def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline_child()
        return
    if args.gn_cpu_only:
        gn_cpu_child()
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = None
    nccl_id = None
    if world > 1:
        import torch.distributed as dist   # rendezvous / barrier / timing reduction only (gloo, CPU)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import foto
        obj = [None]
        if rank == 0:
            import ctypes
            buf = ctypes.create_string_buffer(128)
            foto._lib.check(foto.lib().foto_nccl_unique_id(buf))
            obj = [bytes(buf.raw)]
        dist.broadcast_object_list(obj, src=0)
        nccl_id = obj[0]

    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian

    rho0, rhoT = translating_gaussian(NX, NY)
    s = BBSolver(rho0, rhoT, NT, NX, NY, r=R, reg_epsilon=EPS, device=local_rank, cg_mode=args.cg_mode,
                 rank=rank, world=world, nccl_id=nccl_id)

    def barrier():
        s.sync()
        if dist is not None:
            dist.barrier()

    # warmup (untimed)
    s.iterate(args.warmup, 0.0, stop_rules=False)
    barrier()
    s.reset_stats()
    its_before = len(s.cg_its)
    t0 = time.perf_counter()
    s.iterate(args.steps, 0.0, stop_rules=False)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    cg_steps = s.cg_its[its_before:]
    st_timed = s.stats()

    # per-launch kernel timing pass: K more steps with a HIP event pair around every launch
    roof = None
    kern = {}
    if not args.no_kernel_timing:
        s.reset_stats()
        s.set_timing(True)
        s.iterate(args.steps, 0.0, stop_rules=False)
        barrier()
        s.set_timing(False)
        kst = s.stats()["kernels"]
        for name, k in kst.items():
            kern[name] = {"launches": k["n"], "avg_us": 1e3 * k["ms"] / max(k["n"], 1),
                          "avg_gbs": (k["bytes"] / max(k["n"], 1)) / (1e-3 * k["ms"] / max(k["n"], 1)) / 1e9
                          if k["ms"] > 0 else None}
        dom = "spec_cg" if args.cg_mode != 0 else "cg_upd"
        if dom in kst and kst[dom]["ms"] > 0:
            k = kst[dom]
            avg_s = 1e-3 * k["ms"] / k["n"]
            ach = (k["bytes"] / k["n"]) / avg_s / 1e9
            traffic = None
            pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                try:
                    traffic = json.load(open(pmc)).get(dom, {}).get("hbm_bytes_per_launch")
                except Exception:
                    traffic = None
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": dom,
                    "alg_bytes_per_launch": k["bytes"] / k["n"], "avg_launch_us": round(avg_s * 1e6, 2)}

    line = None
    if rank == 0:
        value = args.steps / elapsed
        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (translating Gaussian pair, SURVEY.md §8(d); no Middlebury offline)",
            "config": {"workload": "FOTO Benamou-Brenier outer iteration, 640x480x32, r=1, eps=1e-2, "
                                   "CG rtol=1e-6 (scipy rule), stop rules off",
                       "grid": [NX, NY, NT], "cg_mode": ["stencil", "spectral-cg", "spectral-sstep8"][args.cg_mode],
                       "parallelism": f"time-slab x{world}" if world > 1 else "single GPU"},
            "cg_iters_per_step": round(float(np.mean(cg_steps)), 2) if cg_steps else None,
            "cg_iters_per_s": round(float(np.sum(cg_steps)) / elapsed, 1) if cg_steps else None,
            "phase_ms": {k: round(st_timed[k], 3) for k in ("ms_rhs", "ms_cg", "ms_prox")},
            "roofline": roof,
            "kernels": kern,
            "epe": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline()
            line["cpu_baseline"] = {"value": round(1.0 / cb["loop_s"], 6), "unit": "iters/s", "cores": 1,
                                    "kind": "port",
                                    "sample": f"oracle (numpy/scipy CSR + scipy-rule CG + vectorised stepB), first "
                                              f"outer iteration of the same 640x480x32 workload "
                                              f"({cb['cg_its']} CG its, {cb['loop_s']:.1f} s loop body)"}
            line["speedup_vs_cpu"] = round(value * cb["loop_s"], 1)
    s.close()
    if line is not None and world == 1 and not args.no_gn:
        line["gn"] = gn_side(with_cpu=not args.no_cpu_baseline)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    if line is not None:
        print(json.dumps(line))


if __name__ == "__main__":
    main()
