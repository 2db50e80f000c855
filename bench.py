#!/usr/bin/env python3
"""FOTO hot-path benchmark: Benamou-Brenier outer iterations/s on the 640x480x32 grid.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cg-mode 0|1|2|3] [--mode batch|sharded]
                    [--no-cpu-baseline] [--no-gn] [--no-strong]

A "step" is one outer iteration of benamou_brenier.solve (benamou_brenier.py:204-258:
RHS + CG Poisson solve + stepB/stepC + criterion) over the synthetic 640x480x32
translating-Gaussian pair (SURVEY.md §8(d) S-metric; r = 1, eps = 1e-2, run.sh:114
parameters), with every input and all solver state resident in HBM.  The stop rules are
disabled so exactly K steps run.  With N > 1 (torch.distributed.run, one process per GPU):
  * --mode batch (default; "scaling": "weak"): every GPU solves its own 640x480x32 pair, as
    run.py streams independent sequences over GPUs (config 5, run.sh:81-157); value = the outer
    iterations of all N solves per second (whole job), the slowest rank's clock.  The same run
    then also measures the "strong" object: ONE problem time-sharded over the N GPUs (config 4's
    decomposition: N time slabs, the slab <-> row-box all-to-alls and halos over RCCL), its
    outer iterations per second -- guarded by a watchdog (FOTO_BENCH_STRONG_TIMEOUT, 180 s) so
    a stuck collective cannot cost the headline line;
  * --mode sharded: that time-sharded strong-scaling run as the headline ("scaling": "strong").
At N = 1 both are the single-GPU solve.

At N = 1 the line also carries a "gn" object: the GN baseline (classical.py)
solved on the GPU at 640x480 (and 320x240), and the oracle's SuperLU solve of the 640x480 pair
on one host core beside it (~75 s, run next to the BB CPU baseline on another core).

Multi-GPU runs need no PyTorch: the ranks (launched by torch.distributed.run, which only sets
RANK / WORLD_SIZE / LOCAL_RANK) meet through files in a directory keyed by the launcher's
MASTER_PORT and process id (FileRendezvous): rank 0's RCCL unique id, the barriers and the
max-over-ranks timing.

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
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cg-mode", type=int, default=int(os.environ.get("FOTO_CG_MODE", "3")),
                    help="0 stencil CG, 1 spectral CG (one GPU), 2 spectral s-step CG, 3 Gauss-compressed spectral CG (default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gn", action="store_true", help="skip the GN (classical.py, config 3) side measurement")
    ap.add_argument("--no-stencil", action="store_true", help="skip the literal stencil-CG side measurement")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--gn-cpu-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-launch HIP-event pass (roofline fields become null)")
    ap.add_argument("--mode", choices=["batch", "sharded"], default="batch",
                    help="N > 1: batch = one solve per GPU (weak scaling, default); sharded = one solve time-sharded "
                         "over the N GPUs (strong scaling)")
    ap.add_argument("--no-strong", action="store_true", help="N > 1, batch mode: skip the time-sharded side run")
    ap.add_argument("--strong-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


CPU_K = 2   # outer iterations the CPU baseline runs (BASELINE.md / SURVEY.md §8(d): K = 2 on CPU)


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
    q = np.zeros(3 * N)
    cg = []
    t1 = time.perf_counter()
    for _ in range(CPU_K):
        phi, info, its = O.solve_step(mu, q, rho0, rhoT, R, A.dot, NT, NY, NX)
        g = O.grad_st(phi, NT, NY, NX)
        q = O.stepB(g + (1.0 / R) * mu, N)
        mu = mu + R * (g - q)
        mu[:N] = np.maximum(mu[:N], 0)
        cg.append(int(its))
    loop = time.perf_counter() - t1
    print(json.dumps({"loop_s": loop, "assemble_s": total, "cg_its": cg, "k": CPU_K}))


GN_W, GN_H, GN_ALPHA, GN_LAMBDA = 640, 480, 0.1, 0.2   # config 3 size, run.sh:103 parameters
GN_CPU_W, GN_CPU_H = 640, 480                          # the CPU solve at the config's size (spsolve ~75 s)
GN_SMALL = (320, 240)                                  # second GPU size (latency-bound levels)


class FileRendezvous:
    """Rendezvous of the bench's ranks on one node without torch.distributed: a directory
    keyed by MASTER_PORT and the launcher's pid (every rank is a child of the same
    torch.distributed.run agent), files for the RCCL unique id, barriers and per-rank times."""

    def __init__(self, rank, world, timeout=300.0, dir=None):
        import tempfile
        self.rank, self.world, self.timeout, self.n = rank, world, timeout, 0
        key = f"{os.environ.get('MASTER_PORT', '0')}_{os.getppid()}"
        self.dir = dir or os.path.join(tempfile.gettempdir(), f"foto_bench_{key}")
        os.makedirs(self.dir, exist_ok=True)

    def _wait(self, paths):
        t0 = time.perf_counter()
        spin = 0
        while not all(os.path.exists(p) for p in paths):
            spin += 1
            if spin > 2000:
                time.sleep(0.0002)
            if time.perf_counter() - t0 > self.timeout:
                raise TimeoutError(f"rendezvous {self.dir}: waited {self.timeout} s for {paths}")

    def _put(self, name, data):
        tmp = os.path.join(self.dir, f".{name}.{self.rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(data)
        os.replace(tmp, os.path.join(self.dir, name))

    def broadcast(self, name, data=None):
        """rank 0's bytes to every rank"""
        if self.rank == 0:
            self._put(name, data)
        p = os.path.join(self.dir, name)
        self._wait([p])
        with open(p, "rb") as f:
            return f.read()

    def barrier(self):
        self.n += 1
        self._put(f"bar{self.n}_{self.rank}", b"")
        self._wait([os.path.join(self.dir, f"bar{self.n}_{g}") for g in range(self.world)])

    def max(self, value):
        self.n += 1
        self._put(f"max{self.n}_{self.rank}", repr(float(value)).encode())
        names = [os.path.join(self.dir, f"max{self.n}_{g}") for g in range(self.world)]
        self._wait(names)
        return max(float(open(p).read()) for p in names)

    def close(self):
        """Every rank but 0 leaves its final file and returns at once; rank 0 waits for all of
        them before it removes the directory, so no rank can still be polling for a file of a
        removed directory (a full barrier here let rank 0 delete the files a slower rank was
        about to check, and that rank then timed out)."""
        self.n += 1
        self._put(f"end{self.n}_{self.rank}", b"")
        if self.rank == 0:
            import shutil
            self._wait([os.path.join(self.dir, f"end{self.n}_{g}") for g in range(self.world)])
            shutil.rmtree(self.dir, ignore_errors=True)


def gn_cpu_child():
    """The oracle's GN solve (classical.py:113-130: SuperLU spsolve) on the CPU sample pair."""
    sys.path.insert(0, REPO)
    from oracle import foto_oracle as O
    from foto.synthetic import sinusoid_pair
    f1, f2 = sinusoid_pair(GN_CPU_W, GN_CPU_H)
    t = time.perf_counter()
    O.gn_solve(f1, f2, GN_CPU_W, GN_CPU_H, GN_ALPHA, GN_LAMBDA)
    print(json.dumps({"solve_s": time.perf_counter() - t}))


def gn_levels(w, h, coarse=1024):
    """Cell counts of the multigrid hierarchy (foto_gn.hip: halve until <= 1024 cells)."""
    out = [(w, h)]
    while w * h > coarse:
        w, h = (w + 1) // 2, (h + 1) // 2
        out.append((w, h))
    return [a * b for a, b in out]


def gn_bytes_per_iteration(w, h):
    """Algorithmic HBM bytes of one MG-PCG iteration: k_gnp_dir 12 n, k_gnp_upd
    18 n, per level k_mg_down2 18 n_l + 3 n_l+1 and k_mg_up2 21 n_l + 3 n_l+1, the coarsest
    level 18 n_c fp64 values."""
    ns = gn_levels(w, h)
    v = 12 * ns[0] + 18 * ns[0]
    for l in range(len(ns) - 1):
        v += 18 * ns[l] + 21 * ns[l] + 6 * ns[l + 1]
    v += 18 * ns[-1]
    return 8 * v


def gn_side():
    """GN baseline (SURVEY.md §8(d) config 3 stand-in: sinusoid pair, alpha 0.1, lambda 0.2):
    GPU solve time at 640x480 and 320x240 -- one-shot (foto_gn_solve: plan made, used,
    destroyed) and with a reused plan (a batch of same-size pairs).  gn_attach_cpu puts the
    oracle's spsolve of the 640x480 pair (timed in a child process) beside it."""
    from foto import gn
    from foto.synthetic import sinusoid_pair
    out = {"workload": f"GN classical solve, sinusoid pair, alpha={GN_ALPHA}, lambda={GN_LAMBDA}, "
                       f"CG preconditioned by a symmetric multigrid V-cycle to rtol {gn.GN_RTOL}"}
    for (w, h) in ((GN_W, GN_H), GN_SMALL):
        f1, f2 = sinusoid_pair(w, h)                  # the CPU sample's pair (at 640x480)
        g1, g2 = sinusoid_pair(w, h, dx=0.7, dy=1.1)  # another pair of the same size
        t = time.perf_counter()
        gn.solve(g1, g2, w, h, GN_ALPHA, GN_LAMBDA)   # makes the cached plan (foto_gn_solve)
        first = time.perf_counter() - t
        times = []
        for _ in range(3):   # f1, f2 through the cached plan: fresh (its count unknown), then repeated
            t = time.perf_counter()
            _, _, _, info, its = gn.solve(f1, f2, w, h, GN_ALPHA, GN_LAMBDA)
            times.append(time.perf_counter() - t)
        rec = {"solve_ms": round(1e3 * min(times[1:]), 2),
               "solve_ms_note": "foto_gn_solve with its cached plan, the same pair again (best case of a "
                                "same-size batch); fresh_pair_ms: the pair's first solve through the cached plan",
               "fresh_pair_ms": round(1e3 * times[0], 2),
               "first_call_ms": round(1e3 * first, 2), "pcg_its": its, "info": info}
        with gn.Plan(w, h, GN_ALPHA, GN_LAMBDA) as P:
            warm, tm = None, None
            for _ in range(4):
                t = time.perf_counter()
                P.solve(f1, f2)
                dt = time.perf_counter() - t
                if warm is None or dt < warm:
                    warm, tm = dt, P.timing()
        by = gn_bytes_per_iteration(w, h)
        ach = by * tm["iterations"] / (1e-3 * tm["ms_pcg"]) / 1e9
        rec.update({"plan_solve_ms": round(1e3 * warm, 2), "plan_device_ms": {"setup": round(tm["ms_setup"], 3),
                                                                               "pcg": round(tm["ms_pcg"], 3)},
                    "us_per_pcg_it": round(1e3 * tm["ms_pcg"] / max(tm["iterations"], 1), 1),
                    "roofline": {"bound": "hbm", "alg_bytes_per_it": by, "achieved": round(ach, 1),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                 "note": "PCG phase: 10 launches per iteration (the update folded into the level-0 down leg, the last level + coarsest in one LDS-resident block), 4 iterations per graph replay, small levels at the launch floor"}})
        out[f"gpu_{w}x{h}"] = rec
    return out


def gn_attach_cpu(out, cpu_s):
    if cpu_s is not None:
        gpu_s = out[f"gpu_{GN_CPU_W}x{GN_CPU_H}"]["fresh_pair_ms"] / 1e3
        out["cpu_baseline"] = {"value_s": round(cpu_s, 3), "kind": "port", "cores": 1,
                               "sample": f"oracle spsolve (SuperLU, classical.py:113-130) on the "
                                         f"{GN_CPU_W}x{GN_CPU_H} pair (the config's size)"}
        out["speedup_vs_cpu"] = round(cpu_s / gpu_s, 1)
        out["speedup_note"] = (f"oracle spsolve vs the GPU's fresh-pair solve, both at {GN_CPU_W}x{GN_CPU_H}")


def start_cpu_children(with_gn):
    """The CPU baselines as child processes on two different host cores (one thread each):
    the BB oracle (K = 2 outer iterations) and, with_gn, the GN oracle's spsolve at 640x480."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    cores = sorted(os.sched_getaffinity(0))
    kids = {}
    for j, (name, flag) in enumerate((("bb", "--cpu-baseline-only"), ("gn", "--gn-cpu-only"))):
        if name == "gn" and not with_gn:
            continue
        core = cores[(len(cores) - 1 - j) % len(cores)]
        kids[name] = (subprocess.Popen([sys.executable, os.path.abspath(__file__), flag], env=env,
                                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                       preexec_fn=(lambda c=core: os.sched_setaffinity(0, {c}))), core)
    return kids


def collect_cpu_child(kids, name, timeout=900):
    if name not in kids:
        return None
    p, core = kids[name]
    out, err = p.communicate(timeout=timeout)
    if p.returncode != 0:
        raise RuntimeError(f"cpu baseline {name} failed: " + err[-2000:])
    res = json.loads(out.strip().splitlines()[-1])
    res["core"] = core
    return res


def literal_stencil_rate(rho0, rhoT, device, steps=3, warmup=1):
    """Secondary line: the literal algorithm (mode 0: scipy's CG on the 7-point stencil, no DCT
    basis) on the same workload, so the spectral substitution is visible beside `value`."""
    from foto.bb import BBSolver
    with BBSolver(rho0, rhoT, NT, NX, NY, r=R, reg_epsilon=EPS, device=device, cg_mode=0) as s:
        s.iterate(warmup, 0.0, stop_rules=False)
        s.sync()
        n0 = len(s.cg_its)
        t0 = time.perf_counter()
        s.iterate(steps, 0.0, stop_rules=False)
        s.sync()
        dt = time.perf_counter() - t0
        k = float(np.mean(s.cg_its[n0:]))
    b = survey_bytes(k)
    return {"cg_mode": "stencil", "value": round(steps / dt, 3), "unit": "iters/s", "steps": steps,
            "ms_per_step": round(1e3 * dt / steps, 3), "cg_iters_per_step": round(k, 2),
            "survey_model_gbs": round(b / (dt / steps) / 1e9, 1),
            "survey_model_frac": round(b / (dt / steps) / 1e9 / HBM_PEAK_GBS, 4)}


def stream_ceiling(world, pass_us):
    """The dominant pass against the device's own stream rate for the same traffic
    (foto_stream_probe: read + write the rank's r^, q^ box, 16 B per lane, no moments or
    plan): the pass's 157 MB working set is Infinity-Cache resident, so the plain r, q stream
    exceeds the guide's 6.3 TB/s "achievable HBM"; stream_frac is what the pass keeps of it."""
    import ctypes
    from foto import _lib
    n = NT * (NY // world + (1 if NY % world else 0)) * NX
    n -= n % 2
    us = (ctypes.c_double * 2)()
    _lib.check(_lib.lib().foto_stream_probe(n, 20, us))
    best = min(us[0], us[1])
    return {"stream_us": round(best, 2), "stream_gbs": round(32.0 * n / (best * 1e-6) / 1e9, 1),
            "stream_frac": round(best / pass_us, 4),
            "stream_note": f"foto_stream_probe over the {n}-element box: plain stores {us[0]:.1f} us, "
                           f"write-through {us[1]:.1f} us per launch"}


def stream_ceiling_prox(prox_us):
    """The fused prox + RHS kernel against the device's stream rate for its traffic
    (foto_stream_probe4: 4 fields of the grid in, 4 out, 64 B per voxel -- 629 MB at the bench
    size, beyond the 256 MiB Infinity Cache, so this is the practical HBM rate of that access
    pattern on this box); stream_frac is what k_prox_rhs keeps of it."""
    import ctypes
    from foto import _lib
    n = NT * NY * NX
    n -= n % 2
    us = (ctypes.c_double * 1)()
    _lib.check(_lib.lib().foto_stream_probe4(n, 10, us))
    return {"stream_us": round(us[0], 2), "stream_gbs": round(64.0 * n / (us[0] * 1e-6) / 1e9, 1),
            "stream_frac": round(us[0] / prox_us, 4),
            "stream_note": f"foto_stream_probe4: 4 x {n} doubles in, 4 out (64 B per voxel), "
                           f"{us[0]:.1f} us per launch"}


# Algorithmic HBM bytes per voxel of one outer iteration of the default path (cg_mode 3, one
# GPU): every x / y / t DCT pass reads and writes the grid once (16 B; 3 forward,
# 3 inverse), the Gauss histogram reads b^ and its 4-B bin-order list entry (12 B), x^ = Q b^
# reads b^ and writes x^ (16 B), the fused prox + next RHS 64 B.  The node CG, nodes and table
# move nothing per voxel.
STEP_BYTES_PER_VOXEL = {"dct_fwd_xyt": 48, "gq_hist": 12, "gq_xhat": 16, "dct_inv_tyx": 48, "prox_rhs": 64}


def step_roofline(cg_mode, world, step_s):
    """The whole outer iteration against HBM peak: the itemised algorithmic bytes above over
    the measured step time, and the PMC-measured bytes per step (profiles/pmc_traffic.json
    "_step", written by tools/summarize_profile.py from the same workload)."""
    if cg_mode != 3 or world != 1:
        return None
    n = NX * NY * NT
    by = sum(STEP_BYTES_PER_VOXEL.values()) * n
    ach = by / step_s / 1e9
    out = {"alg_bytes_per_voxel": sum(STEP_BYTES_PER_VOXEL.values()), "items": STEP_BYTES_PER_VOXEL,
           "alg_bytes": by, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None}
    pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        st = json.load(open(pmc)).get("_step")
        if st:
            out["traffic"] = st["hbm_bytes_per_step"]
            out["traffic_frac_at_this_step_time"] = round(st["hbm_bytes_per_step"] / step_s / 1e9 / HBM_PEAK_GBS, 4)
            out["traffic_source"] = st.get("source")
    except Exception:
        pass
    return out


def survey_bytes(k):
    """SURVEY.md §8(d) algorithmic bytes of one outer iteration of the literal algorithm:
    (21 + 10 k) N 8 B with k CG iterations."""
    return (21 + 10 * k) * NX * NY * NT * 8


def strong_side(args, rdv, rank, world, local_rank):
    """Batch mode, N > 1: ONE solve time-sharded over the N GPUs (config 4's decomposition over
    RCCL) on the same workload, run by a child process per rank (`--strong-child`): warmup,
    barrier, K timed outer iterations, the slowest rank's clock.  Each rank waits for its child
    at most FOTO_BENCH_STRONG_TIMEOUT s (default 180) and kills it after that -- a collective that
    never completes, or a crash inside RCCL, cannot cost the data-parallel headline, which this
    process prints either way (the RCCL calls have run only through the in-process transport
    before, never across GPUs)."""
    import subprocess
    limit = float(os.environ.get("FOTO_BENCH_STRONG_TIMEOUT", "180"))
    env = dict(os.environ, FOTO_BENCH_RDV_DIR=os.path.join(rdv.dir, "strong"), FOTO_BENCH_PARENT_RDV=rdv.dir,
               FOTO_BENCH_LOCAL_DEVICE=str(local_rank))
    cmd = [sys.executable, os.path.abspath(__file__), "--strong-child", "--gpus", str(world), "--steps",
           str(args.steps), "--warmup", str(args.warmup), "--cg-mode", str(args.cg_mode)]
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        out, err = proc.communicate(timeout=limit)
    except subprocess.TimeoutExpired:
        proc.kill()   # (this rank's own child, by its handle)
        proc.communicate()
        return {"error": f"timeout after {limit:.0f} s"}
    if proc.returncode != 0:
        tail = (err or "").strip().splitlines()[-3:]
        return {"error": f"strong side run exited {proc.returncode}: {' | '.join(tail)}"[:300]}
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    if rank != 0:
        return None
    return json.loads(lines[-1]) if lines else {"error": "no result line"}


def strong_child(args):
    """The strong side run's worker (one per rank, started by strong_side): its own rendezvous
    directory inside the parent's, the RCCL id rank 0's parent broadcast, the same workload."""
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    device = int(os.environ["FOTO_BENCH_LOCAL_DEVICE"])
    rdv = FileRendezvous(rank, world, timeout=120, dir=os.environ["FOTO_BENCH_RDV_DIR"])
    with open(os.path.join(os.environ["FOTO_BENCH_PARENT_RDV"], "nccl_id"), "rb") as f:
        nccl_id = f.read()
    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian
    rho0, rhoT = translating_gaussian(NX, NY)
    with BBSolver(rho0, rhoT, NT, NX, NY, r=R, reg_epsilon=EPS, device=device, cg_mode=args.cg_mode,
                  rank=rank, world=world, nccl_id=nccl_id) as t:
        t.iterate(args.warmup, 0.0, stop_rules=False)
        t.sync()
        rdv.barrier()
        n0 = len(t.cg_its)
        t0 = time.perf_counter()
        t.iterate(args.steps, 0.0, stop_rules=False)
        t.sync()
        el = rdv.max(time.perf_counter() - t0)
        rdv.barrier()
        cg = t.cg_its[n0:]
    rdv.close()
    if rank == 0:
        print(json.dumps({"value": round(args.steps / el, 4), "unit": "iters/s", "ms_per_step": round(1e3 * el / args.steps, 3),
                          "steps": args.steps, "scaling": "strong", "n_gpus": world,
                          "cg_iters_per_step": round(float(np.mean(cg)), 2) if cg else None,
                          "parallelism": f"time-slab x{world}: {NT} planes split over {world} ranks, slab <-> row-box "
                                         f"all-to-alls and the w_t halo over RCCL (DESIGN.md 5)"}), flush=True)




def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline_child()
        return
    if args.gn_cpu_only:
        gn_cpu_child()
        return
    if args.strong_child:
        strong_child(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # FOTO_BENCH_DEVICES=0,0: rank i on device LIST[i mod len] (tests: two batch-mode ranks on
    # one GPU); default: the rank's own GPU
    devs = [int(v) for v in os.environ.get("FOTO_BENCH_DEVICES", "").split(",") if v.strip()]
    if devs:
        local_rank = devs[local_rank % len(devs)]
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    rdv = None
    nccl_id = None
    sharded = world > 1 and args.mode == "sharded"
    want_strong = world > 1 and args.mode == "batch" and not args.no_strong
    if world > 1:
        rdv = FileRendezvous(rank, world)
        if sharded or want_strong:
            buf = None
            if rank == 0:
                import ctypes
                import foto
                b = ctypes.create_string_buffer(128)
                foto._lib.check(foto.lib().foto_nccl_unique_id(b))
                buf = bytes(b.raw)
            nccl_id = rdv.broadcast("nccl_id", buf)

    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian

    rho0, rhoT = translating_gaussian(NX, NY)
    # batch mode: this rank's own solve (no RCCL); sharded mode: its slab of the one solve
    s = BBSolver(rho0, rhoT, NT, NX, NY, r=R, reg_epsilon=EPS, device=local_rank, cg_mode=args.cg_mode,
                 rank=rank if sharded else 0, world=world if sharded else 1, nccl_id=nccl_id if sharded else None)
    solves = world if (world > 1 and not sharded) else 1   # problems the timed region advances

    def barrier():
        s.sync()
        if rdv is not None:
            rdv.barrier()

    # warmup (untimed)
    s.iterate(args.warmup, 0.0, stop_rules=False)
    barrier()
    s.reset_stats()
    its_before = len(s.cg_its)
    t0 = time.perf_counter()
    s.iterate(args.steps, 0.0, stop_rules=False)
    s.sync()
    elapsed = time.perf_counter() - t0
    if rdv is not None:
        elapsed = rdv.max(elapsed)   # (includes every rank's own device sync)
        rdv.barrier()
    cg_steps = s.cg_its[its_before:]
    st_timed = s.stats()

    # per-launch kernel timing pass: K more steps with a HIP event pair around every launch
    roof = None
    kern = {}
    phase_ms = None
    if not args.no_kernel_timing:
        s.reset_stats()
        s.set_timing(True)
        s.iterate(args.steps, 0.0, stop_rules=False)
        barrier()
        s.set_timing(False)
        st_k = s.stats()
        # (the RHS / CG / prox phase events run with the kernel timing only: they cost ~2 % of
        # the step, so the timed pass above records none)
        phase_ms = {k: round(st_k[k], 3) for k in ("ms_rhs", "ms_cg", "ms_prox")}
        kst = st_k["kernels"]
        for name, k in kst.items():
            kern[name] = {"launches": k["n"], "avg_us": 1e3 * k["ms"] / max(k["n"], 1),
                          "avg_gbs": (k["bytes"] / max(k["n"], 1)) / (1e-3 * k["ms"] / max(k["n"], 1)) / 1e9
                          if k["ms"] > 0 else None}
        # the dominant single kernel: the s-step pass (mode 1/2), the stencil CG update (mode 0);
        # with the Gauss-compressed CG (mode 3) the CG is ~6 small kernels and the fused
        # prox + next RHS (k_prox_rhs, one launch per outer iteration) is the largest one
        dom = {0: "cg_upd", 3: "prox"}.get(args.cg_mode, "spec_cg")
        if dom in kst and kst[dom]["ms"] > 0:
            k = kst[dom]
            avg_s = 1e-3 * k["ms"] / k["n"]
            ach = (k["bytes"] / k["n"]) / avg_s / 1e9
            traffic, traffic_src = None, None
            pmc = os.path.join(REPO, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                try:
                    pj = json.load(open(pmc))
                    traffic = pj.get(dom, {}).get("hbm_bytes_per_launch")
                    traffic_src = pj.get("_source", "profiles/pmc_traffic.json")
                except Exception:
                    traffic = None
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": dom, "alg_bytes_per_launch": k["bytes"] / k["n"], "avg_launch_us": round(avg_s * 1e6, 2)}
            # the same kernel's duration in the timed loop itself (no events between launches), from
            # the committed rocprofv3 trace of this bench command (tools/prox_segments.py): the
            # event-bracketed duration above leaves out the hand-over from the previous kernel that
            # the loop charges to this launch -- both are reported, the loop one is the stricter
            lt = os.path.join(REPO, "profiles", "prox_loop_trace.json")
            if dom == "prox" and os.path.exists(lt):
                try:
                    lj = json.load(open(lt))
                    lus = float(lj["loop_avg_us"])
                    roof["loop_trace"] = {"avg_launch_us": lus,
                                          "frac": round((k["bytes"] / k["n"]) / (lus * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                                          "event_avg_us_same_trace": lj.get("event_avg_us"), "source": lj.get("source")}
                except Exception:
                    pass
            try:
                if dom == "spec_cg":
                    roof.update(stream_ceiling(world if sharded else 1, avg_s * 1e6))
                elif dom == "prox" and not sharded:
                    roof.update(stream_ceiling_prox(avg_s * 1e6))
            except Exception as e:   # an older library in an A/B run (FOTO_LIB) has no probe
                roof["stream_note"] = f"stream probe unavailable: {e}"

    line = None
    if rank == 0:
        value = solves * args.steps / elapsed
        line = {
            "metric": METRIC,
            "value": round(value, 4),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if sharded else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (translating Gaussian pair, SURVEY.md §8(d); no Middlebury offline)",
            "config": {"workload": "FOTO Benamou-Brenier outer iteration, 640x480x32, r=1, eps=1e-2, "
                                   "CG rtol=1e-6 (scipy rule), stop rules off",
                       "grid": [NX, NY, NT], "cg_mode": ["stencil", "spectral-cg", "spectral-sstep8", "spectral-gauss"][args.cg_mode],
                       "parallelism": (f"time-slab x{world} (one solve over {world} GPUs, RCCL)" if sharded else
                                       f"data-parallel x{world} (one solve per GPU, independent pairs as run.py "
                                       f"streams sequences; 'strong': one solve time-sharded over the {world} GPUs)"
                                       if world > 1 else "single GPU")},
            "cg_iters_per_step": round(float(np.mean(cg_steps)), 2) if cg_steps else None,
            "cg_iters_per_s": round(solves * float(np.sum(cg_steps)) / elapsed, 1) if cg_steps else None,
            "phase_ms": phase_ms,
            "cg_redo": int(st_timed["cg_redo"]),
            "roofline": roof,
            "survey_model": {"bytes_per_step": survey_bytes(float(np.mean(cg_steps))) if cg_steps else None,
                             "equiv_gbs": round(survey_bytes(float(np.mean(cg_steps))) / (elapsed / args.steps) / 1e9, 1)
                             if cg_steps else None,
                             "note": "SURVEY.md 8(d) bytes of the literal stencil algorithm, (21 + 10k) N 8 B per "
                                     "outer iteration, over this run's step time: above HBM peak because the default "
                                     "path solves the same CG recurrence in the DCT basis (DESIGN.md 3.1)"},
            "kernels": kern,
            "epe": None,
        }
        if roof is not None:
            roof["step"] = step_roofline(args.cg_mode, world if sharded else 1, elapsed / args.steps)
    s.close()
    if want_strong:   # (child processes: a hang or crash in RCCL is reported, not fatal)
        strong = strong_side(args, rdv, rank, world, local_rank)
        if line is not None:
            line["strong"] = strong
    if line is not None and world == 1 and args.cg_mode != 0 and not args.no_stencil:
        line["literal_stencil"] = literal_stencil_rate(rho0, rhoT, local_rank)
    # the CPU baselines run after every GPU measurement (no host load beside the timed GPU work),
    # side by side on two cores
    kids = {}
    gn = gn_side() if (line is not None and world == 1 and not args.no_gn) else None
    if line is not None and world == 1 and not args.no_cpu_baseline:
        kids = start_cpu_children(with_gn=gn is not None)
    if gn is not None:
        gn_cpu = collect_cpu_child(kids, "gn", timeout=1200)
        gn_attach_cpu(gn, gn_cpu["solve_s"] if gn_cpu else None)
        line["gn"] = gn
    if "bb" in kids:
        cb = collect_cpu_child(kids, "bb")
        cpu_value = cb["k"] / cb["loop_s"]
        line["cpu_baseline"] = {"value": round(cpu_value, 6), "unit": "iters/s", "cores": 1,
                                "kind": "port", "nproc": os.cpu_count(),
                                "affinity": len(os.sched_getaffinity(0)), "core": cb["core"],
                                "sample": f"oracle (numpy/scipy CSR + scipy-rule CG + vectorised stepB), first "
                                          f"{cb['k']} outer iterations of the same 640x480x32 workload "
                                          f"(CG its {cb['cg_its']}, {cb['loop_s']:.1f} s loop body), "
                                          f"OMP/BLAS threads 1 (single-core path), pinned to one core"}
        line["speedup_vs_cpu"] = round(line["value"] / cpu_value, 1)
    if rdv is not None:
        rdv.close()
    if line is not None:
        print(json.dumps(line))


if __name__ == "__main__":
    main()
