#!/usr/bin/env python3
"""FOTO hot-path benchmark: Benamou-Brenier outer iterations/s on the 640x480x32 grid.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cg-mode 0|1|2|3]
                    [--no-cpu-baseline] [--no-gn] [--no-stencil] [--no-batch] [--no-c4]

A "step" is one outer iteration of benamou_brenier.solve (benamou_brenier.py:204-258:
RHS + CG Poisson solve + stepB/stepC + criterion) over the synthetic 640x480x32
translating-Gaussian pair (SURVEY.md §8(d) S-metric; r = 1, eps = 1e-2, run.sh:114
parameters), with every input and all solver state resident in HBM.  The stop rules are
disabled so exactly K steps run.

N = 1: the single-GPU solve; the line also carries a "gn" object (the GN baseline, classical.py,
SURVEY.md config 3, at 640x480 and 320x240 with the oracle's SuperLU solve beside it), the
literal stencil-CG rate and the CPU baseline (the oracle on one host core).

N > 1 (torch.distributed.run, one process per GPU): the headline is north_star's decomposition --
ONE 640x480x32 solve time-sharded over the N GPUs (N time slabs; the slab <-> row-box all-to-alls,
the phi / w_t halos and the histogram all-gather over RCCL), "scaling": "strong",
value = its outer iterations per second on the slowest rank's clock.  It runs in a child process
per rank under a watchdog (FOTO_BENCH_SHARD_TIMEOUT, 180 s): if RCCL fails or hangs on any rank,
value is null and the line says why -- it is never replaced by another number.  Side objects:
  * "c4": BASELINE config 4, the 1024x1024x64 pair time-sharded over the same N GPUs (its own
    child per rank, its own communicator);
  * "batch": N independent 640x480x32 solves, one per GPU (config 5's shape: run.py streams
    independent sequences), value = all N solves' outer iterations per second -- weak scaling,
    no collective in its data path.
"rccl_ranks" is ncclCommCount of every rank's communicator (the line checks they agree).

Multi-GPU runs need no PyTorch: the ranks (launched by torch.distributed.run, which only sets
RANK / WORLD_SIZE / LOCAL_RANK) meet through files in a directory keyed by the launcher's
MASTER_PORT and process id (FileRendezvous): the RCCL unique id, the barriers and the
max-over-ranks timing.  FOTO_BENCH_MOCK_RCCL=1 (tests only): rank 0's child runs all N ranks as
threads over libfoto_mockrccl.so on one device (tests/test_gpu_bench.py).

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
    ap.add_argument("--no-batch", action="store_true", help="N > 1: skip the data-parallel side object")
    ap.add_argument("--no-c4", action="store_true", help="N > 1: skip the config-4 (1024x1024x64) sharded side run")
    ap.add_argument("--c4-steps", type=int, default=20)
    ap.add_argument("--c4-warmup", type=int, default=2)
    ap.add_argument("--shard-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--grid", type=int, nargs=3, default=[NX, NY, NT], help=argparse.SUPPRESS)
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
        ab = os.path.join(self.dir, "abort")
        while not all(os.path.exists(p) for p in paths):
            if os.path.exists(ab):   # a peer failed (abort): no point waiting for it
                raise RuntimeError(f"rendezvous {self.dir}: a peer aborted: {open(ab).read()[:300]}")
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

    def abort(self, msg):
        """Tell every rank still waiting in this rendezvous that this one failed."""
        try:
            self._put("abort", f"rank {self.rank}: {msg}".encode())
        except OSError:
            pass

    def gather(self, value):
        """Every rank's JSON-able value, in rank order, on every rank."""
        self.n += 1
        self._put(f"gat{self.n}_{self.rank}", json.dumps(value).encode())
        names = [os.path.join(self.dir, f"gat{self.n}_{g}") for g in range(self.world)]
        self._wait(names)
        return [json.loads(open(p).read()) for p in names]

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
    level 18 n_c fp64 values -- except level 0, whose legs form B and D^-1 from (fx, fy, f2)
    instead of loading them (round 6): down 9 n_0, up 12 n_0."""
    ns = gn_levels(w, h)
    v = 12 * ns[0] + 18 * ns[0]
    for l in range(len(ns) - 1):
        v += (9 + 12 if l == 0 else 18 + 21) * ns[l] + 6 * ns[l + 1]
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
                                 "note": "PCG phase: 10 launches per iteration (the update folded into the level-0 down leg, level 0's B and D^-1 formed from fx, fy, f2, the last level + coarsest in one LDS-resident block), 4 iterations per graph replay, small levels at the launch floor"}})
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


# ------------------------------------------------------------------- N > 1: the time-sharded solve

# DESIGN.md §5's model of the time-sharded solve (each rank's compute measured as virtual shards on
# one MI355X, plus the two all-to-alls, the halos and the all-gathers at 64 GB/s per xGMI link
# direction and 10 us per RCCL call; profiles/r06_proxy_scaling.txt, r06_proxy_scaling_c4.txt):
# the curve a measured N-GPU line is read against.  The metric grid's transposition moves more
# bytes per link than the single GPU needs for a whole outer iteration at W = 2, so the model puts
# W = 2 below one GPU there.
MODEL_IT_S = {(640, 480, 32): {1: 1815, 2: 894, 4: 1760, 8: 2388},
              (1024, 1024, 64): {1: 309, 2: 171, 4: 491, 8: 1075}}
C4_GRID = (1024, 1024, 64)   # BASELINE config 4: the 1024x1024 pair, 64 time steps, time-sharded


def sharded_step_model(grid, world, nloc):
    """Per-rank algorithmic HBM bytes of one time-sharded outer iteration: the single-GPU items
    (STEP_BYTES_PER_VOXEL) on the rank's slab / row box (~nloc Nx Ny voxels each), plus the
    all-to-all staging -- each of the two slab <-> box all-to-alls reads (W - 1) / W of the slab
    and writes as much of the box, 8 B each way per voxel -- and the bytes the rank sends over
    xGMI (16 (W - 1) / W B per slab voxel and outer iteration)."""
    nx, ny, nt = grid
    vs = nloc * nx * ny
    frac = (world - 1) / world
    items = dict(STEP_BYTES_PER_VOXEL)
    items["a2a_staging"] = round(32 * frac, 4)
    per_voxel = sum(items.values())
    return {"voxels_per_rank": vs, "alg_bytes_per_voxel": round(per_voxel, 4), "items": items,
            "alg_bytes_per_rank": per_voxel * vs, "xgmi_bytes_per_rank": 16 * frac * vs}


class ThreadSync:
    """FileRendezvous's barrier / max / gather for ranks that are threads of one process
    (FOTO_BENCH_MOCK_RCCL: every rank over the in-process RCCL transport on one device)."""

    def __init__(self, world):
        import threading
        self.world = world
        self.bar = threading.Barrier(world, timeout=300)
        self.slot = [None] * world

    def abort(self):
        self.bar.abort()

    def view(self, rank):
        sync = self

        class View:
            def barrier(self):
                sync.bar.wait()

            def gather(self, value):
                sync.slot[rank] = value
                sync.bar.wait()
                out = list(sync.slot)
                sync.bar.wait()
                return out

            def max(self, value):
                return max(self.gather(float(value)))

        return View()


def shard_rank(rank, world, device, grid, steps, warmup, cg_mode, nccl_id, sync, timing, library=None):
    """One rank of the time-sharded solve: its slab of the grid, warmup, a barrier, K timed outer
    iterations (the slowest rank's clock), then K more with a HIP event pair around every launch
    (the per-rank kernel table).  Returns rank 0's view with every rank's communicator size and
    slab length."""
    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian
    nx, ny, nt = grid
    rho0, rhoT = translating_gaussian(nx, ny)
    with BBSolver(rho0, rhoT, nt, nx, ny, r=R, reg_epsilon=EPS, device=device, cg_mode=cg_mode, rank=rank,
                  world=world, nccl_id=nccl_id, library=library) as t:
        ranks = t.comm_size()
        t.iterate(warmup, 0.0, stop_rules=False)
        t.sync()
        sync.barrier()
        n0 = len(t.cg_its)
        t0 = time.perf_counter()
        t.iterate(steps, 0.0, stop_rules=False)
        t.sync()
        el = sync.max(time.perf_counter() - t0)
        cg = t.cg_its[n0:]
        kern = None
        if timing:
            t.reset_stats()
            t.set_timing(True)
            t.iterate(steps, 0.0, stop_rules=False)
            t.sync()
            t.set_timing(False)
            kern = t.stats()["kernels"]
        _, nloc = t.shard()
        info = sync.gather({"rccl_ranks": ranks, "nloc": nloc})
    return {"elapsed": el, "cg": cg, "kernels": kern, "ranks": info}


def shard_summary(res, grid, world, steps, warmup, cg_mode):
    """Rank 0's object for a time-sharded run: iters/s, every rank's ncclCommCount, the per-rank
    kernel table, the dominant kernel's roofline and the per-rank step roofline."""
    el = res["elapsed"]
    step_s = el / steps
    rr = [r["rccl_ranks"] for r in res["ranks"]]
    nloc_max = max(r["nloc"] for r in res["ranks"])
    out = {"value": round(steps / el, 4), "unit": "iters/s", "ms_per_step": round(1e3 * step_s, 3), "steps": steps,
           "warmup": warmup, "n_gpus": world, "scaling": "strong", "grid": list(grid),
           "rccl_ranks": rr[0] if len(set(rr)) == 1 else None, "rccl_ranks_per_rank": rr,
           "planes_per_rank": [r["nloc"] for r in res["ranks"]],
           "cg_iters_per_step": round(float(np.mean(res["cg"])), 2) if res["cg"] else None,
           "model_it_s": MODEL_IT_S.get(tuple(grid), {}).get(world)}
    kern = res["kernels"]
    roof = None
    if kern:
        out["kernels"] = {name: {"launches": k["n"], "avg_us": round(1e3 * k["ms"] / max(k["n"], 1), 2)}
                          for name, k in kern.items()}
        k = kern.get("prox")
        if k and k["ms"] > 0:
            avg_s = 1e-3 * k["ms"] / k["n"]
            ach = (k["bytes"] / k["n"]) / avg_s / 1e9
            roof = {"bound": "hbm", "kernel": "prox", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "alg_bytes_per_launch": k["bytes"] / k["n"],
                    "avg_launch_us": round(avg_s * 1e6, 2), "note": "rank 0's slab (HIP events, timing pass)"}
    if cg_mode == 3:
        m = sharded_step_model(grid, world, nloc_max)
        ach = m["alg_bytes_per_rank"] / step_s / 1e9
        m.update({"achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                  "xgmi_gbs_per_rank": round(m["xgmi_bytes_per_rank"] / step_s / 1e9, 1),
                  "note": "per rank: the largest slab's algorithmic bytes over the slowest rank's step time"})
        if roof is None:
            roof = {"bound": "hbm", "kernel": None}
        roof["step"] = m
    out["roofline"] = roof
    return out


def shard_child(args):
    """--shard-child: one rank of a time-sharded run (started by run_shard_side with its own
    rendezvous directory), or, with FOTO_BENCH_MOCK_RCCL=1, every rank as a thread over the
    in-process RCCL transport on one device (tests)."""
    world = args.gpus
    grid = tuple(args.grid)
    device = int(os.environ.get("FOTO_BENCH_LOCAL_DEVICE", "0"))
    timing = not args.no_kernel_timing
    import ctypes
    from foto import _lib
    if os.environ.get("FOTO_BENCH_MOCK_RCCL") == "1":
        import threading
        L = _lib.load(os.path.join(REPO, "optical-flow-optimal-transport_amd", "foto", "libfoto_mockrccl.so"))
        buf = ctypes.create_string_buffer(128)
        _lib.check(L.foto_nccl_unique_id(buf), L)
        ts = ThreadSync(world)
        out, errs = [None] * world, []

        def run(g):
            try:
                out[g] = shard_rank(g, world, device, grid, args.steps, args.warmup, args.cg_mode, bytes(buf.raw),
                                    ts.view(g), timing, L)
            except BaseException as e:  # noqa: BLE001 -- reported below
                errs.append(f"rank {g}: {e}")
                ts.abort()

        th = [threading.Thread(target=run, args=(g,)) for g in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise SystemExit("; ".join(sorted(errs))[:600])
        res = out[0]
    else:
        rank = int(os.environ["RANK"])
        rdv = FileRendezvous(rank, world, timeout=150, dir=os.environ["FOTO_BENCH_RDV_DIR"])
        try:
            buf = None
            if rank == 0:
                b = ctypes.create_string_buffer(128)
                _lib.check(_lib.lib().foto_nccl_unique_id(b))
                buf = bytes(b.raw)
            nid = rdv.broadcast("nccl_id", buf)
            res = shard_rank(rank, world, device, grid, args.steps, args.warmup, args.cg_mode, nid, rdv, timing)
        except BaseException as e:
            rdv.abort(str(e))   # (the peers' children stop waiting for this one at once)
            raise
        rdv.close()
        if rank != 0:
            return
    print(json.dumps(shard_summary(res, grid, world, args.steps, args.warmup, args.cg_mode)), flush=True)


def run_shard_side(args, rdv, rank, world, local_rank, grid, steps, warmup, tag):
    """A time-sharded run over the N GPUs in child processes (one per rank, `--shard-child`):
    each rank waits for its child at most FOTO_BENCH_SHARD_TIMEOUT s (default 180) and kills it
    after that, then every rank's outcome is gathered -- a failure or a hang inside RCCL on ANY
    rank comes back to rank 0 as (None, error), never as a number.  Returns (result, error) on
    rank 0, (None, None) elsewhere."""
    mock = os.environ.get("FOTO_BENCH_MOCK_RCCL") == "1"
    limit = float(os.environ.get("FOTO_BENCH_SHARD_TIMEOUT", "180"))
    res, err = None, None
    if not mock or rank == 0:
        env = dict(os.environ, FOTO_BENCH_RDV_DIR=os.path.join(rdv.dir, tag), FOTO_BENCH_LOCAL_DEVICE=str(local_rank))
        # RCCL's bootstrap over loopback: the ranks share one node, and the container's hostname
        # or default interface may not resolve (the intra-node transports are P2P / SHM either way)
        env.setdefault("NCCL_SOCKET_IFNAME", "lo")
        cmd = [sys.executable, os.path.abspath(__file__), "--shard-child", "--gpus", str(world), "--steps", str(steps),
               "--warmup", str(warmup), "--cg-mode", str(args.cg_mode), "--grid", *[str(v) for v in grid]]
        if args.no_kernel_timing:
            cmd.append("--no-kernel-timing")
        proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        try:
            out, errtxt = proc.communicate(timeout=limit)
        except subprocess.TimeoutExpired:
            proc.kill()   # (this rank's own child, by its handle)
            proc.communicate()
            err = f"rank {rank}: no result after {limit:.0f} s (killed)"
        else:
            if proc.returncode != 0:
                tail = [ln for ln in (errtxt or "").strip().splitlines() if ln.strip()][-3:]
                err = f"rank {rank}: exited {proc.returncode}: {' | '.join(tail)}"[:400]
            elif rank == 0:
                lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
                res = json.loads(lines[-1]) if lines else None
                if res is None:
                    err = "rank 0: no result line"
    errs = [e for e in rdv.gather(err) if e]
    if rank != 0:
        return None, None
    if errs:
        return None, "; ".join(errs)[:800]
    return res, None


# ----------------------------------------------------------------------- the solve on this GPU

def measure_local(args, device, rdv):
    """This GPU's own 640x480x32 solve (N = 1: the headline; N > 1: one of the batch's
    independent solves): warmup, barrier, K timed steps (max over ranks), then K more with a HIP
    event pair around every launch (kernel table, dominant kernel's roofline)."""
    from foto.bb import BBSolver
    from foto.synthetic import translating_gaussian
    rho0, rhoT = translating_gaussian(NX, NY)
    s = BBSolver(rho0, rhoT, NT, NX, NY, r=R, reg_epsilon=EPS, device=device, cg_mode=args.cg_mode)

    def barrier():
        s.sync()
        if rdv is not None:
            rdv.barrier()

    s.iterate(args.warmup, 0.0, stop_rules=False)   # warmup (untimed)
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

    roof, kern, phase_ms = None, {}, None
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
            ev = {"achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_us": round(avg_s * 1e6, 2)}
            roof = {"bound": "hbm", "achieved": ev["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ev["frac"], "traffic": traffic, "traffic_source": traffic_src,
                    "kernel": dom, "alg_bytes_per_launch": k["bytes"] / k["n"], "avg_launch_us": ev["avg_launch_us"],
                    "frac_source": "event"}
            # the headline fraction is the kernel's duration in the timed loop itself (no events
            # between launches), from the committed rocprofv3 trace of this bench command
            # (tools/prox_segments.py) when there is one: the event-bracketed duration leaves out
            # the hand-over from the previous kernel that the loop charges to this launch.  Both
            # are reported; the loop one is the stricter.
            lt = os.path.join(REPO, "profiles", "prox_loop_trace.json")
            if dom == "prox" and os.path.exists(lt):
                try:
                    lj = json.load(open(lt))
                    lus = float(lj["loop_avg_us"])
                    lach = (k["bytes"] / k["n"]) / (lus * 1e-6) / 1e9
                    roof.update({"achieved": round(lach, 1), "frac": round(lach / HBM_PEAK_GBS, 4),
                                 "avg_launch_us": lus, "frac_source": "loop_trace"})
                    roof["event_bracketed"] = ev
                    roof["loop_trace"] = {"avg_launch_us": lus, "event_avg_us_same_trace": lj.get("event_avg_us"),
                                          "source": lj.get("source")}
                except Exception:
                    pass
            try:
                if dom == "spec_cg":
                    roof.update(stream_ceiling(1, avg_s * 1e6))
                elif dom == "prox":
                    roof.update(stream_ceiling_prox(avg_s * 1e6))
            except Exception as e:   # an older library in an A/B run (FOTO_LIB) has no probe
                roof["stream_note"] = f"stream probe unavailable: {e}"
    s.close()
    return {"elapsed": elapsed, "cg": cg_steps, "cg_redo": int(st_timed["cg_redo"]), "roofline": roof,
            "kernels": kern, "phase_ms": phase_ms, "rho0": rho0, "rhoT": rhoT}


def visible_device(local_rank):
    """The HIP ordinal of this rank's GPU: LOCAL_RANK, unless the launcher narrowed the visible
    devices (HIP_ / ROCR_ / CUDA_VISIBLE_DEVICES listing fewer than LOCAL_RANK + 1 of them, e.g.
    one per process) -- then the rank's GPU is the one it can see."""
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(k)
        if v is not None and v.strip():
            n = len([d for d in v.split(",") if d.strip()])
            if 0 < n <= local_rank:
                return local_rank % n
    return local_rank


def line_base(args, world):
    return {"metric": METRIC, "value": None, "unit": "iters/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
            "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (translating Gaussian pair, SURVEY.md §8(d); no Middlebury offline)",
            "config": {"workload": "FOTO Benamou-Brenier outer iteration, 640x480x32, r=1, eps=1e-2, "
                                   "CG rtol=1e-6 (scipy rule), stop rules off",
                       "grid": [NX, NY, NT],
                       "cg_mode": ["stencil", "spectral-cg", "spectral-sstep8", "spectral-gauss"][args.cg_mode],
                       "parallelism": (f"time-slab x{world}: one 640x480x32 solve sharded on t over {world} GPUs "
                                       f"(slab <-> row-box all-to-alls, phi / w_t halos, histogram all-gather over "
                                       f"RCCL; DESIGN.md 5)" if world > 1 else "single GPU")},
            "epe": None}


def main():
    args = parse()
    if args.cpu_baseline_only:
        cpu_baseline_child()
        return
    if args.gn_cpu_only:
        gn_cpu_child()
        return
    if args.shard_child:
        shard_child(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # FOTO_BENCH_DEVICES=0,0: rank i on device LIST[i mod len] (tests: several ranks on one GPU);
    # default: the rank's own GPU
    devs = [int(v) for v in os.environ.get("FOTO_BENCH_DEVICES", "").split(",") if v.strip()]
    if devs:
        local_rank = devs[local_rank % len(devs)]
    else:
        local_rank = visible_device(local_rank)
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    if world > 1:
        rdv = FileRendezvous(rank, world)
        # 1. the headline: the metric grid time-sharded over the N GPUs
        shard, err = run_shard_side(args, rdv, rank, world, local_rank, (NX, NY, NT), args.steps, args.warmup, "shard")
        # 2. config 4 time-sharded over the same GPUs (its own children and communicator)
        c4 = None
        if not args.no_c4:
            c4, c4err = run_shard_side(args, rdv, rank, world, local_rank, C4_GRID, args.c4_steps, args.c4_warmup, "c4")
            if c4err:
                c4 = {"value": None, "error": c4err}
            if c4 is not None:
                c4["workload"] = "BASELINE config 4: 1024x1024x64 synthetic pair, r=1, eps=1e-2, time-sharded"
        # 3. the data-parallel side object: one independent solve per GPU, no collective
        batch = None
        if not args.no_batch:
            loc = measure_local(args, local_rank, rdv)
            if rank == 0:
                batch = {"value": round(world * args.steps / loc["elapsed"], 4), "unit": "iters/s",
                         "scaling": "weak", "n_gpus": world,
                         "ms_per_step": round(1e3 * loc["elapsed"] / args.steps, 3),
                         "cg_iters_per_step": round(float(np.mean(loc["cg"])), 2) if loc["cg"] else None,
                         "roofline": loc["roofline"],
                         "parallelism": f"data-parallel x{world}: one independent 640x480x32 solve per GPU "
                                        f"(config 5's shape, run.py streams independent sequences); value = "
                                        f"all {world} solves' outer iterations / the slowest rank's time"}
        rdv.close()
        if rank != 0:
            return
        line = line_base(args, world)
        if shard is not None:
            line.update({"value": shard["value"], "ms_per_step": shard["ms_per_step"],
                         "rccl_ranks": shard["rccl_ranks"], "cg_iters_per_step": shard["cg_iters_per_step"],
                         "roofline": shard["roofline"], "sharded": shard})
        else:
            line.update({"rccl_ranks": None, "roofline": None, "error": err})
        line["c4"] = c4
        line["batch"] = batch
        print(json.dumps(line))
        return

    # N = 1
    loc = measure_local(args, local_rank, None)
    elapsed, cg_steps = loc["elapsed"], loc["cg"]
    line = line_base(args, 1)
    line.update({
        "value": round(args.steps / elapsed, 4),
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "cg_iters_per_step": round(float(np.mean(cg_steps)), 2) if cg_steps else None,
        "cg_iters_per_s": round(float(np.sum(cg_steps)) / elapsed, 1) if cg_steps else None,
        "phase_ms": loc["phase_ms"],
        "cg_redo": loc["cg_redo"],
        "roofline": loc["roofline"],
        "survey_model": {"bytes_per_step": survey_bytes(float(np.mean(cg_steps))) if cg_steps else None,
                         "equiv_gbs": round(survey_bytes(float(np.mean(cg_steps))) / (elapsed / args.steps) / 1e9, 1)
                         if cg_steps else None,
                         "note": "SURVEY.md 8(d) bytes of the literal stencil algorithm, (21 + 10k) N 8 B per "
                                 "outer iteration, over this run's step time: above HBM peak because the default "
                                 "path solves the same CG recurrence in the DCT basis (DESIGN.md 3.1)"},
        "kernels": loc["kernels"],
    })
    if line["roofline"] is not None:
        line["roofline"]["step"] = step_roofline(args.cg_mode, 1, elapsed / args.steps)
    if args.cg_mode != 0 and not args.no_stencil:
        line["literal_stencil"] = literal_stencil_rate(loc["rho0"], loc["rhoT"], local_rank)
    # the CPU baselines run after every GPU measurement (no host load beside the timed GPU work),
    # side by side on two cores
    kids = {}
    gn = gn_side() if not args.no_gn else None
    if not args.no_cpu_baseline:
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
    print(json.dumps(line))


if __name__ == "__main__":
    main()
