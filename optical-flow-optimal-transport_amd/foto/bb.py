"""Benamou-Brenier (FOTO) solver on the GPU: Python face of libfoto's BB context.

``solve`` keeps the reference signature and stdout of ``benamou_brenier.solve``
(benamou_brenier.py:151-271): one line ``f"{crit} ({i+1}/{max_it})"`` per outer
iteration (Python ``str`` of a float64), the CG non-convergence warning of
benamou_brenier.py:86-87, and (u, v, m) from the trajectory flow extraction.
"""
import collections
import ctypes
import os
import sys

import numpy as np

from . import _lib
from ._lib import check, dptr, f64, lib

CG_STENCIL = 0
CG_SPECTRAL = 1
CG_SSTEP = 2
CG_GAUSS = 3


class BBSolver:
    """Device-resident Benamou-Brenier state (mu, q, phi stay in HBM between calls).

    Parameters mirror ``benamou_brenier.solve``; ``cg_mode`` picks the Poisson CG
    (0 = the literal 7-point stencil CG, 1 = the same CG run in the DCT-II eigenbasis of A,
    2 = that spectral CG in s-step passes of up to 8 iterations, 3 = scipy's CG recurrence on
    the Gauss-compressed spectral measure of b -- this class's default --, < 0 = auto, the default
    of the C ABI's foto_bb_opts_default and of the drop-in benamou_brenier.solve: 0 on grids of
    at most 2^18 voxels, 3 above);
    ``rank/world/nccl_id`` shard the time axis over processes (RCCL),
    ``virtual_ranks`` shards it in-process on one device (test path); ``library`` is a
    ``_lib.load``-ed build other than the product libfoto.so (tests).
    """

    def __init__(self, rho0, rhoT, Nt, Nx, Ny, r=1.0, reg_epsilon=1e-3, *, device=-1, cg_rtol=1e-6,
                 cg_maxiter=1000, cg_mode=CG_GAUSS, rank=0, world=1, nccl_id=None, virtual_ranks=1,
                 timing=False, library=None):
        self._L = library if library is not None else lib()
        Nt, Nx, Ny = int(Nt), int(Nx), int(Ny)
        if Nt < 2:
            raise ZeroDivisionError("Nt must be >= 2 (benamou_brenier.py:194 divides by Nt - 1)")
        self.Nt, self.Nx, self.Ny = Nt, Nx, Ny
        self.r = float(r)
        self.eps = float(reg_epsilon)
        nxy = Nx * Ny
        self._rho0 = f64(rho0, nxy, "rho0")
        self._rhoT = f64(rhoT, nxy, "rhoT")
        o = _lib.BBOpts()
        self._L.foto_bb_opts_default(ctypes.byref(o))
        o.device = int(device)
        o.cg_rtol = float(cg_rtol)
        o.cg_maxiter = int(cg_maxiter)
        o.cg_mode = int(cg_mode)
        o.rank = int(rank)
        o.world = int(world)
        self._id = None
        if nccl_id is not None:
            self._id = ctypes.create_string_buffer(bytes(nccl_id), 128)
            o.nccl_id = ctypes.cast(self._id, ctypes.c_void_p)
        o.virtual_ranks = int(virtual_ranks)
        o.timing = 1 if timing else 0
        self._ctx = ctypes.c_void_p()
        self._check(self._L.foto_bb_create(dptr(self._rho0), dptr(self._rhoT), Nt, Nx, Ny, self.r, self.eps,
                                   ctypes.byref(o), ctypes.byref(self._ctx)))
        self.world = int(world)
        self.rank = int(rank)
        self.crit = []
        self.cg_its = []
        self.cg_info = []

    def _check(self, rc):
        return check(rc, self._L)

    def reset(self, rho0, rhoT):
        """Start over on a new pair of the same size: the context's fields, CG state and
        predictions go back to what construction leaves (foto_bb_reset), so the solve is
        bit-identical to one on a fresh BBSolver, without its allocations and plans."""
        nxy = self.Nx * self.Ny
        self._rho0 = f64(rho0, nxy, "rho0")
        self._rhoT = f64(rhoT, nxy, "rhoT")
        self._check(self._L.foto_bb_reset(self._ctx, dptr(self._rho0), dptr(self._rhoT)))
        self.crit = []
        self.cg_its = []
        self.cg_info = []

    # -------------------------------------------------------------- lifecycle
    def close(self):
        if getattr(self, "_ctx", None) and self._ctx.value:
            self._L.foto_bb_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        if sys.is_finalizing():   # libfoto / HIP may already be torn down
            return
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -------------------------------------------------------------- iterations
    def iterate(self, n, convergence_tol=0.0, stop_rules=True, callback=None):
        """Run up to n outer iterations; returns True if a reference stop rule fired.
        ``callback(i, crit, cg_its, cg_info)`` is called after each iteration, while iteration
        i + 1 is already on the stream: in the default single-GPU loop ``phi()``, ``state()``
        and ``flow()`` called from it return iteration i's results; the one-in-flight loop
        (sharded contexts, FOTO_PIPE=0) raises FotoError for them there (foto.h)."""
        errors = []

        def _cb(user, it, crit, its, info):
            try:
                self.crit.append(crit)
                self.cg_its.append(its)
                self.cg_info.append(info)
                if callback is not None:
                    callback(it, crit, its, info)
            except BaseException as e:   # never let an exception unwind through C
                errors.append(e)

        cb = _lib.ITER_CB(_cb)
        done = ctypes.c_int(0)
        rc = self._L.foto_bb_iterate(self._ctx, int(n), float(convergence_tol), 1 if stop_rules else 0, cb, None,
                                   ctypes.byref(done))
        if errors:
            raise errors[0]
        self._check(rc)
        return rc == 1

    def flow(self):
        """(u, v, m) from the last phi (rank 0 gets the arrays; other ranks get None)."""
        nxy = self.Nx * self.Ny
        if self.world > 1 and self.rank != 0:
            self._check(self._L.foto_bb_flow(self._ctx, None, None, None))
            return None
        u = np.empty(nxy)
        v = np.empty(nxy)
        m = np.empty(nxy)
        self._check(self._L.foto_bb_flow(self._ctx, dptr(u), dptr(v), dptr(m)))
        return u, v, m

    def shard(self):
        t0 = ctypes.c_int()
        nl = ctypes.c_int()
        self._check(self._L.foto_bb_shard(self._ctx, ctypes.byref(t0), ctypes.byref(nl)))
        return t0.value, nl.value

    def comm_size(self):
        """Ranks of this context's RCCL communicator (ncclCommCount); 0 without one."""
        n = ctypes.c_int()
        self._check(self._L.foto_bb_comm_size(self._ctx, ctypes.byref(n)))
        return n.value

    def phi(self):
        _, nl = self.shard()
        out = np.empty(nl * self.Nx * self.Ny)
        self._check(self._L.foto_bb_get_phi(self._ctx, dptr(out)))
        return out

    def state(self):
        _, nl = self.shard()
        n = nl * self.Nx * self.Ny
        mu = np.empty(3 * n)
        q = np.empty(3 * n)
        self._check(self._L.foto_bb_get_state(self._ctx, dptr(mu), dptr(q)))
        return mu, q

    def stats(self):
        st = _lib.BBStats()
        self._check(self._L.foto_bb_stats_get(self._ctx, ctypes.byref(st)))
        d = {f: getattr(st, f) for f in ("outer_iters", "cg_iters_total", "last_crit", "ms_rhs", "ms_cg",
                                         "ms_prox", "ms_flow", "cg_redo")}
        d["kernels"] = {name: {"n": int(st.n_k[i]), "ms": float(st.ms_k[i]), "bytes": float(st.bytes_k[i])}
                        for i, name in enumerate(_lib.K_NAMES) if st.n_k[i] > 0}
        return d

    def reset_stats(self):
        self._check(self._L.foto_bb_stats_reset(self._ctx))

    def set_timing(self, on):
        self._check(self._L.foto_bb_set_timing(self._ctx, 1 if on else 0))

    def sync(self):
        self._check(self._L.foto_bb_sync(self._ctx))


# One context per (size, parameters) for a batch of same-size frames (run.sh:81-157 solves one
# pair per sequence): a context costs its HBM fields, DCT plans and a stream to build, and
# foto_bb_reset makes a reused one give the same bits as a fresh one.  FOTO_BB_CACHE=0 turns
# it off; sharded contexts (RCCL rank/world) and explicit libraries are never cached.
CONTEXT_CACHE_SIZE = 2
_ctx_cache = collections.OrderedDict()


def _cache_enabled(opts):
    if os.environ.get("FOTO_BB_CACHE", "1") == "0" or CONTEXT_CACHE_SIZE <= 0:
        return False
    return (opts.get("library") is None and opts.get("nccl_id") is None
            and int(opts.get("world", 1)) == 1)


def cached_solver(rho0, rhoT, Nt, Nx, Ny, r, reg_epsilon, **opts):
    """A BBSolver for this size and these options, reset to (rho0, rhoT): reused from the
    cache when one exists, else created (the least recently used context beyond
    CONTEXT_CACHE_SIZE is destroyed)."""
    # FOTO_* tuning variables are read when a context is built: part of its identity
    env = tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("FOTO_")))
    key = (int(Nt), int(Nx), int(Ny), float(r), float(reg_epsilon), tuple(sorted(opts.items())), env)
    s = _ctx_cache.pop(key, None)
    if s is not None:
        s.reset(rho0, rhoT)
    else:
        s = BBSolver(rho0, rhoT, Nt, Nx, Ny, r=r, reg_epsilon=reg_epsilon, **opts)
    _ctx_cache[key] = s
    while len(_ctx_cache) > CONTEXT_CACHE_SIZE:
        _ctx_cache.popitem(last=False)[1].close()
    return s


def clear_context_cache():
    while _ctx_cache:
        _ctx_cache.popitem()[1].close()


def solve(rho0, rhoT, Nt, Nx, Ny, r=1, convergence_tol=0.3, reg_epsilon=1e-3, max_it=100, *, log=print,
          stats=None, **opts):
    """benamou_brenier.solve on the GPU.  Returns (u, v, m)."""
    if max_it <= 0:
        # reference: the loop body never runs and `phi` is unbound at benamou_brenier.py:271
        raise UnboundLocalError("cannot access local variable 'phi' where it is not associated with a value")

    def cb(it, crit, its, info):
        if info > 0:
            log(f"WARNING: CG did not converge in {info} iterations.")
        log(str(np.float64(crit)) + " (" + str(it + 1) + "/" + str(max_it) + ")")

    if _cache_enabled(opts):
        s = cached_solver(rho0, rhoT, Nt, Nx, Ny, r, reg_epsilon, **opts)
        try:
            return _run(s, max_it, convergence_tol, cb, stats)
        except BaseException:   # a failed solve leaves no half-used context behind
            for k, v in list(_ctx_cache.items()):
                if v is s:
                    del _ctx_cache[k]
            s.close()
            raise
    with BBSolver(rho0, rhoT, Nt, Nx, Ny, r=r, reg_epsilon=reg_epsilon, **opts) as s:
        return _run(s, max_it, convergence_tol, cb, stats)


def solve_ex(rho0, rhoT, Nt, Nx, Ny, r=1, convergence_tol=0.3, reg_epsilon=1e-3, max_it=100, *, cap=None,
             want_phi=True, device=-1, cg_mode=CG_GAUSS, cg_rtol=1e-6, cg_maxiter=1000, rank=0, world=1,
             nccl_id=None, virtual_ranks=1, timing=False, library=None):
    """benamou_brenier.solve through the one-shot C entry foto_bb_solve_ex (include/foto.h; the
    SURVEY.md §8(b) boundary): a context made, iterated with the reference's stop rules, the flow
    extracted and the context destroyed in one call.  Returns (u, v, m, report): report holds the
    per-outer-iteration crit / cg_its / cg_info (the first ``cap`` of them, default max_it), phi
    (this rank's slab) and the timings and byte counts of foto_bb_solve_stats.  With world > 1
    every rank calls it; (u, v, m) are None off rank 0."""
    L = library if library is not None else lib()
    Nt, Nx, Ny = int(Nt), int(Nx), int(Ny)
    nxy = Nx * Ny
    a0, aT = f64(rho0, nxy, "rho0"), f64(rhoT, nxy, "rhoT")
    o = _lib.BBOpts()
    L.foto_bb_opts_default(ctypes.byref(o))
    o.device, o.cg_mode, o.cg_rtol, o.cg_maxiter = int(device), int(cg_mode), float(cg_rtol), int(cg_maxiter)
    o.rank, o.world, o.virtual_ranks, o.timing = int(rank), int(world), int(virtual_ranks), 1 if timing else 0
    idbuf = None
    if nccl_id is not None:
        idbuf = ctypes.create_string_buffer(bytes(nccl_id), 128)
        o.nccl_id = ctypes.cast(idbuf, ctypes.c_void_p)
    cap = int(max_it if cap is None else cap)
    crit = np.zeros(max(cap, 1))
    its = np.zeros(max(cap, 1), dtype=np.int32)
    info = np.zeros(max(cap, 1), dtype=np.int32)
    st = _lib.BBSolveStats()
    st.cap = cap
    st.crit = dptr(crit)
    st.cg_its = its.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    st.cg_info = info.ctypes.data_as(ctypes.POINTER(ctypes.c_int))
    on0 = int(world) == 1 or int(rank) == 0
    u, v, m = (np.empty(nxy) for _ in range(3)) if on0 else (None, None, None)
    # the largest slab a rank can hold (split_planes: balanced), or every plane on one GPU
    phi = np.empty(-(-Nt // max(int(world), 1)) * nxy) if want_phi else None
    null = _lib._D()
    check(L.foto_bb_solve_ex(dptr(a0), dptr(aT), Nt, Nx, Ny, float(r), float(convergence_tol), float(reg_epsilon),
                             int(max_it), ctypes.byref(o), dptr(u) if on0 else null, dptr(v) if on0 else null,
                             dptr(m) if on0 else null, dptr(phi) if want_phi else null, ctypes.byref(st)), L)
    n = min(st.outer_iters, cap)
    rep = {"outer_iters": st.outer_iters, "stopped": bool(st.stopped), "crit": crit[:n].copy(),
           "cg_its": its[:n].astype(np.int64), "cg_info": info[:n].astype(np.int64),
           "phi_t0": st.phi_t0, "phi_nloc": st.phi_nloc, "ms_create": st.ms_create, "ms_loop": st.ms_loop,
           "ms_flow": st.ms_flow, "alg_bytes_per_iter": st.alg_bytes_per_iter,
           "cg_iters_total": int(st.bb.cg_iters_total), "cg_redo": int(st.bb.cg_redo),
           "kernels": {name: {"n": int(st.bb.n_k[i]), "ms": float(st.bb.ms_k[i]), "bytes": float(st.bb.bytes_k[i])}
                       for i, name in enumerate(_lib.K_NAMES) if st.bb.n_k[i] > 0}}
    if want_phi:
        rep["phi"] = phi[:st.phi_nloc * nxy].copy()
    return u, v, m, rep


def _run(s, max_it, convergence_tol, cb, stats):
    s.iterate(max_it, convergence_tol=convergence_tol, stop_rules=True, callback=cb)
    out = s.flow()
    if stats is not None:
        stats.update(crit=np.array(s.crit), cg_its=np.array(s.cg_its), cg_info=np.array(s.cg_info),
                     phi=s.phi(), **s.stats())
    return out
