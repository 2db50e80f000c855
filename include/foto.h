/*
 * libfoto -- MI355X-native FOTO hot path (Benamou-Brenier dynamic-OT optical flow
 * solver + the Gennert-Negahdaripour variational baseline) behind a plain C ABI.
 *
 * Every entry point takes caller-owned HOST buffers (float64, row-major, the layout
 * of the reference: voxel k = n*Nx*Ny + j*Nx + i, 3-field vectors SoA
 * [t-part; x-part; y-part]) and returns 0 on success, < 0 on error
 * (foto_last_error() has the message).  Each declaration cites the reference
 * interface it replaces (paths relative to the reference repository root).
 *
 * The reference is pure Python (numpy/scipy); its "FFI" for this path is the
 * Python call surface.  The binding a maintainer adds is the ctypes layer in
 * optical-flow-optimal-transport_amd/foto/_lib.py.
 */
#ifndef FOTO_H
#define FOTO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FOTO_OK 0
#define FOTO_ERR_ARG (-1)     /* bad sizes / arguments (reference: IndexError, ZeroDivisionError) */
#define FOTO_ERR_HIP (-2)     /* HIP runtime error (no device, OOM, launch failure)              */
#define FOTO_ERR_COMM (-3)    /* RCCL error                                                      */
#define FOTO_ERR_STATE (-4)   /* call out of order (e.g. flow before any iteration)              */
#define FOTO_ERR_BC (-5)      /* boundary condition not in {'N','D'}: NotImplementedError        */

const char* foto_last_error(void);
int foto_version(void);
int foto_device_count(int* n);

/* ------------------------------------------------------------------ operators
 * Matrix-free applications of the sparse operators of operators.py (h = 1).   */

/* operators.grad_st(Nt,Nx,Ny,1,1,1,'N') @ phi  (operators.py:114-127)       -> out3[3N] */
int foto_grad_st(const double* phi, int Nt, int Nx, int Ny, double* out3);
/* operators.div_st(Nt,Nx,Ny,1,1,1,'N') @ w3    (operators.py:129-142)       -> out[N]   */
int foto_div_st(const double* w3, int Nt, int Nx, int Ny, double* out);
/* operators.laplacian_st(Nt,Nx,Ny,1,1,1,'N') @ p (operators.py:144-157)     -> out[N]   */
int foto_laplacian_st(const double* p, int Nt, int Nx, int Ny, double* out);
/* (-r*L_st + r*eps*I) @ p                      (benamou_brenier.py:202-203) -> out[N]   */
int foto_apply_A(const double* p, int Nt, int Nx, int Ny, double r, double eps, double* out);
/* operators.grad(Nx,Ny,1,1,bc) @ f             (operators.py:160-169)       -> out2[2*Nx*Ny] */
int foto_grad2(const double* f, int Nx, int Ny, char bc, double* out2);
/* operators.div(Nx,Ny,1,1,bc) @ [u;v]          (operators.py:182-191)       -> out[Nx*Ny] */
int foto_div2(const double* uv, int Nx, int Ny, char bc, double* out);
/* operators.grad_forward(Nx,Ny,1,1,'N') @ f    (operators.py:171-180)       -> out2[2*Nx*Ny] */
int foto_grad2_forward(const double* f, int Nx, int Ny, double* out2);

/* ------------------------------------------------------------------ BB building blocks */

/* benamou_brenier.stepB(p, ...)  (benamou_brenier.py:93-149); M = Nt*Nx*Ny        */
int foto_stepB(const double* p3, int64_t M, double* q3);
/* RHS of solve_benamou_brenier_step: div_st(mu - r q) + temporal BC correction
 * (benamou_brenier.py:64-82)                                                       */
int foto_bb_rhs(const double* mu3, const double* q3, const double* rho0, const double* rhoT,
                int Nt, int Nx, int Ny, double r, double* F);
/* scipy.sparse.linalg.cg(A, b, rtol, maxiter) with A = -r L_st + r eps I, x0 = 0
 * (benamou_brenier.py:85).  Returns info (0 converged, maxiter otherwise) or < 0;
 * *iterations = CG iterations run.  mode: 0 = stencil CG, 1 = spectral CG,
 * 2 = spectral s-step CG, 3 = Gauss-compressed spectral CG (foto_bb_opts.cg_mode). */
int foto_cg(const double* b, int Nt, int Nx, int Ny, double r, double eps, double rtol, int maxiter,
            int mode, double* x, int* iterations);
/* utils.opticalflow_from_benamoubrenier(phi, Nt, Nx, Ny, grad('N'), div('D'))
 * (utils.py:44-99, 148-183)                                                        */
int foto_flow_from_phi(const double* phi, int Nt, int Nx, int Ny, double* u, double* v, double* m);

/* ------------------------------------------------------------------ BB solver context
 * benamou_brenier.solve (benamou_brenier.py:151-271) split into create / iterate /
 * flow so a caller can keep the state resident in HBM between calls.             */
typedef struct foto_bb_ctx foto_bb_ctx;

typedef struct {
    int device;           /* HIP device ordinal; -1 = current device                       */
    int cg_maxiter;       /* 1000 (benamou_brenier.py:85)                                  */
    double cg_rtol;       /* 1e-6 (benamou_brenier.py:85)                                  */
    int cg_mode;          /* 0 = stencil CG (7-point matvec), 1 = spectral CG (DCT-II      */
                          /* eigenbasis, one pass / iteration), 2 = spectral s-step CG     */
                          /* (one pass / up to 8 iterations, any world; mode 1 needs       */
                          /* world == 1; eps <= 0 selects mode 0), 3 = spectral CG on the  */
                          /* Gauss-compressed measure of b^ (one read of b^, the           */
                          /* recurrence on 2048 nodes, any world); < 0 = auto (default):   */
                          /* 0 on grids of <= 2^18 voxels (FOTO_CG_AUTO_MAX), 3 above      */
    int rank, world;      /* time-slab sharding over `world` processes (RCCL); 1 = single  */
    const void* nccl_id;  /* 128-byte ncclUniqueId (foto_nccl_unique_id on rank 0)         */
    int virtual_ranks;    /* >1: shard over this many in-process slabs on ONE device       */
                          /* (tests the sharded path without RCCL; world must be 1)       */
    int timing;           /* 1: time every kernel launch with HIP events (foto_bb_stats)   */
} foto_bb_opts;

/* per outer iteration: crit and the CG iteration count / info of that stepA */
typedef void (*foto_bb_iter_cb)(void* user, int iter, double crit, int cg_iters, int cg_info);

typedef struct {
    int outer_iters;          /* outer iterations completed so far                      */
    int64_t cg_iters_total;   /* CG iterations over all outer iterations                */
    double last_crit;
    double ms_rhs, ms_cg, ms_prox, ms_flow;   /* phase wall time (HIP events; RHS / CG / prox
                                                 only with timing = 1)                   */
    /* per kernel class (timing = 1): launches and summed device time in ms            */
    int64_t n_k[8];
    double ms_k[8];
    double bytes_k[8];        /* algorithmic HBM bytes of those launches, summed        */
    int cg_redo;              /* outer iterations whose deferred CG solve (see foto_bb.cpp) */
                              /* outran its predicted passes and re-ran prox             */
} foto_bb_stats;

/* kernel classes reported in foto_bb_stats.n_k / ms_k / bytes_k */
#define FOTO_K_CG_DIR    0   /* stencil CG: p = r + beta p, A p, p.Ap                    */
#define FOTO_K_CG_UPD    1   /* stencil CG: x += alpha p, r -= alpha A p, r.r            */
#define FOTO_K_RHS       2   /* div_st(mu - r q) + BC                                    */
#define FOTO_K_PROX      3   /* grad_st phi, stepB, mu update, crit sums                 */
#define FOTO_K_SPEC      4   /* spectral CG iteration kernel(s)                          */
#define FOTO_K_DCT       5   /* DCT-II transforms                                        */
#define FOTO_K_FLOW      6   /* trajectory integration + divergence                      */
#define FOTO_K_SLAB      7   /* sharded: the slab-side x / y DCTs (what the pipelined     */
                             /* all-to-alls overlap with communication)                  */
#define FOTO_K_OTHER     FOTO_K_SLAB   /* (older name)                                    */

int foto_bb_opts_default(foto_bb_opts* o);
int foto_bb_create(const double* rho0, const double* rhoT, int Nt, int Nx, int Ny, double r,
                   double reg_epsilon, const foto_bb_opts* opts, foto_bb_ctx** out);
/* Run up to `max_iters` outer iterations (stepA + stepB + stepC + criterion).  With
 * use_stop_rules = 1 it stops like the reference (crit <= tol, or |dcrit| < 1e-5).
 * cb (may be NULL) gets (iteration index, crit, CG iterations, CG info) after each
 * outer iteration.  Returns 1 if a stop rule fired, 0 otherwise, < 0 on error.
 * The callback runs while the NEXT outer iteration is already on the stream.  In the
 * default single-GPU loop (two iterations in flight) foto_bb_get_phi / get_state / flow
 * called from it return the state of the iteration the callback reports (kept intact for a
 * rollback); the one-in-flight loop (sharded, FOTO_PIPE=0) refuses them there with
 * FOTO_ERR_STATE (its next solve overwrites phi).  An error with iterations in flight drains
 * the stream and leaves the context refusing iterate / flow until foto_bb_reset.
 * foto_bb_reset and a nested foto_bb_iterate from the callback return FOTO_ERR_STATE.   */
int foto_bb_iterate(foto_bb_ctx* c, int max_iters, double convergence_tol, int use_stop_rules,
                    foto_bb_iter_cb cb, void* user, int* iters_done);
/* Flow (u, v, m) from the last phi: utils.opticalflow_from_benamoubrenier.
 * With world > 1 the result lands on rank 0; other ranks may pass NULL.           */
int foto_bb_flow(foto_bb_ctx* c, double* u, double* v, double* m);
/* A new pair (rho0, rhoT) of the same size on an existing context: every field, counter and
 * prediction back to what foto_bb_create leaves, so the solve is bit-identical to one on a
 * fresh context -- without its allocations, DCT plans and stream (a batch of same-size
 * frames: run.sh:81-157 runs one solve per sequence).  Also the way back after a failed
 * foto_bb_iterate (whatever it left on the stream is drained first).                     */
int foto_bb_reset(foto_bb_ctx* c, const double* rho0, const double* rhoT);
/* Copy this shard's slab range of phi / mu / q to host (t0, nloc via foto_bb_shard). */
int foto_bb_get_phi(foto_bb_ctx* c, double* phi);
int foto_bb_get_state(foto_bb_ctx* c, double* mu3, double* q3);
int foto_bb_shard(const foto_bb_ctx* c, int* t0, int* nloc);
/* Ranks of the context's RCCL communicator (ncclCommCount); 0 for a context without one (one
 * GPU, or virtual ranks in one process).                                                   */
int foto_bb_comm_size(const foto_bb_ctx* c, int* nranks);
int foto_bb_stats_get(const foto_bb_ctx* c, foto_bb_stats* st);
int foto_bb_stats_reset(foto_bb_ctx* c);
/* enable / disable per-launch HIP-event timing (foto_bb_stats.n_k / ms_k) */
int foto_bb_set_timing(foto_bb_ctx* c, int on);
int foto_bb_sync(foto_bb_ctx* c);
void foto_bb_destroy(foto_bb_ctx* c);

/* One-shot benamou_brenier.solve(rho0, rhoT, Nt, Nx, Ny, r, convergence_tol,
 * reg_epsilon, max_it) -> (u, v, m) on one GPU.                                     */
int foto_bb_solve(const double* rho0, const double* rhoT, int Nt, int Nx, int Ny, double r,
                  double convergence_tol, double reg_epsilon, int max_it, foto_bb_iter_cb cb, void* user,
                  double* u, double* v, double* m);

/* Per-solve report of foto_bb_solve_ex (outer iterations, the per-iteration
 * crit and CG counts, per-phase time and HBM bytes).  The caller owns the three arrays (any may
 * be NULL) and sets cap to their length; entries beyond cap are counted but not stored.       */
typedef struct {
    int cap;                  /* in: length of crit / cg_its / cg_info                        */
    double* crit;             /* out: crit of outer iteration i (benamou_brenier.py:249)       */
    int* cg_its;              /* out: CG iterations of that stepA (scipy cg at :85)           */
    int* cg_info;             /* out: CG info (0 converged, maxiter otherwise; :86-87 warning) */
    int outer_iters;          /* out: outer iterations run                                    */
    int stopped;              /* out: 1 if a stop rule ended the run (:253-258)               */
    int phi_t0, phi_nloc;     /* out: the time planes phi_or_null received (this rank's slab) */
    double ms_create;         /* out: host wall time of context creation (uploads, plans)     */
    double ms_loop;           /* out: host wall time of the outer-iteration loop (the metric) */
    double ms_flow;           /* out: host wall time of the flow extraction + download        */
    double alg_bytes_per_iter;/* out: algorithmic HBM bytes of one outer iteration on this
                                 rank (188 B per voxel for the default path)     */
    foto_bb_stats bb;         /* out: the context's counters (kernel classes with opts.timing) */
} foto_bb_solve_stats;

/* One-shot benamou_brenier.solve (benamou_brenier.py:151-271) with the options of a context
 * (opts may be NULL: foto_bb_opts_default; opts->world > 1: this process is rank opts->rank of
 * a time-slab sharded solve over RCCL -- config 4 -- and every rank calls it with the same
 * arguments), the reference's stop rules, and the per-solve report above.  (u, v, m) land on
 * rank 0 (other ranks may pass NULL); phi_or_null gets this rank's slab of the last phi
 * (st->phi_t0, st->phi_nloc planes; all Nt planes on one GPU).  st may be NULL.  Returns 0,
 * or < 0 on error; CG non-convergence is reported in st->cg_info (a warning, not an error). */
int foto_bb_solve_ex(const double* rho0, const double* rhoT, int Nt, int Nx, int Ny, double r,
                     double convergence_tol, double reg_epsilon, int max_it, const foto_bb_opts* opts,
                     double* u, double* v, double* m, double* phi_or_null, foto_bb_solve_stats* st);

/* RCCL unique id for foto_bb_opts.nccl_id (call on rank 0, broadcast 128 bytes). */
int foto_nccl_unique_id(void* out128);

/* Test entry (host only, no device): the point-to-point calls rank `rank` of `world` issues
 * over RCCL for one exchange of the time-sharded solve (the loop of benamou_brenier.py:204-258
 * split into time slabs), in issue order.  Each call is 5 int64:
 * {op (FOTO_CALL_*), peer, offset, count, copy destination offset}, offsets in doubles from
 * the buffer the exchange picks (send / copy: source; recv: destination).  Sends and receives
 * go in one ncclGroupStart/End; copies follow the group.  arg: the relay step j (RELAY).    */
#define FOTO_XFER_HALO 0          /* halo planes of a slab field (plane -1 / nloc)            */
#define FOTO_XFER_SLAB_TO_BOX 1   /* spectral all-to-all: time slabs -> row boxes             */
#define FOTO_XFER_BOX_TO_SLAB 2   /* spectral all-to-all: row boxes -> time slabs             */
#define FOTO_XFER_RELAY 3         /* trajectory positions rank j -> j + 1 (flow extraction)   */
#define FOTO_XFER_DELIVER 4       /* (u, v, m) last rank -> rank 0                            */
#define FOTO_XFER_HALO2 5         /* two halo planes per side (phi of the fused prox + RHS)   */
/* the pipelined all-to-alls: arg = part | parts << 8 | halo << 16 (foto_xfer.h
 * alltoall_part_xfers; the backward one with halo = 1 also delivers phi's halo planes)       */
#define FOTO_XFER_SLAB_TO_BOX_PART 6
#define FOTO_XFER_BOX_TO_SLAB_PART 7
#define FOTO_CALL_SEND 0
#define FOTO_CALL_RECV 1
#define FOTO_CALL_COPY 2
int foto_xfer_calls(int kind, int Nt, int Ny, int Nx, int world, int rank, int arg, int64_t* out, int cap,
                    int* count);

/* Test entry: the orthonormal DCT-II (inverse = 0) or DCT-III (inverse = 1) along the middle
 * axis of a C-order [outer][n][inner] array, as scipy.fft.dct(x, type=2|3, norm="ortho",
 * axis=1) -- the transform pair that diagonalises lap1d (operators.py:33-48) in the spectral
 * CG.  path 0: the FFT kernels when n has a plan, else the MFMA GEMM kernels; 1: FFT only
 * (error without a plan); 2: GEMM only.                                            */
int foto_dct(const double* in, int outer, int n, int inner, int inverse, int path, double* out);

/* Measurement entry (bench.py): the dominant s-step pass's memory traffic alone -- read and
 * write two n-double vectors, 16 B per lane, no arithmetic beyond one update -- timed over
 * `reps` back-to-back launches on this device; us[0] plain stores, us[1] write-through (sc1)
 * stores, microseconds per launch (best of 3).  n even, n * 8 < 2^31.                   */
int foto_stream_probe(int64_t n, int reps, double* us);

/* Measurement entry (bench.py): the fused prox + RHS kernel's traffic alone -- read four
 * n-double fields, write four others (64 B per voxel, the working set well beyond the
 * Infinity Cache at the bench size), one update per element -- microseconds per launch
 * (best of 3 over `reps` launches) in us[0].  n even.                                      */
int foto_stream_probe4(int64_t n, int reps, double* us);

/* ------------------------------------------------------------------ GN baseline
 * classical.GLLOpticalFlow (classical.py:25-130).                                 */
/* assemble(f1, f2).A @ x and .b (classical.py:68-111)                             */
int foto_gn_apply(const double* f1, const double* f2, int w, int h, double alpha, double lambda_,
                  const double* x3, double* y3);
int foto_gn_rhs(const double* f1, const double* f2, int w, int h, double* b3);
/* process(): spsolve replaced by CG preconditioned by one multigrid V-cycle (damped
 * block-Jacobi smoothing on each level; FOTO_GN_MG=0: the plain 3x3 block-Jacobi PCG) to rtol
 * (default 1e-10).
 * Returns 0 (converged) or maxiter (not converged), < 0 on error.  Runs on a plan (below)
 * cached per process for the last (w, h, alpha, lambda, rtol, maxiter, device), as FFT
 * libraries cache plans; FOTO_GN_PLAN_CACHE=0 makes and destroys one per call.       */
int foto_gn_solve(const double* f1, const double* f2, int w, int h, double alpha, double lambda_,
                  double rtol, int maxiter, double* u, double* v, double* m, int* iterations);

/* Per-solve report of foto_gn_solve_ex (SURVEY.md §8(b) foto_gn_stats).                      */
typedef struct {
    int iterations;           /* PCG iterations run                                            */
    int info;                 /* 0 converged, maxiter otherwise (the return value)             */
    int plan_reused;          /* 1: the cached plan of the previous call served this one       */
    int levels;               /* multigrid levels of the preconditioner                        */
    double ms_setup;          /* device time: upload, coefficients, RHS, V-cycle of r0          */
    double ms_pcg;            /* device time of the PCG iterations                             */
    double ms_total;          /* host wall time of the call                                    */
    double alg_bytes_per_iter;/* algorithmic HBM bytes of one PCG iteration   */
} foto_gn_stats;

/* foto_gn_solve with the report above (st may be NULL).                                      */
int foto_gn_solve_ex(const double* f1, const double* f2, int w, int h, double alpha, double lambda_,
                     double rtol, int maxiter, double* u, double* v, double* m, foto_gn_stats* st);

/* A reusable GLLOpticalFlow(w, h) with setAlpha/setLambda applied (classical.py:25-66): device
 * buffers, the multigrid hierarchy and the replayed PCG graph are made once; every
 * foto_gn_plan_solve is one process(f1, f2) (classical.py:68-130: coefficients, right-hand
 * side, multigrid coefficients, PCG) with the same result and return codes as foto_gn_solve.
 * Batches of same-size pairs (run.sh:81-157) reuse one plan.                       */
typedef struct foto_gn_plan foto_gn_plan;
int foto_gn_plan_create(int w, int h, double alpha, double lambda_, double rtol, int maxiter, foto_gn_plan** out);
int foto_gn_plan_solve(foto_gn_plan* p, const double* f1, const double* f2, double* u, double* v, double* m,
                       int* iterations);
/* the last solve: {ms upload + setup + V-cycle of r0, ms PCG iterations (device events),
 * iterations, iterations launched}                                                */
int foto_gn_plan_timing(const foto_gn_plan* p, double* out4);
/* the device the plan was made on (-1 for NULL)                                    */
int foto_gn_plan_device(const foto_gn_plan* p);
void foto_gn_plan_destroy(foto_gn_plan* p);

/* ------------------------------------------------------------------ evaluation
 * the warp and the error metrics of utils.py on the GPU.      */
/* utils.apply_opticalflow(f1, u, v, w, h, m) (utils.py:186-248): backward bilinear
 * warp of (1 + m) f1 (m may be NULL: f1 unscaled).  Bit-identical to the reference. */
int foto_warp(const double* f1, const double* u, const double* v, const double* m, int w, int h, double* out);
/* utils.EE and utils.AE (utils.py:294-338): out4 = {AEE, SDEE, AAE, SDAE}; EE > 50 and
 * NaN angular errors are ignored as in the reference.                               */
int foto_flow_errors(const double* u, const double* v, const double* uGT, const double* vGT, int w, int h,
                     double* out4);
/* utils.IE (utils.py:340-354): RMS of 255 I - 255 IGT.                              */
int foto_intensity_error(const double* I, const double* IGT, int w, int h, double* ie);

#ifdef __cplusplus
}
#endif
#endif /* FOTO_H */
