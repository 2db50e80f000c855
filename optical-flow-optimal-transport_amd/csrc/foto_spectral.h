// Spectral (DCT-II basis) CG for A = -r L_st + r eps I.  See foto_spectral.hip.
#pragma once
#include "foto_internal.h"

namespace foto {

struct SpectralPlan {
    // rank / world: the shard's place in the time-slab decomposition (world > 1 needs
    // sstep = 2; the spectral box of rank g is rows [y0, y0 + nyl) of every kt plane).
    int init(const Geo& g, int rank, int world, double r, double eps, int sstep, hipStream_t s);
    // single shard: b (physical, clobbered) -> x (physical); scipy stopping rule.
    int solve(double* b, double* x, double rtol, int maxiter, int predicted, int* iters, int* info, KTimer* kt,
              hipStream_t s);
    // Deferred variant (single shard, s-step, after a first solve has set the pass count):
    // enqueues the predicted passes and the inverse transforms without waiting; the state
    // travels to a pinned copy behind them.  done_flag() is the device flag a consumer can
    // guard on.  After the caller's stream sync, finish() reports the result; if the passes
    // did not suffice (*redo = 1) it runs the rest of the solve, polling, and recomputes x.
    // The Gauss CG takes up to two deferred solves in flight (two outer iterations on the
    // stream, foto_bb.cpp): finish() completes the oldest; a failed oldest solve (see
    // oldest_needs_redo) is redone only after the newer one has been dropped (drop_newest,
    // after a stream sync) -- its done flag chain kept that one's consumer from running.
    bool deferrable() const;
    int solve_deferred(double* b, double* x, double rtol, int maxiter, KTimer* kt, hipStream_t s);
    const int* done_flag() const;
    int finish(int* iters, int* info, int* redo, KTimer* kt, hipStream_t s);
    int pending() const;
    bool oldest_needs_redo() const;   // after the stream has passed the oldest solve's header store
    int drop_newest(hipStream_t s);

    // ---- sharded phases (driven by foto_bb.cpp, all-to-all / all-gather in between)
    // x, y DCT of own planes [lo, hi), in place in b (the all-to-all's source)
    int fwd_local(double* b, int lo, int hi, KTimer* kt, hipStream_t s);
    int fwd_t(KTimer* kt, hipStream_t s);                   // box_in (after all-to-all) -> b^
    int cg_begin(double rtol, int maxiter, KTimer* kt, hipStream_t s);   // r^ = b^, moments -> gath
    int cg_pass(double rtol, int maxiter, KTimer* kt, hipStream_t s);    // planned CG steps, moments -> gath
    int cg_plan(int init, double rtol, int maxiter, hipStream_t s);      // after the all-gather
    int poll(int* done, int* iters, int* passes, hipStream_t s);
    int inv_t(KTimer* kt, hipStream_t s);                   // x^ = (b^ - r^)/lam, inverse t-DCT -> box_out
    // inverse y, x of planes [lo, hi) of scratch (the all-to-all's target) -> x; lo = -1 / hi =
    // nloc + 1: the halo plane below / above too (scratch and x halo-padded)
    int inv_local(double* scratch, double* x, int lo, int hi, KTimer* kt, hipStream_t s);
    double* box_in() const;    // box-side receive buffer [t][rows][x]
    double* box_out() const;   // box-side send buffer of the inverse
    double* gath() const;      // world * moments() doubles
    static int moments();
    int y0() const;
    int nyl() const;

    // ---- Gauss-compressed CG (cg_mode 3), sharded phases: fwd_t (plain t-DCT), gauss_measure
    // (this box's histogram -> gauss_hist() slot rank), all-gather of gauss_hist_size() doubles,
    // gauss_solve, gauss_wait (host sync; !ok: redo with cg_begin / cg_pass from b^), inv_t, ...
    bool gauss() const;
    static int gauss_hist_size();
    double* gauss_hist() const;
    int gauss_measure(KTimer* kt, hipStream_t s);
    int gauss_solve(double rtol, int maxiter, KTimer* kt, hipStream_t s);
    int gauss_wait(int maxiter, int* ok, int* iters, int* info, hipStream_t s);
    // gauss_wait without the sync (the caller has waited past the solve's header copy); ends the
    // Gauss solve either way (!ok: the caller redoes it with the s-step CG)
    int gauss_result(int maxiter, int* ok, int* iters, int* info, hipStream_t s);
    void gauss_end();

    // back to the state init() leaves (no solve in flight, no pass-count prediction, the
    // whole-spectrum interval): a reused context solves a new pair exactly as a fresh one would
    int reset(hipStream_t s);

    ~SpectralPlan();
    void* impl = nullptr;
};

}  // namespace foto
