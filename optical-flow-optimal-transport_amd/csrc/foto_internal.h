// Internal declarations shared by the libfoto translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/foto.h"

namespace foto {

// ----------------------------------------------------------------------------- errors
void set_error(const char* fmt, ...);

#define FOTO_HIP_CHECK(call)                                                                  \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess) {                                                              \
            ::foto::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
            return FOTO_ERR_HIP;                                                             \
        }                                                                                    \
    } while (0)

#define FOTO_TRY(expr)          \
    do {                        \
        int rc_ = (expr);       \
        if (rc_ < 0) return rc_; \
    } while (0)

// ----------------------------------------------------------------------------- streams
// Streams come from a process-wide pool (foto_bb.cpp): a hipStreamCreate costs ~10 ms on the
// MI355X box (FOTO_GN_TRACE), which every BB context, GN plan and per-call scope paid -- a
// batch of solves paid it per solve.  acquire returns a stream of the current device; release
// takes back a stream with no work pending (callers synchronise first).  Never destroyed.
int stream_acquire(hipStream_t* out);
void stream_release(hipStream_t s);
int stream_device(hipStream_t s);   // the device a pooled stream belongs to (-1: not pooled)

// ----------------------------------------------------------------------------- geometry
// One time-slab shard of the (Nt, Ny, Nx) grid: local planes l in [0, nloc) are global
// planes t0 + l.  Every field array is allocated with one halo plane below (l = -1) and
// one above (l = nloc); the device pointer handed to kernels points at local plane 0.
struct Geo {
    int Nt, Ny, Nx;
    int t0, nloc;
    int64_t nxy;
};

constexpr int TX = 64;   // march tile width  (one wave = one 64-voxel x-row, 512 B of fp64)
constexpr int TY = 4;    // march tile height (4 waves, 256 threads)
constexpr int NT = 256;  // threads per block for every kernel

inline int march_blocks(const Geo& g) { return ((g.Nx + TX - 1) / TX) * ((g.Ny + TY - 1) / TY); }
inline int flat_blocks(int64_t n) { return (int)((n + NT - 1) / NT); }

// Device-side CG scalars (one per shard).  Written only by the last block of a kernel
// (or by block 0 for the done flag); read by later kernels.
struct CGScal {
    double bb;     // b.b
    double atol;   // rtol * ||b||
    double rho;    // r_k . r_k of the current iteration (scipy's rho_cur)
    double pap;    // p_k . A p_k
    int done;      // converged (top-of-iteration test passed) or b == 0
    int iters;     // iteration index at which `done` was set
    int pad[2];
};

// Per-shard reduction scratch: `partials` holds one value per block per quantity,
// `ticket` is the last-block counter, `gath` holds one slot per rank (allgathered).
struct RedBuf {
    double* partials;
    unsigned* ticket;
    int cap;   // blocks * quantities capacity
};

// ----------------------------------------------------------------------------- per-launch timing

struct KTimer {
    bool on = false;
    std::vector<hipEvent_t> pool;
    struct Pend { hipEvent_t a, b; int cls; double bytes; size_t id; };
    std::vector<Pend> pend;
    int64_t n[8] = {0};
    double ms[8] = {0};
    double bytes[8] = {0};

    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        // timing only, no system-scope fence: a fenced record writes the L2's dirty lines back
        // before the next launch, which the untimed loop never does -- the launch after it then
        // ran on a clean L2 (k_prox_rhs 171 us against 179.5 in the loop; FOTO_KT_FENCE=1: fenced)
        static const bool fence = [] {
            const char* f = getenv("FOTO_KT_FENCE");
            return f && atoi(f) == 1;
        }();
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, fence ? hipEventDefault : hipEventDisableSystemFence) != hipSuccess)
            return nullptr;
        return e;
    }
    // returns the start event to be paired by stop()
    hipEvent_t start(hipStream_t s) {
        if (!on) return nullptr;
        hipEvent_t e = get();
        if (e) (void)hipEventRecord(e, s);
        return e;
    }
    void stop(hipEvent_t a, hipStream_t s, int cls, double by) {
        if (!on || !a) return;
        hipEvent_t b = get();
        if (!b) return;
        (void)hipEventRecord(b, s);
        pend.push_back({a, b, cls, by, next_id++});
    }
    // drop the `count` most recent pending records of class cls (launches that turned out to
    // be no-ops, e.g. s-step passes enqueued after the solve had finished)
    void discard_last(int cls, int count) {
        for (int i = (int)pend.size() - 1; i >= 0 && count > 0; --i) {
            if (pend[i].cls != cls) continue;
            pool.push_back(pend[i].a);
            pool.push_back(pend[i].b);
            pend.erase(pend.begin() + i);
            --count;
        }
    }
    // marks are record ids (records are pushed in id order; ids survive discard_last)
    size_t next_id = 0;
    size_t mark() const { return next_id; }
    size_t count_before(size_t m) const {
        size_t n = 0;
        while (n < pend.size() && pend[n].id < m) ++n;
        return n;
    }
    // drop every record from mark m on (launches of an outer iteration that was rolled back)
    void discard_from(size_t m) {
        const size_t keep = count_before(m);
        for (size_t k = keep; k < pend.size(); ++k) {
            pool.push_back(pend[k].a);
            pool.push_back(pend[k].b);
        }
        pend.resize(keep);
    }
    // the pending intervals before mark m (all complete: recorded before the last stream sync)
    void resolve_upto(size_t m) { resolve_first(count_before(m)); }
    void resolve_first(size_t n) {
        n = std::min(n, pend.size());
        for (size_t k = 0; k < n; ++k) {
            Pend& p = pend[k];
            float t = 0.f;
            if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) {
                this->n[p.cls] += 1;
                ms[p.cls] += t;
                bytes[p.cls] += p.bytes;
            }
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pend.erase(pend.begin(), pend.begin() + n);
    }
    void resolve() {   // call after a stream sync
        for (auto& p : pend) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, p.a, p.b) == hipSuccess) {
                n[p.cls] += 1;
                ms[p.cls] += t;
                bytes[p.cls] += p.bytes;
            }
            pool.push_back(p.a);
            pool.push_back(p.b);
        }
        pend.clear();
    }
    void reset() {
        std::fill(n, n + 8, 0);
        std::fill(ms, ms + 8, 0.0);
        std::fill(bytes, bytes + 8, 0.0);
    }
    ~KTimer() {
        for (auto& p : pend) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};


// ----------------------------------------------------------------------------- kernel launchers
// (defined in foto_kernels.hip; all enqueue on `s` and never synchronise)
struct CGArgs {
    double r, eps, rtol;
    int world, rank;
};

hipError_t launch_apply_A(const Geo& g, const double* p, double* out, double r, double eps, int lap_only,
                          hipStream_t s);
hipError_t launch_grad_st(const Geo& g, const double* phi, double* gt, double* gx, double* gy, hipStream_t s);
hipError_t launch_div_st(const Geo& g, const double* wt, const double* wx, const double* wy, double* out,
                         hipStream_t s);
hipError_t launch_grad2(int Nx, int Ny, const double* f, double* gx, double* gy, int bcD, hipStream_t s);
hipError_t launch_div2(int Nx, int Ny, const double* u, const double* v, double* out, int bcD, double sign,
                       hipStream_t s);
hipError_t launch_grad2_forward(int Nx, int Ny, const double* f, double* gx, double* gy, hipStream_t s);
hipError_t launch_stepB(int64_t M, const double* pa, const double* p1, const double* p2, double* qa,
                        double* q1, double* q2, hipStream_t s);
hipError_t launch_init_mu(const Geo& g, const double* rho0, const double* rhoT, double* mut, double* mux,
                          double* muy, double* qt, double* qx, double* qy, hipStream_t s);
// F = div_st(mu - r q) + BC, written to `F`; F.F partial -> gath[rank]
hipError_t launch_rhs(const Geo& g, const double* mut, const double* mux, const double* muy, const double* qt,
                      const double* qx, const double* qy, const double* rho0, const double* rhoT, double r,
                      double* F, RedBuf rb, double* gath, int rank, hipStream_t s);
// stencil CG iteration kernels
hipError_t launch_cg_dir(const Geo& g, int k, const double* rvec, const double* pold, double* pnew,
                         const CGArgs& a, CGScal* S, RedBuf rb, const double* gath_rr, double* gath_pap,
                         int fused, hipStream_t s);
hipError_t launch_cg_pupd(const Geo& g, int k, const double* rvec, const double* pold, double* pnew,
                          CGScal* S, const double* gath_rr, const CGArgs& a, hipStream_t s);
hipError_t launch_cg_upd(const Geo& g, int k, const double* p, double* x, double* rvec, const CGArgs& a,
                         CGScal* S, RedBuf rb, const double* gath_pap, double* gath_rr, hipStream_t s);
// grad_st phi -> stepB -> mu update -> crit partial sums (num, den) -> gath[2*rank..]
hipError_t launch_prox(const Geo& g, const double* phi, double* mut, double* mux, double* muy, double* qt,
                       double* qx, double* qy, double r, RedBuf rb, double* gath, int rank, hipStream_t s,
                       const int* guard = nullptr);
// k_prox fused with the next iteration's RHS (mu -> nu, F, this rank's crit num/den ->
// gath_crit[0..1], F.F -> gath_rr[0] when non-null); needs rb.cap >= 3 * prox_rhs_blocks(g).
// Sharded (g.t0 > 0 or g.t0 + g.nloc < g.Nt), either: defer_lo / defer_hi = 0 -- stepB is
// recomputed on the neighbours' boundary planes: phi needs two valid halo planes on each side
// and mu one; or defer_lo / defer_hi = 1 on the sides that have a neighbour -- phi needs one
// halo plane, F of that edge plane is left to launch_rhs_edge after w_t's halo exchange
// (wt_out: a halo-padded field, planes 0, 1, nloc - 2, nloc - 1 written; edge: 2 x 4 planes).
int prox_rhs_blocks(const Geo& g);
hipError_t launch_prox_rhs(const Geo& g, const double* phi, const double* mut, const double* mux, const double* muy,
                           double* nut, double* nux, double* nuy, const double* rho0, const double* rhoT, double r,
                           double* F, RedBuf rb, double* gath_crit, double* gath_rr, hipStream_t s,
                           const int* guard = nullptr, int defer_lo = 0, int defer_hi = 0, double* wt_out = nullptr,
                           double* edge = nullptr, double* hcrit = nullptr, int wt_pre = 0);
// w_t = mu'_t - r q_t of the deferred edge planes (0 if defer_lo, nloc - 1 if defer_hi) into
// wt, ahead of launch_prox_rhs (which then gets wt_pre = 1 and leaves those planes alone): the
// w_t exchange can travel while the fused kernel runs.  phi needs its halo planes.
hipError_t launch_wt_pre(const Geo& g, const double* phi, const double* mut, const double* mux, const double* muy,
                         double r, double* wt, int defer_lo, int defer_hi, hipStream_t s, const int* guard = nullptr);
// F of a deferred edge plane n (0 or nloc - 1; edge slot 0 or 1), F.F added to gath_rr[0]
hipError_t launch_rhs_edge(const Geo& g, int n, const double* wt, const double* edge, const double* rho0,
                           const double* rhoT, double r, double* F, RedBuf rb, double* gath_rr, hipStream_t s,
                           const int* guard = nullptr);
// q = Proj_K(grad_st phi + mu / r) only (the stepB output the fused kernel does not store)
hipError_t launch_q_from_phi(const Geo& g, const double* phi, const double* mut, const double* mux,
                             const double* muy, double* qt, double* qx, double* qy, double r, hipStream_t s);
// trajectory steps n in [n_lo, n_hi) using phi planes (local plane index l = n - t0)
hipError_t launch_traj(const Geo& g, const double* phi, int n_lo, int n_hi, double* px, double* py,
                       int init, hipStream_t s);
hipError_t launch_flow_finish(int Nx, int Ny, const double* px, const double* py, double* u, double* v,
                              double* m, hipStream_t s);

hipError_t launch_dot_self(int64_t n, const double* x, RedBuf rb, double* gath, int rank, hipStream_t s);

// GN
hipError_t launch_gn_coeffs(int w, int h, const double* f1, const double* f2, double* fx, double* fy,
                            double* ft, hipStream_t s);
hipError_t launch_gn_rhs(int w, int h, const double* fx, const double* fy, const double* f2, const double* ft,
                         double* b, hipStream_t s);
hipError_t launch_gn_apply(int w, int h, const double* fx, const double* fy, const double* f2, double alpha,
                           double lam, const double* x, double* y, hipStream_t s);
hipError_t launch_gn_pcg_init(int w, int h, const double* fx, const double* fy, const double* f2, double alpha,
                              double lam, const double* b, double* r, double* z, RedBuf rb, double* gath,
                              hipStream_t s);
hipError_t launch_gn_pcg_dir(int w, int h, int k, const double* fx, const double* fy, const double* f2,
                             double alpha, double lam, const double* z, const double* pold, double* pnew,
                             CGScal* S, RedBuf rb, const double* gath_rz, double* gath_pq, double rtol,
                             hipStream_t s);
hipError_t launch_gn_pcg_upd(int w, int h, int k, const double* fx, const double* fy, const double* f2,
                             double alpha, double lam, const double* p, double* x, double* r, double* z,
                             CGScal* S, RedBuf rb, const double* gath_pq, double* gath_rz, hipStream_t s);

}  // namespace foto
