// libfoto host side: the Benamou-Brenier solver context, the device-resident CG driver,
// time-slab sharding (RCCL across processes, or in-process virtual ranks on one device
// for testing the sharded path), and the BB part of the C ABI (include/foto.h).
//
// Reference: benamou_brenier.solve (benamou_brenier.py:151-271).  One outer iteration =
//   stepA: F = div_st(mu - r q) + BC (k_rhs), phi = cg(A, F) (k_cg_dir / k_cg_upd loop)
//   stepB: q = Proj_K(grad_st phi + mu / r); stepC: mu += r (grad phi - q), mu_rho >= 0;
//   crit = sqrt(num / (den + 1e-10))  (all fused in k_prox)
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstddef>
#include <cstring>
#include <memory>
#include <mutex>
#include <utility>

#include "foto_internal.h"
#include "foto_spectral.h"
#include "foto_xfer.h"

namespace foto {

static thread_local char g_err[2048] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

static std::mutex g_pool_mu;
static std::vector<std::pair<int, hipStream_t>> g_pool;   // (device, stream) free list
static std::vector<std::pair<hipStream_t, int>> g_live;   // streams handed out, with their device

// a stream of the current device; stream_release files it under the device it was created on
// (not the device current at release: a context on device 1 closed while device 0 is current)
int stream_acquire(hipStream_t* out) {
    int dev = 0;
    FOTO_HIP_CHECK(hipGetDevice(&dev));
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size(); ++i)
            if (g_pool[i].first == dev) {
                *out = g_pool[i].second;
                g_pool.erase(g_pool.begin() + i);
                g_live.push_back({*out, dev});
                return 0;
            }
    }
    FOTO_HIP_CHECK(hipStreamCreateWithFlags(out, hipStreamNonBlocking));
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_live.push_back({*out, dev});
    return 0;
}

void stream_release(hipStream_t s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_live.size(); ++i)
        if (g_live[i].first == s) {
            g_pool.push_back({g_live[i].second, s});
            g_live.erase(g_live.begin() + i);
            return;
        }
}

int stream_device(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (const auto& e : g_live)
        if (e.first == s) return e.second;
    return -1;
}

#define FOTO_NCCL_CHECK(call)                                                                 \
    do {                                                                                     \
        ncclResult_t r_ = (call);                                                            \
        if (r_ != ncclSuccess) {                                                             \
            ::foto::set_error("%s:%d %s: %s", __FILE__, __LINE__, #call, ncclGetErrorString(r_)); \
            return FOTO_ERR_COMM;                                                            \
        }                                                                                    \
    } while (0)

// ----------------------------------------------------------------------------- shards

struct Shard {
    Geo g{};
    int rank = 0;
    // fields: halo-padded planes (l = -1 .. nloc), pointers at local plane 0
    double* mu[3] = {nullptr, nullptr, nullptr};
    double* q[3] = {nullptr, nullptr, nullptr};
    double* nu[3] = {nullptr, nullptr, nullptr};   // second mu buffer of the fused prox + RHS
    double* xi[3] = {nullptr, nullptr, nullptr};   // third mu buffer (two outer iterations in flight)
    double* phi = nullptr;   // CG iterate x (two halo planes per side: the fused prox reads them)
    double* phi_alt = nullptr;   // the other phi of the pipelined loop
    // the last fused prox + RHS launch's mu in / out (fz_src is the mu stepB of phi used)
    double* fz_src[3] = {nullptr, nullptr, nullptr};
    double* fz_dst[3] = {nullptr, nullptr, nullptr};
    // sharded fused prox with deferred edges: w_t next to the slab edges (halo-padded) and the
    // edge planes' (w_x, w_y, mu'_t, q_t), slot 0 = plane 0, slot 1 = plane nloc - 1
    double* wt = nullptr;
    double* edge = nullptr;
    double* rv = nullptr;    // CG residual (starts as F)
    double* p[2] = {nullptr, nullptr};
    double* rho0 = nullptr;
    double* rhoT = nullptr;
    double* px = nullptr;    // trajectory positions
    double* py = nullptr;
    double* fu = nullptr;    // flow output (last rank)
    double* fv = nullptr;
    double* fm = nullptr;
    RedBuf rb{};
    double* gath = nullptr;  // [0,W) rr | [W,2W) pap | [2W,4W) crit num/den
    CGScal* S = nullptr;
    std::vector<void*> allocs;
    std::unique_ptr<SpectralPlan> spec;

    double* gath_rr() { return gath; }
    double* gath_pap(int W) { return gath + W; }
    double* gath_crit(int W) { return gath + 2 * W; }

    int alloc(size_t bytes, void** out) {
        FOTO_HIP_CHECK(hipMalloc(out, bytes));
        allocs.push_back(*out);
        return 0;
    }
    // (nloc + 2 h) planes (h halo planes per side), zeroed on the context's stream: a hipMemset
    // (null stream) is not ordered with the non-blocking stream the kernels run on -- it raced
    // with k_init_mu
    int alloc_field(double** out, hipStream_t st, int h = 1) {
        void* b = nullptr;
        const size_t n = (size_t)(g.nloc + 2 * h) * (size_t)g.nxy;
        FOTO_TRY(alloc(n * sizeof(double), &b));
        FOTO_HIP_CHECK(hipMemsetAsync(b, 0, n * sizeof(double), st));
        *out = (double*)b + (size_t)h * g.nxy;
        return 0;
    }
    ~Shard() {
        for (void* a : allocs) (void)hipFree(a);
    }
};

}  // namespace foto

using namespace foto;

// ----------------------------------------------------------------------------- context

struct foto_bb_ctx {
    int Nt = 0, Nx = 0, Ny = 0;
    double r = 1, eps = 1e-3;
    foto_bb_opts o{};
    int W = 1;            // total ranks (processes * virtual)
    bool rccl = false;
    ncclComm_t nc = nullptr;
    hipStream_t s = nullptr;
    // RCCL: every collective and send / receive group goes on its own stream, ordered against
    // the compute stream s by events (comm_fork / comm_join), so a group can travel while s
    // transforms the next part of the slab (the pipelined all-to-alls below)
    hipStream_t sc = nullptr;
    hipEvent_t cfork = nullptr, cjoin = nullptr;
    hipEvent_t cpart[8] = {};      // the backward all-to-all's parts, landed
    bool phi_halo = false;         // phi's halo planes came with the backward all-to-all
    // the w_t halo of the deferred slab edges, issued on sc before k_prox_rhs (wt_overlap); the
    // next forward finishes the edge planes' F (k_rhs_edge) from it
    bool wt_pending = false;       // issued on sc by prox_rhs, not yet consumed
    bool wt_guarded = false;       // (the prox it belongs to was launched behind a solve's done flag)
    std::vector<std::unique_ptr<Shard>> sh;   // local shards
    CGScal* hS = nullptr;                     // pinned host mirror of shard 0's CG scalars
    int last_cg = 0;
    int last_passes = 0;   // s-step passes of the previous sharded spectral solve
    int have_phi = 0;
    // prox fused with the next RHS (k_prox_rhs); F in rv is then produced by the previous
    // outer iteration (f_ready), mu rotates through Shard::mu / nu (/ xi)
    bool fuse = false;
    bool f_ready = false;
    // Two outer iterations in flight (single shard, fused, Gauss CG; FOTO_PIPE=0: one): the
    // host enqueues iteration i + 1 before it waits for iteration i's crit, so the GPU never
    // idles while the host wakes up and launches.  mu rotates through three buffers and phi
    // alternates between two, so an iteration the stop rules turn out not to want is dropped
    // (rollback) with iteration i's state intact; a failed Gauss solve is redone after its
    // successor, which its done-flag chain kept from touching the state, is dropped.
    bool pipe = false;
    struct Enq {            // an outer iteration on the stream (outer_tail -> outer_complete)
        int par = 0;        // its event / readback slot
        SpectralPlan* dsp = nullptr;   // deferred solve to finish (single shard)
        bool sdefer = false;           // sharded Gauss solve enqueued without a host wait
        int its = 0, info = 0;         // a synchronous solve's result
        size_t kmark = 0;              // KTimer mark before its launches
        // host state before it (restored by a rollback)
        double* mu[3];
        double* nu[3];
        double* xi[3];
        double* phi;
        double* phi_alt;
        double* fz_src[3];
        double* fz_dst[3];
        bool f_ready;
        int hpar;
        bool pev;                      // phase events recorded (ph[par][0..3])
    };
    std::vector<Enq> inflight;   // oldest first
    // an iterate call failed with iterations on the stream: they were drained (drain_inflight),
    // the host state no longer matches the device's, so only foto_bb_reset brings it back
    bool broken = false;
    // inside foto_bb_iterate (its callback runs with iterations on the stream): reset and a
    // nested iterate are refused there instead of resetting state under the running loop
    bool in_iterate = false;
    // bookkeeping
    double prev_crit = -1;
    foto_bb_stats st{};
    KTimer kt;
    hipEvent_t ph[2][4] = {};      // per slot: RHS start | CG start | prox start | crit readback
    hipEvent_t fin[2] = {};        // per slot: crit readback without timing (phase events off)
    hipEvent_t fl[2] = {};         // flow extraction
    double* hgath[2] = {nullptr, nullptr};   // pinned host mirrors of gath, per slot
    double* dgath[2] = {nullptr, nullptr};   // their device addresses (coherent host memory)
    bool hcrit = false;            // single shard, fused prox: the kernel writes crit to hgath itself
    bool phase_force = false;      // FOTO_PHASE_EV=1: phase events even without kernel timing
    int hpar = 0;                  // slot of the last head
    ~foto_bb_ctx() {
        if (sc) (void)hipStreamSynchronize(sc);
        if (s) (void)hipStreamSynchronize(s);   // (before the shards free their buffers)
        sh.clear();
        if (nc) (void)ncclCommDestroy(nc);
        if (hS) (void)hipHostFree(hS);
        for (double* h : hgath) if (h) (void)hipHostFree(h);
        for (auto& p : ph)
            for (auto e : p) if (e) (void)hipEventDestroy(e);
        for (auto e : fl) if (e) (void)hipEventDestroy(e);
        for (auto e : fin) if (e) (void)hipEventDestroy(e);
        for (auto e : {cfork, cjoin}) if (e) (void)hipEventDestroy(e);
        for (auto e : cpart) if (e) (void)hipEventDestroy(e);
        if (sc) {
            (void)hipStreamSynchronize(sc);
            stream_release(sc);
        }
        if (s) {
            (void)hipStreamSynchronize(s);
            stream_release(s);
        }
    }
};

namespace foto {

// ----------------------------------------------------------------------------- communication
// Every exchange between shards is a list of point-to-point transfers (foto_xfer.h), built by
// the same code on every rank and for every transport; only its execution differs:
//   virtual ranks (one process, all shards on one device and stream): one device copy per
//   transfer, in list order;
//   RCCL (one shard per process): the calls rccl_calls() lists -- in one group, ncclSend for
//   each transfer from this rank and ncclRecv for each transfer to it (pairs match in list
//   order, which is the same on every rank), then a device copy for each transfer to itself.
// Offsets are in doubles from the pointer a picker returns for the shard (negative: the halo
// plane below).  The virtual-rank GPU tests therefore run the very lists RCCL executes, and
// tests/test_xfer.py checks the RCCL call sequences of every rank against each other.
// compute stream -> communication stream: what s has enqueued so far happens before what sc
// runs next (RCCL only; virtual ranks run everything on s)
static int comm_fork(foto_bb_ctx* c) {
    if (!c->sc) return 0;
    FOTO_HIP_CHECK(hipEventRecord(c->cfork, c->s));
    FOTO_HIP_CHECK(hipStreamWaitEvent(c->sc, c->cfork, 0));
    return 0;
}
// communication stream -> compute stream
static int comm_join(foto_bb_ctx* c) {
    if (!c->sc) return 0;
    FOTO_HIP_CHECK(hipEventRecord(c->cjoin, c->sc));
    FOTO_HIP_CHECK(hipStreamWaitEvent(c->s, c->cjoin, 0));
    return 0;
}

// one list, issued on the communication stream (RCCL) or as copies on s (virtual ranks); the
// caller orders it against s (exchange() below does, the pipelined all-to-alls do per part)
template <class SrcPick, class DstPick>
static int exchange_raw(foto_bb_ctx* c, const std::vector<Xfer>& xs, SrcPick sp, DstPick dp) {
    if (!c->rccl) {
        for (const Xfer& x : xs)
            FOTO_HIP_CHECK(hipMemcpyAsync(dp(*c->sh[x.dst]) + x.doff, sp(*c->sh[x.src]) + x.soff,
                                          (size_t)x.n * sizeof(double), hipMemcpyDeviceToDevice, c->s));
        return 0;
    }
    hipStream_t st = c->sc ? c->sc : c->s;
    Shard& s = *c->sh[0];
    const std::vector<Call> cs = rccl_calls(xs, s.rank);
    const bool grouped = !cs.empty() && cs.front().op != CALL_COPY;
    if (grouped) FOTO_NCCL_CHECK(ncclGroupStart());
    bool open = grouped;
    for (const Call& k : cs) {
        if (k.op == CALL_COPY && open) {
            FOTO_NCCL_CHECK(ncclGroupEnd());
            open = false;
        }
        if (k.op == CALL_SEND)
            FOTO_NCCL_CHECK(ncclSend(sp(s) + k.off, (size_t)k.n, ncclDouble, k.peer, c->nc, st));
        else if (k.op == CALL_RECV)
            FOTO_NCCL_CHECK(ncclRecv(dp(s) + k.off, (size_t)k.n, ncclDouble, k.peer, c->nc, st));
        else
            FOTO_HIP_CHECK(hipMemcpyAsync(dp(s) + k.doff, sp(s) + k.off, (size_t)k.n * sizeof(double),
                                          hipMemcpyDeviceToDevice, st));
    }
    if (open) FOTO_NCCL_CHECK(ncclGroupEnd());
    return 0;
}

template <class SrcPick, class DstPick>
static int exchange(foto_bb_ctx* c, const std::vector<Xfer>& xs, SrcPick sp, DstPick dp) {
    FOTO_TRY(comm_fork(c));
    FOTO_TRY(exchange_raw(c, xs, sp, dp));
    return comm_join(c);
}

// each rank's `cnt` doubles at slot [rank] of the picked array to every rank's same slot
// (RCCL: one ncclAllGather, in place; virtual ranks: the equivalent copies)
template <class Pick>
static int allgather(foto_bb_ctx* c, Pick pick, int cnt) {
    if (c->W == 1) return 0;
    if (c->rccl) {
        Shard& s = *c->sh[0];
        double* base = pick(s);
        FOTO_TRY(comm_fork(c));
        FOTO_NCCL_CHECK(ncclAllGather(base + (size_t)s.rank * cnt, base, cnt, ncclDouble, c->nc, c->sc ? c->sc : c->s));
        return comm_join(c);
    }
    return exchange(c, allgather_xfers(c->W, cnt), pick, pick);
}

template <class Pick>
static int halo(foto_bb_ctx* c, Pick pick) {
    if (c->W == 1) return 0;
    return exchange(c, halo_xfers(c->Nt, (int64_t)c->Nx * c->Ny, c->W), pick, pick);
}

// ----------------------------------------------------------------------------- context setup

static int ctx_init(foto_bb_ctx* c, const double* rho0, const double* rhoT) {
    const int64_t nxy = (int64_t)c->Nx * c->Ny;
    if (c->o.device >= 0) FOTO_HIP_CHECK(hipSetDevice(c->o.device));
    FOTO_TRY(stream_acquire(&c->s));
    FOTO_HIP_CHECK(hipHostMalloc((void**)&c->hS, sizeof(CGScal)));
    const int W = c->W;
    for (int k = 0; k < 2; ++k) {
        FOTO_HIP_CHECK(hipHostMalloc((void**)&c->hgath[k], sizeof(double) * 4 * W,
                                     hipHostMallocMapped | hipHostMallocCoherent));
        FOTO_HIP_CHECK(hipHostGetDevicePointer((void**)&c->dgath[k], c->hgath[k], 0));
    }
    for (auto& p : c->ph)
        for (int k = 0; k < 4; ++k)   // (phase boundaries: timing only; the crit event keeps the fence)
            FOTO_HIP_CHECK(hipEventCreateWithFlags(&p[k], k < 3 ? hipEventDisableSystemFence : hipEventDefault));
    for (auto& e : c->fl) FOTO_HIP_CHECK(hipEventCreate(&e));
    if (c->rccl) {
        ncclUniqueId id;
        memcpy(&id, c->o.nccl_id, sizeof(id));
        FOTO_NCCL_CHECK(ncclCommInitRank(&c->nc, W, id, c->o.rank));
        // FOTO_COMM_STREAM=0: every RCCL call on the compute stream (A/B runs)
        const char* cs = getenv("FOTO_COMM_STREAM");
        if (!(cs && atoi(cs) == 0)) {
            FOTO_TRY(stream_acquire(&c->sc));
            FOTO_HIP_CHECK(hipEventCreateWithFlags(&c->cfork, hipEventDisableTiming));
            FOTO_HIP_CHECK(hipEventCreateWithFlags(&c->cjoin, hipEventDisableTiming));
            for (auto& e : c->cpart) FOTO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
    }
    const int nlocal = c->rccl ? 1 : W;
    {
        const char* e = getenv("FOTO_FUSE_PR");   // 0: separate k_prox / k_rhs (A/B runs)
        c->fuse = !(e && atoi(e) == 0);
        const char* pe = getenv("FOTO_PIPE");   // 0: one outer iteration in flight (A/B runs)
        c->pipe = W == 1 && c->fuse && c->o.cg_mode == 3 && !(pe && atoi(pe) == 0);
        // the crit readback as two stores of k_prox_rhs's last block into the slot (a copy launch
        // on the stream costs ~4 us; FOTO_HOST_CRIT=0: the copy)
        // phase events (the RHS / CG / prox split of foto_bb_stats) only with kernel timing on:
        // three timed event records per outer iteration cost ~13 us of GPU time at the bench
        // grid (1561-1572 vs 1603-1616 it/s, same box), and the crit sync uses a timing-free one
        const char* pv = getenv("FOTO_PHASE_EV");
        c->phase_force = pv && atoi(pv) == 1;
        const char* hc = getenv("FOTO_HOST_CRIT");
        c->hcrit = W == 1 && c->fuse && !(hc && atoi(hc) == 0);
        // the crit sync: with the crit pair and the Gauss header stored into coherent host memory
        // by the kernels themselves (fenced there), the event needs no system-scope fence of its
        // own -- a fenced record writes the L2's dirty lines back once per outer iteration
        // (FOTO_SYNC_FENCE=1: fenced)
        const char* sf = getenv("FOTO_SYNC_FENCE");
        const unsigned ff = (c->hcrit && !(sf && atoi(sf) == 1)) ? hipEventDisableSystemFence : 0u;
        for (auto& e : c->fin) FOTO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming | ff));
    }
    for (int j = 0; j < nlocal; ++j) {
        auto sp = std::make_unique<Shard>();
        Shard& s = *sp;
        s.rank = c->rccl ? c->o.rank : j;
        s.g.Nt = c->Nt; s.g.Ny = c->Ny; s.g.Nx = c->Nx; s.g.nxy = nxy;
        if (split_planes(c->Nt, W, s.rank, &s.g.t0, &s.g.nloc) != 0) {
            set_error("world size %d exceeds Nt = %d (each rank needs >= 1 time slab)", W, c->Nt);
            return FOTO_ERR_ARG;
        }
        for (int f = 0; f < 3; ++f) { FOTO_TRY(s.alloc_field(&s.mu[f], c->s)); FOTO_TRY(s.alloc_field(&s.q[f], c->s)); }
        if (c->fuse)
            for (int f = 0; f < 3; ++f) FOTO_TRY(s.alloc_field(&s.nu[f], c->s));
        if (c->pipe) {
            for (int f = 0; f < 3; ++f) FOTO_TRY(s.alloc_field(&s.xi[f], c->s));
            FOTO_TRY(s.alloc_field(&s.phi_alt, c->s, 2));
        }
        if (c->fuse && W > 1) {
            FOTO_TRY(s.alloc_field(&s.wt, c->s));
            void* eb = nullptr;
            FOTO_TRY(s.alloc(sizeof(double) * 8 * nxy, &eb));
            FOTO_HIP_CHECK(hipMemsetAsync(eb, 0, sizeof(double) * 8 * nxy, c->s));
            s.edge = (double*)eb;
        }
        FOTO_TRY(s.alloc_field(&s.phi, c->s, 2));
        FOTO_TRY(s.alloc_field(&s.rv, c->s));
        FOTO_TRY(s.alloc_field(&s.p[0], c->s));
        FOTO_TRY(s.alloc_field(&s.p[1], c->s));
        void* b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.rho0 = (double*)b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.rhoT = (double*)b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.px = (double*)b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.py = (double*)b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.fu = (double*)b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.fv = (double*)b;
        FOTO_TRY(s.alloc(nxy * sizeof(double), &b)); s.fm = (double*)b;
        const int64_t nb = std::max<int64_t>(march_blocks(s.g), flat_blocks((int64_t)s.g.nloc * nxy));
        s.rb.cap = (int)std::max<int64_t>(2 * nb, 3 * (int64_t)prox_rhs_blocks(s.g));
        FOTO_TRY(s.alloc(sizeof(double) * s.rb.cap, &b)); s.rb.partials = (double*)b;
        FOTO_TRY(s.alloc(sizeof(unsigned) * 64, &b)); s.rb.ticket = (unsigned*)b;
        FOTO_HIP_CHECK(hipMemsetAsync(s.rb.ticket, 0, sizeof(unsigned) * 64, c->s));
        FOTO_TRY(s.alloc(sizeof(double) * 4 * W, &b)); s.gath = (double*)b;
        FOTO_HIP_CHECK(hipMemsetAsync(s.gath, 0, sizeof(double) * 4 * W, c->s));
        FOTO_TRY(s.alloc(sizeof(CGScal), &b)); s.S = (CGScal*)b;
        FOTO_HIP_CHECK(hipMemcpyAsync(s.rho0, rho0, nxy * sizeof(double), hipMemcpyHostToDevice, c->s));
        FOTO_HIP_CHECK(hipMemcpyAsync(s.rhoT, rhoT, nxy * sizeof(double), hipMemcpyHostToDevice, c->s));
        FOTO_HIP_CHECK(launch_init_mu(s.g, s.rho0, s.rhoT, s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], c->s));
        if (c->o.cg_mode >= 1 && c->o.cg_mode <= 3) {
            s.spec.reset(new SpectralPlan());
            FOTO_TRY(s.spec->init(s.g, s.rank, W, c->r, c->eps, c->o.cg_mode, c->s));
        }
        c->sh.push_back(std::move(sp));
    }
    // the Gauss CG may fall back to the s-step CG for boxes its voxel list cannot pack
    if (c->pipe && !(c->sh[0]->spec && c->sh[0]->spec->gauss())) c->pipe = false;
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    return 0;
}

// ----------------------------------------------------------------------------- CG driver

static CGArgs cg_args(foto_bb_ctx* c, const Shard& s) {
    CGArgs a;
    a.r = c->r;
    a.eps = c->eps;
    a.rtol = c->o.cg_rtol;
    a.world = c->W;
    a.rank = s.rank;
    return a;
}

static int cg_iteration(foto_bb_ctx* c, int k) {
    const int W = c->W;
    const bool fused = (W == 1);
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        double* pold = s.p[k & 1];
        double* pnew = s.p[(k + 1) & 1];
        const CGArgs a = cg_args(c, s);
        const double nv = (double)s.g.nloc * (double)s.g.nxy;
        if (!fused) FOTO_HIP_CHECK(launch_cg_pupd(s.g, k, s.rv, pold, pnew, s.S, s.gath_rr(), a, c->s));
        (void)nv;
    }
    if (!fused) FOTO_TRY(halo(c, [k](Shard& s) { return s.p[(k + 1) & 1]; }));
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        const CGArgs a = cg_args(c, s);
        const double nv = (double)s.g.nloc * (double)s.g.nxy;
        hipEvent_t e = c->kt.start(c->s);
        FOTO_HIP_CHECK(launch_cg_dir(s.g, k, s.rv, s.p[k & 1], s.p[(k + 1) & 1], a, s.S, s.rb, s.gath_rr(),
                                     s.gath_pap(W), fused ? 1 : 0, c->s));
        c->kt.stop(e, c->s, FOTO_K_CG_DIR, fused ? (k == 0 ? 16.0 : 24.0) * nv : 8.0 * nv);
    }
    FOTO_TRY(allgather(c, [W](Shard& s) { return s.gath_pap(W); }, 1));
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        const CGArgs a = cg_args(c, s);
        const double nv = (double)s.g.nloc * (double)s.g.nxy;
        hipEvent_t e = c->kt.start(c->s);
        FOTO_HIP_CHECK(launch_cg_upd(s.g, k, s.p[(k + 1) & 1], s.phi, s.rv, a, s.S, s.rb, s.gath_pap(W),
                                     s.gath_rr(), c->s));
        c->kt.stop(e, c->s, FOTO_K_CG_UPD, (k == 0 ? 32.0 : 40.0) * nv);
    }
    FOTO_TRY(allgather(c, [](Shard& s) { return s.gath_rr(); }, 1));
    return 0;
}

// The slab <-> row-box all-to-alls (foto_xfer.h), pipelined in parts: the forward one sends a
// part of every slab once its x / y DCTs have run, while the compute stream transforms the next
// part; the backward one lands in parts and each part's inverse y / x DCTs start as soon as it
// is in, while the next part travels.  The backward one also delivers phi's halo planes (a2a_halo)
// -- rows of the neighbours' boundary planes from every box owner, over all links, transformed
// here with the own planes -- so the fused prox + RHS needs no separate one-plane phi exchange
// over the single link to each neighbour.  Virtual ranks run the same lists as copies on s.
// Both pay off where a plane is large against the compute it adds (two planes of inverse x / y
// DCT for the halo, twice the DCT launches for two parts): by default they are on for planes of
// >= 2^19 voxels (C4's 1024 x 1024: 8.4 MB per plane, 131 us over one link; 2 parts, the halo
// inside) and off below (the bench grid's 640 x 480: 2.5 MB, where the compute-only proxy gave
// 0.337 against 0.300 ms per rank at W = 8 with them on, profiles/r05_proxy_scaling.txt).
// FOTO_A2A_PARTS (1..8) and FOTO_A2A_HALO (0 / 1) override (A/B runs, tests).
static bool a2a_big_planes(const foto_bb_ctx* c) { return (int64_t)c->Nx * c->Ny >= (1 << 19); }

static int a2a_parts(const foto_bb_ctx* c) {
    const char* e = getenv("FOTO_A2A_PARTS");
    const int v = e ? atoi(e) : (a2a_big_planes(c) ? 2 : 1);
    return std::max(1, std::min(8, v));
}

static int a2a_halo(const foto_bb_ctx* c) {
    if (c->W == 1) return 0;
    const char* e = getenv("FOTO_A2A_HALO");
    if (e ? atoi(e) == 0 : !a2a_big_planes(c)) return 0;
    // the deferred-edge fused prox (and the unfused prox) read one phi halo plane per side; the
    // edge-recompute variant (FOTO_PR_EDGE=0) reads two and keeps its own exchange
    const char* pe = getenv("FOTO_PR_EDGE");
    return (c->fuse && pe && atoi(pe) == 0) ? 0 : 1;
}

// F on the deferred edge planes of every local shard, from its w_t halo (k_rhs_edge)
static int wt_edges(foto_bb_ctx* c, bool guarded) {
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        const int dlo = s.g.t0 > 0, dhi = s.g.t0 + s.g.nloc < c->Nt;
        double* rr = c->o.cg_mode == 0 ? s.gath_rr() + s.rank : nullptr;
        const int* gd = guarded ? s.spec->done_flag() : nullptr;
        if (dlo)
            FOTO_HIP_CHECK(launch_rhs_edge(s.g, 0, s.wt, s.edge, s.rho0, s.rhoT, c->r, s.rv, s.rb, rr, c->s, gd));
        if (dhi && !(dlo && s.g.nloc == 1))
            FOTO_HIP_CHECK(launch_rhs_edge(s.g, s.g.nloc - 1, s.wt, s.edge + 4 * s.g.nxy, s.rho0, s.rhoT, c->r, s.rv,
                                           s.rb, rr, c->s, gd));
    }
    return 0;
}

// (round 5) the w_t exchange overlapped with k_prox_rhs: k_wt_pre computes the edge planes' w_t
// first, the exchange travels on the communication stream while k_prox_rhs runs, and the next
// forward finishes the edge planes' F (k_rhs_edge) before transforming them.  RCCL on its own
// stream, a spectral CG (the stencil CG needs F.F at once), slabs of >= 3 planes;
// FOTO_WT_OVERLAP=0: exchange and finish the edges after k_prox_rhs
static bool slabs_of_3(const foto_bb_ctx* c) {
    // all ranks decide alike (the call sequences stay identical whichever way, tests/test_xfer.py),
    // so the rule rests on the smallest slab of the split
    for (int r = 0; r < c->W; ++r) {
        int t0 = 0, nl = 0;
        if (split_planes(c->Nt, c->W, r, &t0, &nl) != 0 || nl < 3) return false;
    }
    return true;
}
static bool wt_overlap(const foto_bb_ctx* c) {
    if (!c->rccl || !c->sc || c->o.cg_mode == 0 || c->sh.size() != 1 || !slabs_of_3(c)) return false;
    const char* e = getenv("FOTO_WT_OVERLAP");
    return !(e && atoi(e) == 0);
}

// k_wt_pre ahead of k_prox_rhs: RCCL where wt_overlap holds; virtual ranks with FOTO_WT_PRE=1
// (the same kernel sequence, exchanged by copies on s -- tests, tools/proxy_scaling.py)
static bool wt_pre_on(const foto_bb_ctx* c) {
    if (c->rccl) return wt_overlap(c);
    const char* e = getenv("FOTO_WT_PRE");
    return c->W > 1 && c->o.cg_mode != 0 && e && atoi(e) == 1 && slabs_of_3(c);
}

// a w_t exchange that no forward will consume (a new prox supersedes it): forget or wait for it
static int wt_drop(foto_bb_ctx* c) {
    if (!c->wt_pending) return 0;
    c->wt_pending = false;
    return comm_join(c);
}

// Spectral CG over time-slab shards, in phases: x/y DCTs on the own planes, all-to-all to row
// boxes and the t-DCT (sharded_fwd); the Gauss-compressed CG -- one all-gather of the boxes'
// histograms, summed in rank order on every rank, and the small serial solve on every rank
// (sharded_gauss) -- or the s-step CG from b^ with one NACC-double all-gather per pass (moments
// summed in rank order, so all ranks plan identically; sharded_sstep); then x^, the inverse
// t-DCT, the all-to-all back and the inverse x/y DCTs (sharded_inv).
static int sharded_fwd(foto_bb_ctx* c) {
    KTimer* kt = &c->kt;
    const int parts = a2a_parts(c);
    // the slab side is the shard's RHS buffer: fwd_local leaves the x / y DCTs of F there
    auto sbuf = [](Shard& s) { return s.rv; };
    auto rbuf = [](Shard& s) { return s.spec->box_in(); };
    // w_t exchanged behind k_prox_rhs (wt_overlap; landed by now: the crit all-gather queued
    // behind it on sc was joined): the edge planes' F before their x / y DCTs
    if (c->wt_pending) {
        FOTO_TRY(comm_join(c));
        c->wt_pending = false;
        FOTO_TRY(wt_edges(c, c->wt_guarded));
    }
    for (int p = 0; p < parts; ++p) {
        for (auto& sp : c->sh) {
            int lo, hi;
            split_part(sp->g.nloc, parts, p, &lo, &hi);
            if (hi > lo) FOTO_TRY(sp->spec->fwd_local(sp->rv, lo, hi, kt, c->s));
        }
        FOTO_TRY(comm_fork(c));
        FOTO_TRY(exchange_raw(c, alltoall_part_xfers(c->Nt, c->Ny, c->Nx, c->W, true, p, parts, 0), sbuf, rbuf));
    }
    FOTO_TRY(comm_join(c));
    for (auto& sp : c->sh) FOTO_TRY(sp->spec->fwd_t(kt, c->s));
    return 0;
}

static int sharded_gauss(foto_bb_ctx* c) {
    KTimer* kt = &c->kt;
    for (auto& sp : c->sh) FOTO_TRY(sp->spec->gauss_measure(kt, c->s));
    FOTO_TRY(allgather(c, [](Shard& s) { return s.spec->gauss_hist(); }, SpectralPlan::gauss_hist_size()));
    for (auto& sp : c->sh) FOTO_TRY(sp->spec->gauss_solve(c->o.cg_rtol, c->o.cg_maxiter, kt, c->s));
    return 0;
}

static int sharded_inv(foto_bb_ctx* c) {
    KTimer* kt = &c->kt;
    for (auto& sp : c->sh) FOTO_TRY(sp->spec->inv_t(kt, c->s));
    const int parts = a2a_parts(c), halo = a2a_halo(c);
    // inv_local takes the inverse's slab (and halo planes) from the RHS buffer (F is consumed by then)
    auto sbuf = [](Shard& s) { return s.spec->box_out(); };
    auto rbuf = [](Shard& s) { return s.rv; };
    FOTO_TRY(comm_fork(c));
    for (int p = 0; p < parts; ++p) {
        FOTO_TRY(exchange_raw(c, alltoall_part_xfers(c->Nt, c->Ny, c->Nx, c->W, false, p, parts, halo), sbuf, rbuf));
        if (c->sc) FOTO_HIP_CHECK(hipEventRecord(c->cpart[p], c->sc));
    }
    for (int p = 0; p < parts; ++p) {
        if (c->sc) FOTO_HIP_CHECK(hipStreamWaitEvent(c->s, c->cpart[p], 0));
        for (auto& sp : c->sh) {
            int lo, hi;
            alltoall_part_planes(c->Nt, c->W, sp->rank, p, parts, halo, &lo, &hi);
            if (hi > lo) FOTO_TRY(sp->spec->inv_local(sp->rv, sp->phi, lo, hi, kt, c->s));
        }
    }
    c->phi_halo = halo != 0;
    return 0;
}

static int sharded_sstep(foto_bb_ctx* c, int* iters, int* info) {
    const int maxiter = c->o.cg_maxiter;
    const double rtol = c->o.cg_rtol;
    const int M = SpectralPlan::moments();
    KTimer* kt = &c->kt;
    for (auto& sp : c->sh) FOTO_TRY(sp->spec->cg_begin(rtol, maxiter, kt, c->s));
    FOTO_TRY(allgather(c, [](Shard& s) { return s.spec->gath(); }, M));
    for (auto& sp : c->sh) FOTO_TRY(sp->spec->cg_plan(1, rtol, maxiter, c->s));
    int passes = 0, done = 0, its = 0, planned = 0;
    const int first = c->last_passes > 0 ? c->last_passes + 2 : 8;   // over-predict (see solve_s2)
    while (true) {
        const int chunk = (passes == 0) ? first : 2;
        for (int j = 0; j < chunk; ++j, ++passes) {
            for (auto& sp : c->sh) FOTO_TRY(sp->spec->cg_pass(rtol, maxiter, kt, c->s));
            FOTO_TRY(allgather(c, [](Shard& s) { return s.spec->gath(); }, M));
            for (auto& sp : c->sh) FOTO_TRY(sp->spec->cg_plan(0, rtol, maxiter, c->s));
        }
        FOTO_TRY(c->sh[0]->spec->poll(&done, &its, &planned, c->s));
        if (done) break;
        if (passes > maxiter + 4) {
            set_error("sharded spectral CG did not terminate");
            return FOTO_ERR_STATE;
        }
    }
    *iters = its;
    *info = (done == 1) ? 0 : maxiter;
    c->last_passes = planned;
    kt->discard_last(FOTO_K_SPEC, std::max(0, passes - planned) * (int)c->sh.size());   // no-op passes
    return 0;
}

// the whole sharded solve, waiting for it on the host (FOTO_CG_DEFER=0, or the s-step CG)
static int cg_solve_spectral_sharded(foto_bb_ctx* c, int* iters, int* info) {
    const int maxiter = c->o.cg_maxiter;
    FOTO_TRY(sharded_fwd(c));
    if (c->sh[0]->spec->gauss()) {
        FOTO_TRY(sharded_gauss(c));
        int ok = 1;
        for (auto& sp : c->sh) {
            int k_ok = 0;
            FOTO_TRY(sp->spec->gauss_wait(maxiter, &k_ok, iters, info, c->s));
            ok = ok && k_ok;   // identical on every shard and rank (same gathered histograms)
        }
        if (ok) {
            FOTO_TRY(sharded_inv(c));
            for (auto& sp : c->sh) sp->spec->gauss_end();
            c->last_cg = *iters;
            return 0;
        }
        c->st.cg_redo += 1;   // the s-step CG from b^ (cg_begin takes its INIT moments)
    }
    FOTO_TRY(sharded_sstep(c, iters, info));
    FOTO_TRY(sharded_inv(c));
    c->last_cg = *iters;
    return 0;
}

// Solve A x = F (F already in rv, F.F gathered in gath_rr) to scipy's stopping rule.
// The loop runs on the device; the host only polls the done flag between chunks.  Every
// rank takes the same decisions (the flag is a function of gathered scalars), so the
// collective call sequence stays identical across ranks.
static int cg_solve(foto_bb_ctx* c, int* iters, int* info) {
    const int maxiter = c->o.cg_maxiter;
    if (c->o.cg_mode != 0) {
        if (c->W > 1) return cg_solve_spectral_sharded(c, iters, info);
        Shard& s = *c->sh[0];
        FOTO_TRY(s.spec->solve(s.rv, s.phi, c->o.cg_rtol, maxiter, c->last_cg, iters, info, &c->kt, c->s));
        c->last_cg = *iters;
        return 0;
    }
    for (auto& sp : c->sh) FOTO_HIP_CHECK(hipMemsetAsync(sp->S, 0, sizeof(CGScal), c->s));
    int k = 0;
    bool done = false;
    const int first = c->last_cg > 4 ? c->last_cg - 3 : 6;
    while (k < maxiter) {
        int chunk = (k == 0) ? first : 2;
        chunk = std::min(chunk, maxiter - k);
        for (int j = 0; j < chunk; ++j, ++k) FOTO_TRY(cg_iteration(c, k));
        FOTO_HIP_CHECK(hipMemcpyAsync(c->hS, c->sh[0]->S, sizeof(CGScal), hipMemcpyDeviceToHost, c->s));
        FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
        if (c->hS->done) { done = true; break; }
    }
    if (done) {
        *iters = c->hS->iters;
        *info = 0;
        if (*iters == 0)
            for (auto& sp : c->sh)
                FOTO_HIP_CHECK(hipMemsetAsync(sp->phi, 0, sizeof(double) * sp->g.nloc * sp->g.nxy, c->s));
    } else {
        *iters = maxiter;
        *info = maxiter;
    }
    c->last_cg = *iters;
    return 0;
}

// ----------------------------------------------------------------------------- outer iteration

// One outer iteration in two halves.  outer_head + outer_tail put the iteration's work on the
// stream (a non-deferred CG solve waits for itself inside) and push an Enq record;
// outer_complete waits for the oldest record's crit readback, finishes its deferred solve and
// computes crit.  outer_head (halos, RHS) only writes F.  With one iteration in flight, a single
// spectral shard gets the next iteration's head on the stream before the host waits for this
// iteration's crit (the stop rules can still end the run there: F is scratch; a CG redo re-runs
// the head).  With two in flight (c->pipe) the whole next iteration is enqueued first.  The
// host callback runs after the next iteration is enqueued.
static bool phase_on(const foto_bb_ctx* c) { return c->phase_force || c->kt.on; }

static int outer_head(foto_bb_ctx* c) {
    c->hpar ^= 1;
    if (phase_on(c)) FOTO_HIP_CHECK(hipEventRecord(c->ph[c->hpar][0], c->s));
    // the previous iteration's k_prox_rhs wrote F (and F.F).  (Enqueuing the next solve's x-DCT
    // here, ahead of the crit wait, measured no faster: 457 vs 457 it/s same box.)
    if (c->fuse && c->f_ready) return 0;
    FOTO_TRY(wt_drop(c));   // (F recomputed whole: no edge planes left to finish)
    FOTO_TRY(halo(c, [](Shard& s) { return s.mu[0]; }));
    FOTO_TRY(halo(c, [](Shard& s) { return s.q[0]; }));
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        const double nv = (double)s.g.nloc * (double)s.g.nxy;
        hipEvent_t e = c->kt.start(c->s);
        FOTO_HIP_CHECK(launch_rhs(s.g, s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], s.rho0, s.rhoT, c->r,
                                  s.rv, s.rb, c->o.cg_mode == 0 ? s.gath_rr() : nullptr, s.rank, c->s));
        c->kt.stop(e, c->s, FOTO_K_RHS, 56.0 * nv);
    }
    if (c->o.cg_mode == 0) FOTO_TRY(allgather(c, [](Shard& s) { return s.gath_rr(); }, 1));
    return 0;
}

// the fused k_prox_rhs of every local shard on the pair recorded in its fz_src -> fz_dst;
// sharded: the two-plane phi halo and the one-plane halo of the mu it reads go first.
// guarded: each shard's launch returns at once unless its CG's done flag is set.
static int prox_rhs(foto_bb_ctx* c, bool guarded, int par) {
    const int W = c->W;
    double* hcrit = c->hcrit ? c->dgath[par] + 2 * W : nullptr;
    // sharded: defer the slab-edge F (default: two planes per neighbour on the wire, phi and w_t)
    // or recompute the neighbours' boundary stepB (FOTO_PR_EDGE=0: five planes, 2 phi + 3 mu)
    const char* pe = getenv("FOTO_PR_EDGE");
    const bool defer = W > 1 && !(pe && atoi(pe) == 0);
    FOTO_TRY(wt_drop(c));   // (a redo's prox supersedes a pending exchange)
    const bool pre = defer && wt_pre_on(c);
    if (W > 1) {
        if (defer) {
            if (!c->phi_halo) FOTO_TRY(halo(c, [](Shard& s) { return s.phi; }));
        } else {
            FOTO_TRY(exchange(c, halo_depth_xfers(c->Nt, (int64_t)c->Nx * c->Ny, W, 2), [](Shard& s) { return s.phi; },
                              [](Shard& s) { return s.phi; }));
            for (int f = 0; f < 3; ++f) FOTO_TRY(halo(c, [f](Shard& s) { return s.fz_src[f]; }));
        }
    }
    if (pre) {   // the edge planes' w_t first, then on the wire while k_prox_rhs runs
        for (auto& sp : c->sh) {
            Shard& s = *sp;
            const int dlo = s.g.t0 > 0, dhi = s.g.t0 + s.g.nloc < c->Nt;
            hipEvent_t e = c->kt.start(c->s);
            FOTO_HIP_CHECK(launch_wt_pre(s.g, s.phi, s.fz_src[0], s.fz_src[1], s.fz_src[2], c->r, s.wt, dlo, dhi, c->s,
                                         guarded ? s.spec->done_flag() : nullptr));
            c->kt.stop(e, c->s, FOTO_K_PROX, 56.0 * (double)((dlo ? 1 : 0) + (dhi ? 1 : 0)) * (double)s.g.nxy);
        }
        if (c->rccl) {
            FOTO_TRY(comm_fork(c));
            FOTO_TRY(exchange_raw(c, halo_xfers(c->Nt, (int64_t)c->Nx * c->Ny, W), [](Shard& s) { return s.wt; },
                                  [](Shard& s) { return s.wt; }));
            c->wt_pending = true;
            c->wt_guarded = guarded;
        } else {
            FOTO_TRY(halo(c, [](Shard& s) { return s.wt; }));
        }
    }
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        const double nv = (double)s.g.nloc * (double)s.g.nxy;
        const int dlo = defer && s.g.t0 > 0, dhi = defer && s.g.t0 + s.g.nloc < c->Nt;
        hipEvent_t e = c->kt.start(c->s);
        FOTO_HIP_CHECK(launch_prox_rhs(s.g, s.phi, s.fz_src[0], s.fz_src[1], s.fz_src[2], s.fz_dst[0], s.fz_dst[1],
                                       s.fz_dst[2], s.rho0, s.rhoT, c->r, s.rv, s.rb, s.gath_crit(W) + 2 * s.rank,
                                       c->o.cg_mode == 0 ? s.gath_rr() + s.rank : nullptr, c->s,
                                       guarded ? s.spec->done_flag() : nullptr, dlo, dhi, s.wt, s.edge, hcrit,
                                       pre ? 1 : 0));
        c->kt.stop(e, c->s, FOTO_K_PROX, 64.0 * nv);
    }
    if (defer && !c->wt_pending) {   // (RCCL with pre: the next forward finishes the edges)
        if (!pre) FOTO_TRY(halo(c, [](Shard& s) { return s.wt; }));
        FOTO_TRY(wt_edges(c, guarded));
    }
    c->phi_halo = false;   // (consumed: the next prox's phi comes from the next solve)
    // the stencil CG's F.F (its stopping rule) from every rank
    if (c->o.cg_mode == 0) FOTO_TRY(allgather(c, [](Shard& s) { return s.gath_rr(); }, 1));
    return 0;
}

// kmark: the KTimer mark taken before this iteration's head
static int outer_tail(foto_bb_ctx* c, size_t kmark) {
    const int W = c->W;
    Shard& s0 = *c->sh[0];
    foto_bb_ctx::Enq e;
    e.par = c->hpar;
    e.kmark = kmark;
    for (int f = 0; f < 3; ++f) {
        e.mu[f] = s0.mu[f]; e.nu[f] = s0.nu[f]; e.xi[f] = s0.xi[f];
        e.fz_src[f] = s0.fz_src[f]; e.fz_dst[f] = s0.fz_dst[f];
    }
    e.phi = s0.phi;
    e.phi_alt = s0.phi_alt;
    e.f_ready = c->f_ready;
    e.hpar = c->hpar ^ 1;   // (before this iteration's head)
    hipEvent_t* ph = c->ph[e.par];
    e.pev = phase_on(c);
    // phase boundaries are recorded, not waited on: the one host wait per outer iteration
    // is the crit readback below (a wait here idled the GPU for the host's wake-up)
    if (e.pev) FOTO_HIP_CHECK(hipEventRecord(ph[1], c->s));
    // Single shard, spectral: the solve is enqueued without a host wait and prox follows behind
    // it, guarded by the CG's done flag; the one sync (crit) then also delivers the CG result.
    // A solve that needs more work (s-step: more passes than predicted; Gauss: K beyond the
    // table) is finished after that sync, and prox re-runs (FOTO_CG_DEFER=0: always wait).
    const char* de = getenv("FOTO_CG_DEFER");
    const bool defer_on = !(de && atoi(de) == 0);
    SpectralPlan* dsp = (defer_on && W == 1 && c->o.cg_mode != 0 && s0.spec && s0.spec->deferrable())
                            ? s0.spec.get()
                            : nullptr;
    if (c->pipe && !dsp) {
        set_error("outer iteration: the pipelined loop needs a deferrable Gauss solve");
        return FOTO_ERR_STATE;
    }
    // Sharded Gauss CG: likewise enqueued whole -- x^ from the table, the all-to-all back, the
    // inverse DCTs and prox (guarded by each shard's done flag) -- and checked at the crit sync;
    // a failed solve (every rank sees the same status: the same gathered histograms) is redone
    // there with the s-step CG from b^ by every rank, so the collective sequence stays identical
    const bool sdefer = defer_on && W > 1 && s0.spec && s0.spec->gauss();
    if (c->pipe) std::swap(s0.phi, s0.phi_alt);   // this iteration's phi; the last one's stays intact
    if (dsp) {
        FOTO_TRY(dsp->solve_deferred(s0.rv, s0.phi, c->o.cg_rtol, c->o.cg_maxiter, &c->kt, c->s));
    } else if (sdefer) {
        FOTO_TRY(sharded_fwd(c));
        FOTO_TRY(sharded_gauss(c));
        FOTO_TRY(sharded_inv(c));
    } else {
        FOTO_TRY(cg_solve(c, &e.its, &e.info));
    }
    const bool guarded = dsp != nullptr || sdefer;
    if (e.pev) FOTO_HIP_CHECK(hipEventRecord(ph[2], c->s));
    c->have_phi = 1;

    if (c->fuse) {
        // prox + the next iteration's RHS: mu -> nu, F -> rv; then nu is the current mu
        // (pipelined: mu -> nu -> xi -> mu rotate, so the mu before this iteration survives it)
        for (auto& sp : c->sh)
            for (int f = 0; f < 3; ++f) { sp->fz_src[f] = sp->mu[f]; sp->fz_dst[f] = sp->nu[f]; }
        FOTO_TRY(prox_rhs(c, guarded, e.par));
        for (auto& sp : c->sh)
            for (int f = 0; f < 3; ++f) {
                if (c->pipe) {
                    double* m = sp->mu[f];
                    sp->mu[f] = sp->nu[f];
                    sp->nu[f] = sp->xi[f];
                    sp->xi[f] = m;
                } else {
                    std::swap(sp->mu[f], sp->nu[f]);
                }
            }
        c->f_ready = true;
    } else {
        if (!c->phi_halo) FOTO_TRY(halo(c, [](Shard& s) { return s.phi; }));
        c->phi_halo = false;
        for (auto& sp : c->sh) {
            Shard& s = *sp;
            const double nv = (double)s.g.nloc * (double)s.g.nxy;
            hipEvent_t t = c->kt.start(c->s);
            FOTO_HIP_CHECK(launch_prox(s.g, s.phi, s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], c->r, s.rb,
                                       s.gath_crit(W), s.rank, c->s, guarded ? s.spec->done_flag() : nullptr));
            c->kt.stop(t, c->s, FOTO_K_PROX, 80.0 * nv);
        }
    }
    FOTO_TRY(allgather(c, [W](Shard& s) { return s.gath_crit(W); }, 2));
    if (!c->hcrit)
        FOTO_HIP_CHECK(hipMemcpyAsync(c->hgath[e.par], s0.gath, sizeof(double) * 4 * W, hipMemcpyDeviceToHost, c->s));
    FOTO_HIP_CHECK(hipEventRecord(e.pev ? ph[3] : c->fin[e.par], c->s));
    e.dsp = dsp;
    e.sdefer = sdefer;
    c->inflight.push_back(e);
    return 0;
}

// Drop the newest enqueued outer iteration (pipelined loop only): wait for the stream, forget
// its solve and its timings, and put the host state back as it was before it.  F of the last
// kept iteration was overwritten by the dropped one's prox, so the next head recomputes it from
// q, itself recomputed from that iteration's phi and the mu before it (both intact).
static int rollback(foto_bb_ctx* c) {
    if (c->inflight.empty()) return 0;
    const foto_bb_ctx::Enq e = c->inflight.back();
    c->inflight.pop_back();
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    FOTO_TRY(wt_drop(c));   // (the dropped prox's w_t: the next head recomputes F whole)
    Shard& s0 = *c->sh[0];
    if (e.dsp) FOTO_TRY(e.dsp->drop_newest(c->s));
    c->kt.discard_from(e.kmark);
    for (int f = 0; f < 3; ++f) {
        s0.mu[f] = e.mu[f]; s0.nu[f] = e.nu[f]; s0.xi[f] = e.xi[f];
        s0.fz_src[f] = e.fz_src[f]; s0.fz_dst[f] = e.fz_dst[f];
    }
    s0.phi = e.phi;
    s0.phi_alt = e.phi_alt;
    c->hpar = e.hpar;
    if (e.f_ready && s0.fz_src[0]) {
        // q of the kept iteration (stepB of its phi and the mu before it), for the next head's RHS
        FOTO_HIP_CHECK(launch_q_from_phi(s0.g, s0.phi, s0.fz_src[0], s0.fz_src[1], s0.fz_src[2], s0.q[0], s0.q[1],
                                         s0.q[2], c->r, c->s));
    }
    c->f_ready = false;   // (a dropped first iteration leaves mu, q as they were: the head recomputes F)
    return 0;
}

// After an error with outer iterations on the stream: wait for the stream (errors ignored: the
// one being reported is the first), forget their deferred solves and timings, and leave no
// record behind, so foto_bb_reset can start over.
static void drain_inflight(foto_bb_ctx* c) {
    if (c->sc && c->wt_pending) {   // (a pending w_t exchange: let it land, nothing consumes it)
        (void)hipStreamSynchronize(c->sc);
        c->wt_pending = false;
    }
    if (c->inflight.empty()) return;
    (void)hipStreamSynchronize(c->s);
    for (auto it = c->inflight.rbegin(); it != c->inflight.rend(); ++it)
        if (it->dsp) (void)it->dsp->drop_newest(c->s);
    c->kt.discard_from(c->inflight.front().kmark);
    c->inflight.clear();
    c->broken = true;
}

// The host pointers of the last COMPLETED outer iteration.  Inside the iteration callback the
// next iteration is already on the stream and the shard's pointers are its own; the pipelined
// loop keeps the completed iteration's phi and mu intact (the record of the one in flight holds
// them), the one-in-flight loop does not (its next solve overwrites phi), so there a call from
// the callback is refused.
struct Completed {
    double* phi;
    double* mu[3];
    double* fz_src[3];
};
static int completed_state(foto_bb_ctx* c, const char* who, Completed* out) {
    Shard& s0 = *c->sh[0];
    if (c->inflight.empty()) {
        out->phi = s0.phi;
        for (int f = 0; f < 3; ++f) { out->mu[f] = s0.mu[f]; out->fz_src[f] = s0.fz_src[f]; }
        return 0;
    }
    if (!c->pipe) {
        set_error("%s: called while the next outer iteration is on the stream (from the iteration callback of "
                  "the one-in-flight loop, whose next solve overwrites phi); call it after foto_bb_iterate returns",
                  who);
        return FOTO_ERR_STATE;
    }
    const foto_bb_ctx::Enq& e = c->inflight.front();
    out->phi = e.phi;
    for (int f = 0; f < 3; ++f) { out->mu[f] = e.mu[f]; out->fz_src[f] = e.fz_src[f]; }
    return 0;
}

static int outer_complete(foto_bb_ctx* c, double* crit, int* cg_iters, int* cg_info) {
    const int W = c->W;
    if (c->inflight.empty()) {
        set_error("outer iteration: nothing in flight");
        return FOTO_ERR_STATE;
    }
    const foto_bb_ctx::Enq e = c->inflight.front();
    c->inflight.erase(c->inflight.begin());
    SpectralPlan* dsp = e.dsp;
    *cg_iters = e.its;
    *cg_info = e.info;
    hipEvent_t* ph = c->ph[e.par];
    const hipEvent_t done = e.pev ? ph[3] : c->fin[e.par];   // the crit readback
    FOTO_HIP_CHECK(hipEventSynchronize(done));
    if (dsp) {
        // a failed solve is redone once the iteration behind it (whose prox its done-flag chain
        // skipped) is dropped; the loop enqueues that iteration again
        if (!c->inflight.empty() && dsp->oldest_needs_redo()) FOTO_TRY(rollback(c));
        int redo = 0;
        FOTO_TRY(dsp->finish(cg_iters, cg_info, &redo, &c->kt, c->s));
        c->last_cg = *cg_iters;
        if (redo) {   // the guarded prox returned at once: drop its timing, run it on the final phi
            Shard& s = *c->sh[0];
            const double nv = (double)s.g.nloc * (double)s.g.nxy;
            c->kt.discard_last(FOTO_K_PROX, 1);
            if (c->fuse) {
                FOTO_TRY(prox_rhs(c, false, e.par));
                c->f_ready = true;   // (a rollback before the redo had cleared it)
            } else {
                hipEvent_t t = c->kt.start(c->s);
                FOTO_HIP_CHECK(launch_prox(s.g, s.phi, s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], c->r,
                                           s.rb, s.gath_crit(W), s.rank, c->s));
                c->kt.stop(t, c->s, FOTO_K_PROX, 80.0 * nv);
            }
            if (!c->hcrit)
                FOTO_HIP_CHECK(hipMemcpyAsync(c->hgath[e.par], s.gath, sizeof(double) * 4 * W, hipMemcpyDeviceToHost,
                                              c->s));
            FOTO_HIP_CHECK(hipEventRecord(done, c->s));
            FOTO_HIP_CHECK(hipEventSynchronize(done));
            c->st.cg_redo += 1;
        }
    }
    if (e.sdefer) {
        int ok = 1;
        for (auto& sp : c->sh) {
            int k_ok = 0;
            FOTO_TRY(sp->spec->gauss_result(c->o.cg_maxiter, &k_ok, cg_iters, cg_info, c->s));
            ok = ok && k_ok;   // identical on every shard and rank
        }
        if (!ok) {
            // every rank: the s-step CG from b^ (still intact: x^ went to the box scratch), the
            // inverse again, then the prox that the done flags held back, and a new crit readback
            c->kt.discard_last(FOTO_K_PROX, (int)c->sh.size());
            FOTO_TRY(sharded_sstep(c, cg_iters, cg_info));
            FOTO_TRY(sharded_inv(c));
            if (c->fuse) {
                FOTO_TRY(prox_rhs(c, false, e.par));
            } else {
                if (!c->phi_halo) FOTO_TRY(halo(c, [](Shard& s) { return s.phi; }));
                c->phi_halo = false;
                for (auto& sp : c->sh) {
                    Shard& s = *sp;
                    FOTO_HIP_CHECK(launch_prox(s.g, s.phi, s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], c->r,
                                               s.rb, s.gath_crit(W), s.rank, c->s));
                }
            }
            FOTO_TRY(allgather(c, [W](Shard& s) { return s.gath_crit(W); }, 2));
            FOTO_HIP_CHECK(hipMemcpyAsync(c->hgath[e.par], c->sh[0]->gath, sizeof(double) * 4 * W,
                                          hipMemcpyDeviceToHost, c->s));
            FOTO_HIP_CHECK(hipEventRecord(done, c->s));
            FOTO_HIP_CHECK(hipEventSynchronize(done));
            c->st.cg_redo += 1;
        }
        c->last_cg = *cg_iters;
    }
    float t_rhs = 0.f, t_cg = 0.f, t_prox = 0.f;
    if (e.pev) {
        FOTO_HIP_CHECK(hipEventElapsedTime(&t_rhs, ph[0], ph[1]));
        FOTO_HIP_CHECK(hipEventElapsedTime(&t_cg, ph[1], ph[2]));
        FOTO_HIP_CHECK(hipEventElapsedTime(&t_prox, ph[2], ph[3]));
    }
    c->st.ms_rhs += t_rhs;
    c->st.ms_cg += t_cg;
    c->st.ms_prox += t_prox;

    const double* hg = c->hgath[e.par];
    double num = 0.0, den = 0.0;
    for (int g = 0; g < W; ++g) { num += hg[2 * W + 2 * g]; den += hg[2 * W + 2 * g + 1]; }
    *crit = std::sqrt(num / (den + 1e-10));
    c->st.outer_iters += 1;
    c->st.cg_iters_total += *cg_iters;
    c->st.last_crit = *crit;
    return 0;
}

static int flow(foto_bb_ctx* c, double* u, double* v, double* m) {
    if (!c->have_phi) {
        set_error("foto_bb_flow: no outer iteration has run yet (reference: UnboundLocalError for max_it=0)");
        return FOTO_ERR_STATE;
    }
    const int W = c->W;
    FOTO_HIP_CHECK(hipEventRecord(c->fl[0], c->s));
    // Trajectories relay rank to rank: rank j runs the steps of its planes, then its
    // positions travel to rank j + 1; the last rank finishes (u, v, m) and delivers them to
    // rank 0.  The same transfer lists for both transports (exchange()).
    const int64_t nxy = (int64_t)c->Nx * c->Ny;
    auto local = [&](int rank) -> Shard* {
        for (auto& sp : c->sh)
            if (sp->rank == rank) return sp.get();
        return nullptr;
    };
    for (int j = 0; j < W; ++j) {
        if (Shard* s = local(j)) {
            const int n_lo = s->g.t0, n_hi = std::min(s->g.t0 + s->g.nloc, c->Nt - 1);
            FOTO_HIP_CHECK(launch_traj(s->g, s->phi, n_lo, std::max(n_lo, n_hi), s->px, s->py, j == 0, c->s));
            if (j == W - 1) FOTO_HIP_CHECK(launch_flow_finish(c->Nx, c->Ny, s->px, s->py, s->fu, s->fv, s->fm, c->s));
        }
        if (j + 1 < W) {
            const std::vector<Xfer> xs = relay_xfers(nxy, j);
            FOTO_TRY(exchange(c, xs, [](Shard& s) { return s.px; }, [](Shard& s) { return s.px; }));
            FOTO_TRY(exchange(c, xs, [](Shard& s) { return s.py; }, [](Shard& s) { return s.py; }));
        }
    }
    if (W > 1) {
        const std::vector<Xfer> xs = deliver_xfers(nxy, W);
        FOTO_TRY(exchange(c, xs, [](Shard& s) { return s.fu; }, [](Shard& s) { return s.fu; }));
        FOTO_TRY(exchange(c, xs, [](Shard& s) { return s.fv; }, [](Shard& s) { return s.fv; }));
        FOTO_TRY(exchange(c, xs, [](Shard& s) { return s.fm; }, [](Shard& s) { return s.fm; }));
    }
    if (Shard* s0 = local(0)) {
        if (u && v && m) {
            FOTO_HIP_CHECK(hipMemcpyAsync(u, s0->fu, nxy * sizeof(double), hipMemcpyDeviceToHost, c->s));
            FOTO_HIP_CHECK(hipMemcpyAsync(v, s0->fv, nxy * sizeof(double), hipMemcpyDeviceToHost, c->s));
            FOTO_HIP_CHECK(hipMemcpyAsync(m, s0->fm, nxy * sizeof(double), hipMemcpyDeviceToHost, c->s));
        }
    }
    FOTO_HIP_CHECK(hipEventRecord(c->fl[1], c->s));
    FOTO_HIP_CHECK(hipEventSynchronize(c->fl[1]));
    float t = 0.f;
    FOTO_HIP_CHECK(hipEventElapsedTime(&t, c->fl[0], c->fl[1]));
    c->st.ms_flow += t;
    return 0;
}

}  // namespace foto

// ============================================================================ C ABI (BB)

extern "C" {

const char* foto_last_error(void) { return foto::g_err; }
int foto_version(void) { return 1; }

int foto_device_count(int* n) {
    FOTO_HIP_CHECK(hipGetDeviceCount(n));
    return 0;
}

int foto_bb_opts_default(foto_bb_opts* o) {
    if (!o) return FOTO_ERR_ARG;
    memset(o, 0, sizeof(*o));
    o->device = -1;
    o->cg_maxiter = 1000;
    o->cg_rtol = 1e-6;
    o->cg_mode = -1;  // auto (foto_bb_create): the stencil CG on small grids, the Gauss-compressed spectral CG above
    o->rank = 0;
    o->world = 1;
    o->nccl_id = nullptr;
    o->virtual_ranks = 1;
    o->timing = 0;
    return 0;
}

int foto_xfer_calls(int kind, int Nt, int Ny, int Nx, int world, int rank, int arg, int64_t* out, int cap,
                    int* count) {
    if (!out || !count || world < 1 || rank < 0 || rank >= world || Nt < world || Ny < world || Nx < 1) {
        set_error("foto_xfer_calls: bad arguments");
        return FOTO_ERR_ARG;
    }
    const int64_t nxy = (int64_t)Nx * Ny;
    std::vector<Xfer> xs;
    switch (kind) {
        case FOTO_XFER_HALO: xs = halo_xfers(Nt, nxy, world); break;
        case FOTO_XFER_SLAB_TO_BOX: xs = alltoall_xfers(Nt, Ny, Nx, world, true); break;
        case FOTO_XFER_BOX_TO_SLAB: xs = alltoall_xfers(Nt, Ny, Nx, world, false); break;
        case FOTO_XFER_RELAY:
            if (arg < 0 || arg + 1 >= world) { set_error("foto_xfer_calls: relay step out of range"); return FOTO_ERR_ARG; }
            xs = relay_xfers(nxy, arg);
            break;
        case FOTO_XFER_DELIVER: xs = deliver_xfers(nxy, world); break;
        case FOTO_XFER_HALO2: xs = halo_depth_xfers(Nt, nxy, world, 2); break;
        case FOTO_XFER_SLAB_TO_BOX_PART:
        case FOTO_XFER_BOX_TO_SLAB_PART: {
            const int part = arg & 0xff, parts = (arg >> 8) & 0xff, halo = (arg >> 16) & 0xff;
            if (parts < 1 || part >= parts || halo > 1) { set_error("foto_xfer_calls: bad part / parts / halo"); return FOTO_ERR_ARG; }
            xs = alltoall_part_xfers(Nt, Ny, Nx, world, kind == FOTO_XFER_SLAB_TO_BOX_PART, part, parts, halo);
            break;
        }
        default: set_error("foto_xfer_calls: unknown kind %d", kind); return FOTO_ERR_ARG;
    }
    const std::vector<Call> cs = rccl_calls(xs, rank);
    *count = (int)cs.size();
    if ((int)cs.size() > cap) { set_error("foto_xfer_calls: %d calls, capacity %d", (int)cs.size(), cap); return FOTO_ERR_ARG; }
    for (size_t i = 0; i < cs.size(); ++i) {
        int64_t* o = out + 5 * i;
        o[0] = cs[i].op; o[1] = cs[i].peer; o[2] = cs[i].off; o[3] = cs[i].n; o[4] = cs[i].doff;
    }
    return 0;
}

int foto_nccl_unique_id(void* out128) {
    ncclUniqueId id;
    FOTO_NCCL_CHECK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(out128, &id, sizeof(id));
    return 0;
}

static int check_grid(int Nt, int Nx, int Ny) {
    if (Nt < 2) {
        set_error("Nt = %d: the reference needs Nt >= 2 (benamou_brenier.py:194 divides by Nt-1)", Nt);
        return FOTO_ERR_ARG;
    }
    if (Nx < 2 || Ny < 2) {
        set_error("Nx = %d, Ny = %d: operators need >= 2 points per axis (operators.py lap1d IndexError)", Nx, Ny);
        return FOTO_ERR_ARG;
    }
    return 0;
}

int foto_bb_create(const double* rho0, const double* rhoT, int Nt, int Nx, int Ny, double r, double reg_epsilon,
                   const foto_bb_opts* opts, foto_bb_ctx** out) {
    if (!rho0 || !rhoT || !out) { set_error("null argument"); return FOTO_ERR_ARG; }
    FOTO_TRY(check_grid(Nt, Nx, Ny));
    foto_bb_opts o;
    if (opts) o = *opts; else foto_bb_opts_default(&o);
    if (o.world < 1 || o.rank < 0 || o.rank >= o.world) { set_error("bad rank/world"); return FOTO_ERR_ARG; }
    if (o.world > 1 && o.virtual_ranks > 1) { set_error("virtual_ranks requires world == 1"); return FOTO_ERR_ARG; }
    if (o.world > 1 && !o.nccl_id) { set_error("world > 1 needs nccl_id"); return FOTO_ERR_ARG; }
    if (o.cg_maxiter < 0) { set_error("cg_maxiter < 0"); return FOTO_ERR_ARG; }
    if (o.cg_mode > 3) { set_error("cg_mode %d: 0..3, or < 0 for auto", o.cg_mode); return FOTO_ERR_ARG; }
    // auto (cg_mode < 0, the default): the literal 7-point stencil CG on grids of at most
    // FOTO_CG_AUTO_MAX voxels (2^18: the reference's config 1 and its golden grids, where it
    // costs milliseconds and rounds like scipy's matvec -- crit within 1e-8 of the reference, where
    // the DCT-basis CGs sit at the reference's own last-bit sensitivity, 2.6e-6 on config 1), the
    // Gauss-compressed spectral CG above (the metric grid, configs 2-5)
    if (o.cg_mode < 0) {
        const char* e = getenv("FOTO_CG_AUTO_MAX");
        const long long lim = e ? atoll(e) : (1LL << 18);
        o.cg_mode = ((long long)Nt * Nx * Ny <= lim) ? 0 : 3;
    }
    // the spectral CGs recover x = C^T((b^ - r^) / lam) and need lam > 0, i.e. eps > 0; with
    // eps <= 0 (A singular, as the reference then runs it) only the stencil CG applies
    if (o.cg_mode != 0 && !(reg_epsilon > 0.0)) o.cg_mode = 0;
    auto c = std::make_unique<foto_bb_ctx>();
    c->Nt = Nt; c->Nx = Nx; c->Ny = Ny; c->r = r; c->eps = reg_epsilon; c->o = o;
    c->rccl = o.world > 1;
    c->W = c->rccl ? o.world : std::max(1, o.virtual_ranks);
    c->kt.on = o.timing != 0;
    int rc = ctx_init(c.get(), rho0, rhoT);
    if (rc < 0) return rc;
    *out = c.release();
    return 0;
}

static int iterate_loop(foto_bb_ctx* c, int max_iters, double tol, int use_stop_rules, foto_bb_iter_cb cb,
                        void* user, int* iters_done);

int foto_bb_iterate(foto_bb_ctx* c, int max_iters, double tol, int use_stop_rules, foto_bb_iter_cb cb, void* user,
                    int* iters_done) {
    if (!c) { set_error("null ctx"); return FOTO_ERR_ARG; }
    if (iters_done) *iters_done = 0;
    if (c->broken) {
        set_error("foto_bb_iterate: a previous call failed with outer iterations in flight; foto_bb_reset the context");
        return FOTO_ERR_STATE;
    }
    if (c->in_iterate) { set_error("foto_bb_iterate: called from its own iteration callback"); return FOTO_ERR_STATE; }
    if (!c->inflight.empty()) { set_error("foto_bb_iterate: an outer iteration is still in flight"); return FOTO_ERR_STATE; }
    c->in_iterate = true;
    const int rc = iterate_loop(c, max_iters, tol, use_stop_rules, cb, user, iters_done);
    c->in_iterate = false;
    if (rc < 0) drain_inflight(c);   // (an error leaves no record behind; only a reset continues)
    return rc;
}

}  // extern "C"

static int iterate_loop(foto_bb_ctx* c, int max_iters, double tol, int use_stop_rules, foto_bb_iter_cb cb,
                        void* user, int* iters_done) {
    int done = 0;
    int stopped = 0;
    auto stop_test = [&](double crit) {
        const double prev = c->prev_crit;
        c->prev_crit = crit;
        if (!use_stop_rules) return 0;
        if (crit <= tol) return 1;
        return (prev >= 0 && std::fabs(prev - crit) < 1e-5) ? 1 : 0;
    };
    if (c->pipe) {
        // two outer iterations in flight: iteration i + 1 is on the stream before the host
        // waits for iteration i (dropped again if the stop rules end the run at i)
        int enq = 0;
        for (int i = 0; i < max_iters; ++i) {
            while ((int)c->inflight.size() < 2 && enq < max_iters) {
                const size_t km = c->kt.mark();
                FOTO_TRY(outer_head(c));
                FOTO_TRY(outer_tail(c, km));
                ++enq;
            }
            double crit;
            int its, info;
            const size_t n_before = c->inflight.size();
            FOTO_TRY(outer_complete(c, &crit, &its, &info));
            if (c->inflight.size() + 1 < n_before) --enq;   // a redo dropped the iteration behind
            ++done;
            stopped = stop_test(crit);
            if (stopped && !c->inflight.empty()) {
                FOTO_TRY(rollback(c));
                --enq;
            }
            c->kt.resolve_upto(c->inflight.empty() ? c->kt.mark() : c->inflight.front().kmark);
            if (cb) cb(user, c->st.outer_iters - 1, crit, its, info);
            if (stopped) break;
        }
        if (iters_done) *iters_done = done;
        return stopped;
    }
    // one outer iteration in flight; the next RHS goes on the stream early for a single
    // spectral shard (see outer_head)
    const bool early = c->W == 1 && c->o.cg_mode != 0;
    if (max_iters > 0) {
        const size_t km = c->kt.mark();
        FOTO_TRY(outer_head(c));
        FOTO_TRY(outer_tail(c, km));
    }
    for (int i = 0; i < max_iters; ++i) {
        double crit;
        int its, info;
        const size_t mark = c->kt.mark();
        const bool head_early = early && i + 1 < max_iters;
        if (head_early) FOTO_TRY(outer_head(c));
        const int redo0 = c->st.cg_redo;
        FOTO_TRY(outer_complete(c, &crit, &its, &info));
        ++done;
        stopped = stop_test(crit);
        // the next iteration goes on the stream before the host's bookkeeping for this one
        if (!stopped && i + 1 < max_iters) {
            // a redo re-ran this iteration's prox after the early head read mu, q: head again
            if (!head_early || c->st.cg_redo != redo0) FOTO_TRY(outer_head(c));
            FOTO_TRY(outer_tail(c, mark));
        }
        c->kt.resolve_upto(mark);
        if (cb) cb(user, c->st.outer_iters - 1, crit, its, info);
        if (stopped) break;
    }
    if (iters_done) *iters_done = done;
    return stopped;
}

extern "C" {

int foto_bb_reset(foto_bb_ctx* c, const double* rho0, const double* rhoT) {
    if (!c || !rho0 || !rhoT) { set_error("null argument"); return FOTO_ERR_ARG; }
    if (c->in_iterate) {   // (from the iteration callback: the loop still owns the in-flight state)
        set_error("foto_bb_reset: called from foto_bb_iterate's callback");
        return FOTO_ERR_STATE;
    }
    drain_inflight(c);   // (outside foto_bb_iterate nothing is in flight: a no-op unless a call failed)
    c->broken = false;
    const int64_t nxy = (int64_t)c->Nx * c->Ny;
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    for (auto& sp : c->sh) {
        Shard& s = *sp;
        const size_t bytes = (size_t)(s.g.nloc + 2) * (size_t)nxy * sizeof(double);
        double* fields[] = {s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], s.nu[0], s.nu[1], s.nu[2],
                            s.xi[0], s.xi[1], s.xi[2], s.rv, s.p[0], s.p[1]};
        for (double* f : fields)   // as ctx_init leaves them: zero, halo planes included
            if (f) FOTO_HIP_CHECK(hipMemsetAsync(f - nxy, 0, bytes, c->s));
        if (s.wt) FOTO_HIP_CHECK(hipMemsetAsync(s.wt - nxy, 0, bytes, c->s));
        if (s.edge) FOTO_HIP_CHECK(hipMemsetAsync(s.edge, 0, sizeof(double) * 8 * nxy, c->s));
        for (double* f : {s.phi, s.phi_alt})   // (two halo planes per side)
            if (f) FOTO_HIP_CHECK(hipMemsetAsync(f - 2 * nxy, 0, bytes + 2 * nxy * sizeof(double), c->s));
        FOTO_HIP_CHECK(hipMemsetAsync(s.gath, 0, sizeof(double) * 4 * c->W, c->s));
        FOTO_HIP_CHECK(hipMemsetAsync(s.rb.ticket, 0, sizeof(unsigned) * 64, c->s));
        FOTO_HIP_CHECK(hipMemsetAsync(s.S, 0, sizeof(CGScal), c->s));
        FOTO_HIP_CHECK(hipMemcpyAsync(s.rho0, rho0, nxy * sizeof(double), hipMemcpyHostToDevice, c->s));
        FOTO_HIP_CHECK(hipMemcpyAsync(s.rhoT, rhoT, nxy * sizeof(double), hipMemcpyHostToDevice, c->s));
        FOTO_HIP_CHECK(launch_init_mu(s.g, s.rho0, s.rhoT, s.mu[0], s.mu[1], s.mu[2], s.q[0], s.q[1], s.q[2], c->s));
        if (s.spec) FOTO_TRY(s.spec->reset(c->s));
    }
    c->last_cg = 0;
    c->last_passes = 0;
    c->have_phi = 0;
    c->f_ready = false;
    for (auto& sp : c->sh)
        for (int f = 0; f < 3; ++f) sp->fz_src[f] = sp->fz_dst[f] = nullptr;
    c->prev_crit = -1;
    c->st = foto_bb_stats{};
    c->kt.resolve();
    c->kt.reset();
    c->hpar = 0;
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    return 0;
}

int foto_bb_flow(foto_bb_ctx* c, double* u, double* v, double* m) {
    if (!c) { set_error("null ctx"); return FOTO_ERR_ARG; }
    if (c->broken) { set_error("foto_bb_flow: a failed foto_bb_iterate left the context inconsistent; foto_bb_reset it"); return FOTO_ERR_STATE; }
    Completed k;
    FOTO_TRY(completed_state(c, "foto_bb_flow", &k));
    // (pipelined loop, from the callback: the completed iteration's phi, then the one in flight's back)
    Shard& s0 = *c->sh[0];
    double* keep = s0.phi;
    s0.phi = k.phi;
    const int rc = flow(c, u, v, m);
    s0.phi = keep;
    return rc;
}

int foto_bb_shard(const foto_bb_ctx* c, int* t0, int* nloc) {
    if (!c) return FOTO_ERR_ARG;
    if (c->rccl) { *t0 = c->sh[0]->g.t0; *nloc = c->sh[0]->g.nloc; }
    else { *t0 = 0; *nloc = c->Nt; }
    return 0;
}

int foto_bb_comm_size(const foto_bb_ctx* c, int* nranks) {
    if (!c || !nranks) return FOTO_ERR_ARG;
    *nranks = 0;
    if (c->rccl && c->nc) FOTO_NCCL_CHECK(ncclCommCount(c->nc, nranks));
    return 0;
}

int foto_bb_get_phi(foto_bb_ctx* c, double* phi) {
    if (!c || !phi) return FOTO_ERR_ARG;
    Completed k;
    FOTO_TRY(completed_state(c, "foto_bb_get_phi", &k));
    size_t off = 0;
    for (auto& sp : c->sh) {
        const size_t n = (size_t)sp->g.nloc * sp->g.nxy;
        const double* src = (sp.get() == c->sh[0].get()) ? k.phi : sp->phi;
        FOTO_HIP_CHECK(hipMemcpyAsync(phi + off, src, n * sizeof(double), hipMemcpyDeviceToHost, c->s));
        off += n;
    }
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    return 0;
}

int foto_bb_get_state(foto_bb_ctx* c, double* mu3, double* q3) {
    if (!c) return FOTO_ERR_ARG;
    Completed k;
    FOTO_TRY(completed_state(c, "foto_bb_get_state", &k));
    auto is0 = [&](const Shard& s) { return &s == c->sh[0].get(); };
    if (q3 && c->fuse && c->have_phi) {   // the fused kernel never stores q: recompute it (bit-identical)
        for (auto& sp : c->sh) {   // (phi's halo planes are the ones the last prox read)
            Shard& s = *sp;
            double* const* src = is0(s) ? k.fz_src : s.fz_src;
            if (!src[0]) continue;
            FOTO_HIP_CHECK(launch_q_from_phi(s.g, is0(s) ? k.phi : s.phi, src[0], src[1], src[2], s.q[0], s.q[1],
                                             s.q[2], c->r, c->s));
        }
    }
    size_t tot = 0;
    for (auto& sp : c->sh) tot += (size_t)sp->g.nloc * sp->g.nxy;
    for (int f = 0; f < 3; ++f) {
        size_t off = 0;
        for (auto& sp : c->sh) {
            const size_t n = (size_t)sp->g.nloc * sp->g.nxy;
            const double* mu = is0(*sp) ? k.mu[f] : sp->mu[f];
            if (mu3) FOTO_HIP_CHECK(hipMemcpyAsync(mu3 + f * tot + off, mu, n * 8, hipMemcpyDeviceToHost, c->s));
            if (q3) FOTO_HIP_CHECK(hipMemcpyAsync(q3 + f * tot + off, sp->q[f], n * 8, hipMemcpyDeviceToHost, c->s));
            off += n;
        }
    }
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    return 0;
}

int foto_bb_stats_get(const foto_bb_ctx* c, foto_bb_stats* st) {
    if (!c || !st) return FOTO_ERR_ARG;
    *st = c->st;
    for (int k = 0; k < 8; ++k) { st->n_k[k] = c->kt.n[k]; st->ms_k[k] = c->kt.ms[k]; st->bytes_k[k] = c->kt.bytes[k]; }
    return 0;
}

int foto_bb_stats_reset(foto_bb_ctx* c) {
    if (!c) return FOTO_ERR_ARG;
    const int oi = c->st.outer_iters;
    memset(&c->st, 0, sizeof(c->st));
    c->st.outer_iters = oi;
    c->kt.reset();
    return 0;
}

int foto_bb_set_timing(foto_bb_ctx* c, int on) {
    if (!c) return FOTO_ERR_ARG;
    c->kt.on = on != 0;
    return 0;
}

int foto_bb_sync(foto_bb_ctx* c) {
    if (!c) return FOTO_ERR_ARG;
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    return 0;
}

void foto_bb_destroy(foto_bb_ctx* c) { delete c; }

int foto_bb_solve(const double* rho0, const double* rhoT, int Nt, int Nx, int Ny, double r, double tol, double eps,
                  int max_it, foto_bb_iter_cb cb, void* user, double* u, double* v, double* m) {
    foto_bb_ctx* c = nullptr;
    FOTO_TRY(foto_bb_create(rho0, rhoT, Nt, Nx, Ny, r, eps, nullptr, &c));
    int done = 0;
    int rc = foto_bb_iterate(c, max_it, tol, 1, cb, user, &done);
    if (rc >= 0) rc = foto_bb_flow(c, u, v, m);
    if (rc >= 0) rc = foto_bb_sync(c);
    foto_bb_destroy(c);
    return rc < 0 ? rc : 0;
}

namespace {
struct SolveLog {
    foto_bb_solve_stats* st;
    int n = 0;
    int64_t cg = 0;
};
void solve_log_cb(void* user, int, double crit, int its, int info) {
    SolveLog* L = (SolveLog*)user;
    foto_bb_solve_stats* st = L->st;
    if (st && L->n < st->cap) {
        if (st->crit) st->crit[L->n] = crit;
        if (st->cg_its) st->cg_its[L->n] = its;
        if (st->cg_info) st->cg_info[L->n] = info;
    }
    L->n += 1;
    L->cg += its;
}
double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

int foto_bb_solve_ex(const double* rho0, const double* rhoT, int Nt, int Nx, int Ny, double r, double tol, double eps,
                     int max_it, const foto_bb_opts* opts, double* u, double* v, double* m, double* phi_or_null,
                     foto_bb_solve_stats* st) {
    if (max_it <= 0) {
        set_error("max_it = %d: the reference's loop never runs and phi is unbound (benamou_brenier.py:271, "
                  "UnboundLocalError)", max_it);
        return FOTO_ERR_STATE;
    }
    if (st) {   // (the caller's arrays and cap stay; every output field starts at zero)
        const foto_bb_solve_stats keep = *st;
        memset(st, 0, sizeof(*st));
        st->cap = std::max(0, keep.cap);
        st->crit = keep.crit; st->cg_its = keep.cg_its; st->cg_info = keep.cg_info;
    }
    auto t0 = std::chrono::steady_clock::now();
    foto_bb_ctx* c = nullptr;
    FOTO_TRY(foto_bb_create(rho0, rhoT, Nt, Nx, Ny, r, eps, opts, &c));
    std::unique_ptr<foto_bb_ctx> guard(c);
    if (st) st->ms_create = ms_since(t0);
    SolveLog L{st};
    int done = 0;
    t0 = std::chrono::steady_clock::now();
    const int rc = foto_bb_iterate(c, max_it, tol, 1, solve_log_cb, &L, &done);
    if (rc < 0) return rc;
    FOTO_TRY(foto_bb_sync(c));
    const double ms_loop = ms_since(t0);
    t0 = std::chrono::steady_clock::now();
    FOTO_TRY(foto_bb_flow(c, u, v, m));
    if (phi_or_null) FOTO_TRY(foto_bb_get_phi(c, phi_or_null));
    FOTO_TRY(foto_bb_sync(c));
    if (st) {
        st->ms_flow = ms_since(t0);
        st->ms_loop = ms_loop;
        st->outer_iters = L.n;
        st->stopped = rc;
        FOTO_TRY(foto_bb_shard(c, &st->phi_t0, &st->phi_nloc));
        FOTO_TRY(foto_bb_stats_get(c, &st->bb));
        // the algorithmic bytes of one outer iteration on this rank: the default path's itemised
        // 188 B per voxel (bench.py STEP_BYTES_PER_VOXEL), the literal stencil
        // CG's (21 + 10 k) 8 B; the other modes from the kernel timers
        const double nv = (double)st->phi_nloc * (double)Nx * (double)Ny;
        if (c->o.cg_mode == 3) st->alg_bytes_per_iter = 188.0 * nv;
        else if (c->o.cg_mode == 0 && L.n > 0) st->alg_bytes_per_iter = (21.0 + 10.0 * (double)L.cg / L.n) * 8.0 * nv;
        else if (L.n > 0) {
            double b = 0;
            for (int k = 0; k < 8; ++k) b += st->bb.bytes_k[k];   // (summed over the launches)
            st->alg_bytes_per_iter = b / L.n;   // (0 without opts->timing)
        }
    }
    return 0;
}

}  // extern "C"

extern "C" int foto_cg(const double* b, int Nt, int Nx, int Ny, double r, double eps, double rtol, int maxiter, int mode,
                       double* x, int* iterations) {
    if (!b || !x) { set_error("null argument"); return FOTO_ERR_ARG; }
    FOTO_TRY(check_grid(Nt, Nx, Ny));
    const int64_t nxy = (int64_t)Nx * Ny, N = nxy * Nt;
    std::vector<double> z((size_t)nxy, 0.0);
    foto_bb_opts o;
    foto_bb_opts_default(&o);
    o.cg_rtol = rtol;
    o.cg_maxiter = maxiter;
    o.cg_mode = mode;
    foto_bb_ctx* c = nullptr;
    FOTO_TRY(foto_bb_create(z.data(), z.data(), Nt, Nx, Ny, r, eps, &o, &c));
    std::unique_ptr<foto_bb_ctx> guard(c);
    Shard& s = *c->sh[0];
    FOTO_HIP_CHECK(hipMemcpyAsync(s.rv, b, N * sizeof(double), hipMemcpyHostToDevice, c->s));
    FOTO_HIP_CHECK(launch_dot_self(N, s.rv, s.rb, s.gath_rr(), 0, c->s));
    int its = 0, info = 0;
    FOTO_TRY(cg_solve(c, &its, &info));
    FOTO_HIP_CHECK(hipMemcpyAsync(x, s.phi, N * sizeof(double), hipMemcpyDeviceToHost, c->s));
    FOTO_HIP_CHECK(hipStreamSynchronize(c->s));
    if (iterations) *iterations = its;
    return info;
}

// ctypes mirrors these layouts (foto/_lib.py); tests/test_cabi.py checks the Python side.
static_assert(sizeof(foto_bb_opts) == 48, "foto_bb_opts layout");
static_assert(offsetof(foto_bb_stats, n_k) == 56, "foto_bb_stats layout");
static_assert(sizeof(foto_bb_stats) == 256, "foto_bb_stats layout");
static_assert(offsetof(foto_bb_solve_stats, ms_create) == 48 && offsetof(foto_bb_solve_stats, bb) == 80 &&
                  sizeof(foto_bb_solve_stats) == 336,
              "foto_bb_solve_stats layout");
static_assert(sizeof(foto_gn_stats) == 48, "foto_gn_stats layout");
