// libfoto HIP kernels for the Benamou-Brenier (FOTO) hot path -- gfx950 / CDNA4.
//
// All arithmetic is float64 and is written in the operation order numpy/scipy use
// in the reference (the library is built with -ffp-contract=off: numpy and scipy's
// sparsetools never fuse a*b+c), so every per-voxel result is the reference's bit for
// bit; only global sums (dot products, crit sums) are reduced in a different -- fixed,
// deterministic -- order.
//
// Layout (reference operators.py:124-126): voxel k = n*Nx*Ny + j*Nx + i.  A shard owns
// planes [t0, t0+nloc); arrays carry one halo plane on each side (local l = -1, nloc).
//
// Hot kernels (stencil CG, one per CG iteration each):
//   k_cg_dir : p = r + beta p (fused), A p with a 64x4 LDS tile + 1-voxel halo, marching
//              along t with the t-neighbours in registers; p.Ap block partials.
//   k_cg_upd : x += alpha p, r -= alpha A p (A p recomputed from p: cheaper than storing
//              and re-reading q), r.r partials.
// Both finish with a last-block reduction (write-through partials + agent-scope ticket,
// MI355X_MICROARCH.md "Valid forms" row 1): no extra launch per dot product.
#include "foto_internal.h"

namespace foto {

// ============================================================================ reductions

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

// Fixed-tree block sum of K values; result valid in thread 0.  `sh` holds K*NT/64 doubles.
template <int K, int NTH = NT>
__device__ __forceinline__ void block_sum(double (&v)[K], double* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v[k] = wave_sum(v[k]);
        if (lane == 0) sh[k * (NTH / 64) + w] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double s = sh[k * (NTH / 64)];
#pragma unroll
            for (int j = 1; j < NTH / 64; ++j) s += sh[k * (NTH / 64) + j];
            v[k] = s;
        }
    }
}

// Every block contributes v[K]; the block whose ticket add comes last sums all block
// partials in block order (deterministic) and returns true with the totals in thread 0.
// Hand-off: partials stored sc1 (write-through) + vmcnt(0) before an agent-scope ticket
// add; the last block reads them with sc1 loads after its add returned and a barrier.
template <int K, int NTH = NT>
__device__ bool grid_reduce_last(double (&v)[K], RedBuf rb, double (&tot)[K]) {
    __shared__ double sh[K * (NTH / 64)];
    __shared__ int is_last;
    block_sum<K, NTH>(v, sh);
    const int nb = gridDim.x;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            __hip_atomic_store(&rb.partials[(int64_t)k * nb + blockIdx.x], v[k], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add(rb.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = (t == (unsigned)(nb - 1));
    }
    __syncthreads();
    if (!is_last) return false;
    double acc[K];
#pragma unroll
    for (int k = 0; k < K; ++k) acc[k] = 0.0;
    for (int i = threadIdx.x; i < nb; i += NTH) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            acc[k] += __hip_atomic_load(&rb.partials[(int64_t)k * nb + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    block_sum<K, NTH>(acc, sh);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) tot[k] = acc[k];
        __hip_atomic_store(rb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// ============================================================================ stencils

// One row of the space-time operator A = -r L_st + r eps I (benamou_brenier.py:202-203,
// operators.py:144-157) in scipy's CSR column order: t-1, y-1, x-1, diag, x+1, y+1, t+1.
// diag = fl(fl(r*c) + fl(r*eps)) with c = number of existing axis neighbours.
__device__ __forceinline__ double row_A(const Geo& g, int t, int y, int x, double c, double xm, double xp,
                                        double ym, double yp, double tm, double tp, double r, double reps) {
    const bool ht = t > 0, hT = t < g.Nt - 1, hy = y > 0, hY = y < g.Ny - 1, hx = x > 0, hX = x < g.Nx - 1;
    const double cnt = (double)((int)ht + (int)hT + (int)hy + (int)hY + (int)hx + (int)hX);
    const double mr = -r;
    const double dg = r * cnt + reps;
    double s = 0.0;
    if (ht) s += mr * tm;
    if (hy) s += mr * ym;
    if (hx) s += mr * xm;
    s += dg * c;
    if (hX) s += mr * xp;
    if (hY) s += mr * yp;
    if (hT) s += mr * tp;
    return s;
}

// L_st row (entries 1 off-diagonal, -c on the diagonal), same column order.
__device__ __forceinline__ double row_L(const Geo& g, int t, int y, int x, double c, double xm, double xp,
                                        double ym, double yp, double tm, double tp) {
    const bool ht = t > 0, hT = t < g.Nt - 1, hy = y > 0, hY = y < g.Ny - 1, hx = x > 0, hX = x < g.Nx - 1;
    const double cnt = (double)((int)ht + (int)hT + (int)hy + (int)hY + (int)hx + (int)hX);
    double s = 0.0;
    if (ht) s += tm;
    if (hy) s += ym;
    if (hx) s += xm;
    s += (-cnt) * c;
    if (hX) s += xp;
    if (hY) s += yp;
    if (hT) s += tp;
    return s;
}

// 2.5-D march over a 64 x TY xy tile: every thread owns one (x, y) column and walks the
// shard's planes, keeping planes t-1, t, t+1 of its column in registers.  The x/y
// neighbours of plane t come from a double-buffered LDS tile with a 1-voxel halo (one
// barrier per plane).  Loads run one plane ahead of use.
//   val(l, off)  -> field value at local plane l, in-plane offset off (in-domain only)
//   body(l, t, off, x, y, c, xm, xp, ym, yp, tm, tp)   for in-domain voxels
// Block -> tile for the column marches.  Workgroups are dispatched to the 8 XCDs round robin
// (block b on XCD b % 8), each with its own L2; give every XCD a contiguous range of row-major
// tiles instead, so the tile below a tile (ntx blocks later) is read through the same L2 and
// the y-halo rows hit there instead of being fetched from HBM again (FOTO_XCD_SWIZZLE=0 in
// the build: plain order, for A/B runs).
#ifndef FOTO_XCD_SWIZZLE
#define FOTO_XCD_SWIZZLE 1
#endif
__device__ __forceinline__ int xcd_tile(int b) {
#if FOTO_XCD_SWIZZLE
    constexpr int NXCD = 8;
    const int nb = gridDim.x, per = nb / NXCD, rem = nb % NXCD;
    const int xcd = b % NXCD, local = b / NXCD;
    return xcd * per + min(xcd, rem) + local;
#else
    return b;
#endif
}

template <class Val, class Body>
__device__ __forceinline__ void march(const Geo& g, int tile_blk, Val val, Body body) {
    const int tile = xcd_tile(tile_blk);
    constexpr int LW = TX + 2, LP = (TY + 2) * LW;
    __shared__ double lds[2 * LP];
    const int ntx = (g.Nx + TX - 1) / TX;
    const int x0 = (tile % ntx) * TX, y0 = (tile / ntx) * TY;
    const int tid = threadIdx.x, tx = tid & (TX - 1), ty = tid / TX;
    const int x = x0 + tx, y = y0 + ty;
    const bool in = (x < g.Nx) && (y < g.Ny);
    const int64_t off = in ? (int64_t)y * g.Nx + x : 0;
    // halo cell owned by this thread (rows above/below by threads 0..127, columns by 128..135)
    int hx = -1, hy = -1, hl = -1;
    if (tid < TX) { hx = x0 + tid; hy = y0 - 1; hl = tid + 1; }
    else if (tid < 2 * TX) { hx = x0 + tid - TX; hy = y0 + TY; hl = (TY + 1) * LW + (tid - TX) + 1; }
    else if (tid < 2 * TX + TY) { hx = x0 - 1; hy = y0 + (tid - 2 * TX); hl = (tid - 2 * TX + 1) * LW; }
    else if (tid < 2 * TX + 2 * TY) { hx = x0 + TX; hy = y0 + (tid - 2 * TX - TY); hl = (tid - 2 * TX - TY + 1) * LW + TX + 1; }
    const bool hv = hl >= 0 && hx >= 0 && hx < g.Nx && hy >= 0 && hy < g.Ny;
    const int64_t hoff = hv ? (int64_t)hy * g.Nx + hx : 0;
    const int ci = (ty + 1) * LW + tx + 1;
    const bool has_lo = g.t0 > 0, has_hi = g.t0 + g.nloc < g.Nt;

    double cm = 0.0, cc = 0.0, cn = 0.0, hc = 0.0;
    if (in) {
        if (has_lo) cm = val(-1, off);
        cc = val(0, off);
        if (g.nloc > 1 || has_hi) cn = val(1, off);
    }
    if (hv) hc = val(0, hoff);
    for (int l = 0; l < g.nloc; ++l) {
        double* buf = lds + (l & 1) * LP;
        buf[ci] = cc;
        if (hl >= 0) buf[hl] = hc;
        double cnn = 0.0, hnn = 0.0;
        if (in && (l + 2 < g.nloc || (l + 2 == g.nloc && has_hi))) cnn = val(l + 2, off);
        if (hv && l + 1 < g.nloc) hnn = val(l + 1, hoff);
        __syncthreads();
        if (in) {
            body(l, g.t0 + l, off, x, y, cc, buf[ci - 1], buf[ci + 1], buf[ci - LW], buf[ci + LW], cm, cn);
        }
        cm = cc;
        cc = cn;
        cn = cnn;
        hc = hnn;
    }
}

// ----------------------------------------------------------------------------- apply A / L

__global__ __launch_bounds__(NT) void k_apply_A(Geo g, const double* __restrict__ p, double* __restrict__ out,
                                                double r, double reps, int lap_only) {
    const int64_t nxy = g.nxy;
    march(g, blockIdx.x, [&](int l, int64_t off) { return p[l * nxy + off]; },
          [&](int l, int t, int64_t off, int x, int y, double c, double xm, double xp, double ym, double yp,
              double tm, double tp) {
              out[l * nxy + off] = lap_only ? row_L(g, t, y, x, c, xm, xp, ym, yp, tm, tp)
                                            : row_A(g, t, y, x, c, xm, xp, ym, yp, tm, tp, r, reps);
          });
}

hipError_t launch_apply_A(const Geo& g, const double* p, double* out, double r, double eps, int lap_only,
                          hipStream_t s) {
    k_apply_A<<<march_blocks(g), NT, 0, s>>>(g, p, out, r, r * eps, lap_only);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------- CG iteration

struct CGPro {
    bool go;
    double rr, atol, beta;
};

// Top of scipy's cg loop for iteration k: rr = r_k . r_k (sum of the per-rank slots, rank
// order), atol = rtol*||b|| (k = 0: rr = b.b), stop if ||r|| < atol; beta = rr / rho_prev.
__device__ __forceinline__ CGPro cg_prologue(int k, const CGScal* S, const double* gath_rr, const CGArgs& a,
                                             CGScal* Sw) {
    CGPro P;
    P.go = false;
    P.beta = 0.0;
    if (S->done) return P;
    double rr = 0.0;
    for (int i = 0; i < a.world; ++i) rr += gath_rr[i];
    P.rr = rr;
    if (k == 0) {
        P.atol = fmax(0.0, a.rtol * sqrt(rr));
        if (rr == 0.0) {
            if (blockIdx.x == 0 && threadIdx.x == 0) { Sw->done = 1; Sw->iters = 0; }
            return P;
        }
    } else {
        P.atol = S->atol;
    }
    if (sqrt(rr) < P.atol) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { Sw->done = 1; Sw->iters = k; }
        return P;
    }
    P.beta = (k > 0) ? rr / S->rho : 0.0;
    P.go = true;
    return P;
}

template <bool FUSED>
__global__ __launch_bounds__(NT) void k_cg_dir(Geo g, int k, const double* __restrict__ rv,
                                               const double* __restrict__ po, double* __restrict__ pn, CGArgs a,
                                               CGScal* S, RedBuf rb, const double* __restrict__ gath_rr,
                                               double* __restrict__ gath_pap) {
    const CGPro P = cg_prologue(k, S, gath_rr, a, S);
    if (!P.go) return;
    const int64_t nxy = g.nxy;
    const double beta = P.beta, r = a.r, reps = a.r * a.eps;
    double acc = 0.0;
    march(
        g, blockIdx.x,
        [&](int l, int64_t off) -> double {
            const int64_t i = l * nxy + off;
            if (!FUSED) return pn[i];
            if (k == 0) return rv[i];
            return beta * po[i] + rv[i];   // scipy: p *= beta; p += z
        },
        [&](int l, int t, int64_t off, int x, int y, double c, double xm, double xp, double ym, double yp,
            double tm, double tp) {
            const double q = row_A(g, t, y, x, c, xm, xp, ym, yp, tm, tp, r, reps);
            acc += c * q;
            if (FUSED) pn[l * nxy + off] = c;
        });
    double v[1] = {acc}, tot[1];
    if (grid_reduce_last<1>(v, rb, tot) && threadIdx.x == 0) {
        S->rho = P.rr;
        if (k == 0) { S->bb = P.rr; S->atol = P.atol; }
        S->pap = tot[0];
        gath_pap[a.rank] = tot[0];
    }
}

// Pointwise p = r + beta p for the sharded (non-fused) path: the halo planes of the new p
// are then exchanged before k_cg_dir<false> applies A.
__global__ __launch_bounds__(NT) void k_cg_pupd(Geo g, int k, const double* __restrict__ rv,
                                                const double* __restrict__ po, double* __restrict__ pn,
                                                CGScal* S, const double* __restrict__ gath_rr, CGArgs a) {
    // decision only (no state writes: k_cg_dir<false> repeats the prologue and writes)
    if (S->done) return;
    double rr = 0.0;
    for (int i = 0; i < a.world; ++i) rr += gath_rr[i];
    double atol = (k == 0) ? fmax(0.0, a.rtol * sqrt(rr)) : S->atol;
    if (rr == 0.0 || sqrt(rr) < atol) return;
    const double beta = (k > 0) ? rr / S->rho : 0.0;
    const int64_t n = (int64_t)g.nloc * g.nxy;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT)
        pn[i] = (k == 0) ? rv[i] : beta * po[i] + rv[i];
}

__global__ __launch_bounds__(NT) void k_cg_upd(Geo g, int k, const double* __restrict__ p, double* __restrict__ xv,
                                               double* __restrict__ rv, CGArgs a, CGScal* S, RedBuf rb,
                                               const double* __restrict__ gath_pap, double* __restrict__ gath_rr) {
    if (S->done) return;
    double pap = 0.0;
    for (int i = 0; i < a.world; ++i) pap += gath_pap[i];
    const double alpha = S->rho / pap;
    const int64_t nxy = g.nxy;
    const double r = a.r, reps = a.r * a.eps;
    double acc = 0.0;
    march(
        g, blockIdx.x, [&](int l, int64_t off) -> double { return p[l * nxy + off]; },
        [&](int l, int t, int64_t off, int x, int y, double c, double xm, double xp, double ym, double yp,
            double tm, double tp) {
            const double q = row_A(g, t, y, x, c, xm, xp, ym, yp, tm, tp, r, reps);
            const int64_t i = l * nxy + off;
            const double ap = alpha * c;
            xv[i] = (k == 0) ? 0.0 + ap : xv[i] + ap;   // x += alpha*p
            const double rn = rv[i] - alpha * q;       // r -= alpha*q
            rv[i] = rn;
            acc += rn * rn;
        });
    double v[1] = {acc}, tot[1];
    if (grid_reduce_last<1>(v, rb, tot) && threadIdx.x == 0) gath_rr[a.rank] = tot[0];
}

hipError_t launch_cg_dir(const Geo& g, int k, const double* rvec, const double* pold, double* pnew,
                         const CGArgs& a, CGScal* S, RedBuf rb, const double* gath_rr, double* gath_pap,
                         int fused, hipStream_t s) {
    if (fused)
        k_cg_dir<true><<<march_blocks(g), NT, 0, s>>>(g, k, rvec, pold, pnew, a, S, rb, gath_rr, gath_pap);
    else
        k_cg_dir<false><<<march_blocks(g), NT, 0, s>>>(g, k, rvec, pold, pnew, a, S, rb, gath_rr, gath_pap);
    return hipGetLastError();
}

hipError_t launch_cg_pupd(const Geo& g, int k, const double* rvec, const double* pold, double* pnew, CGScal* S,
                          const double* gath_rr, const CGArgs& a, hipStream_t s) {
    const int64_t n = (int64_t)g.nloc * g.nxy;
    int nb = (int)std::min<int64_t>((n + NT - 1) / NT, 4096);
    k_cg_pupd<<<nb, NT, 0, s>>>(g, k, rvec, pold, pnew, S, gath_rr, a);
    return hipGetLastError();
}

hipError_t launch_cg_upd(const Geo& g, int k, const double* p, double* x, double* rvec, const CGArgs& a,
                         CGScal* S, RedBuf rb, const double* gath_pap, double* gath_rr, hipStream_t s) {
    k_cg_upd<<<march_blocks(g), NT, 0, s>>>(g, k, p, x, rvec, a, S, rb, gath_pap, gath_rr);
    return hipGetLastError();
}

// ============================================================================ gradients / divergence

// grad_1d_central_weird (bc 'N', h = 1) row at index k of an axis of length n, given the
// values at k-1, k, k+1 (operators.py:33-48).  (-0.5 a) + (0.5 b) == 0.5 (b - a) exactly.
__device__ __forceinline__ double d1w(int k, int n, double m, double c, double p) {
    if (k == 0) return p - c;
    if (k == n - 1) return c - m;
    return 0.5 * (p - m);
}

__global__ __launch_bounds__(NT) void k_grad_st(Geo g, const double* __restrict__ phi, double* __restrict__ gt,
                                                double* __restrict__ gx, double* __restrict__ gy) {
    const int64_t n = (int64_t)g.nloc * g.nxy;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const int l = (int)(i / g.nxy);
    const int64_t off = i - (int64_t)l * g.nxy;
    const int y = (int)(off / g.Nx), x = (int)(off - (int64_t)y * g.Nx), t = g.t0 + l;
    const double c = phi[i];
    gt[i] = d1w(t, g.Nt, t > 0 ? phi[i - g.nxy] : 0.0, c, t < g.Nt - 1 ? phi[i + g.nxy] : 0.0);
    gx[i] = d1w(x, g.Nx, x > 0 ? phi[i - 1] : 0.0, c, x < g.Nx - 1 ? phi[i + 1] : 0.0);
    gy[i] = d1w(y, g.Ny, y > 0 ? phi[i - g.Nx] : 0.0, c, y < g.Ny - 1 ? phi[i + g.Nx] : 0.0);
}

hipError_t launch_grad_st(const Geo& g, const double* phi, double* gt, double* gx, double* gy, hipStream_t s) {
    k_grad_st<<<flat_blocks((int64_t)g.nloc * g.nxy), NT, 0, s>>>(g, phi, gt, gx, gy);
    return hipGetLastError();
}

// div_st row (operators.py:129-142): scipy's COO matvec accumulates the t-block terms, then
// the x-block, then the y-block, each in ascending column order, starting from 0.
__device__ __forceinline__ void acc_d1w(double& s, int k, int n, double m, double c, double p) {
    if (k == 0) { s += -1.0 * c; s += 1.0 * p; }
    else if (k == n - 1) { s += -1.0 * m; s += 1.0 * c; }
    else { s += -0.5 * m; s += 0.5 * p; }
}

template <class W>
__device__ __forceinline__ double div_st_row(const Geo& g, int64_t i, int t, int y, int x, W w) {
    double s = 0.0;
    acc_d1w(s, t, g.Nt, t > 0 ? w(0, i - g.nxy) : 0.0, w(0, i), t < g.Nt - 1 ? w(0, i + g.nxy) : 0.0);
    acc_d1w(s, x, g.Nx, x > 0 ? w(1, i - 1) : 0.0, w(1, i), x < g.Nx - 1 ? w(1, i + 1) : 0.0);
    acc_d1w(s, y, g.Ny, y > 0 ? w(2, i - g.Nx) : 0.0, w(2, i), y < g.Ny - 1 ? w(2, i + g.Nx) : 0.0);
    return s;
}

__global__ __launch_bounds__(NT) void k_div_st(Geo g, const double* __restrict__ wt, const double* __restrict__ wx,
                                               const double* __restrict__ wy, double* __restrict__ out) {
    const int64_t n = (int64_t)g.nloc * g.nxy;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const int l = (int)(i / g.nxy);
    const int64_t off = i - (int64_t)l * g.nxy;
    const int y = (int)(off / g.Nx), x = (int)(off - (int64_t)y * g.Nx);
    const double* W[3] = {wt, wx, wy};
    out[i] = div_st_row(g, i, g.t0 + l, y, x, [&](int f, int64_t j) { return W[f][j]; });
}

hipError_t launch_div_st(const Geo& g, const double* wt, const double* wx, const double* wy, double* out,
                         hipStream_t s) {
    k_div_st<<<flat_blocks((int64_t)g.nloc * g.nxy), NT, 0, s>>>(g, wt, wx, wy, out);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------- RHS (stepA)

// F = div_st(mu - r q); F[t=0] -= rho0 - rho[0] + r a[0]; F[t=Nt-1] += rhoT - rho + r a
// (benamou_brenier.py:64-82, dt = 1).  F.F partial -> gath[rank] (= b.b for CG).
#ifndef FOTO_RHS_TY
#define FOTO_RHS_TY 1
#endif
constexpr int RHS_TY = FOTO_RHS_TY;    // rows per block: the y-neighbour rows a tile re-reads are 2 / RHS_TY extra
constexpr int RHS_NT = TX * RHS_TY;
__global__ __launch_bounds__(RHS_NT) void k_rhs(Geo g, const double* __restrict__ mut, const double* __restrict__ mux,
                                            const double* __restrict__ muy, const double* __restrict__ qt,
                                            const double* __restrict__ qx, const double* __restrict__ qy,
                                            const double* __restrict__ rho0, const double* __restrict__ rhoT,
                                            double r, double* __restrict__ F, RedBuf rb, double* gath, int rank,
                                            int tch) {
    // one thread per (x, y) column of a 64 x RHS_TY tile, marching over a chunk of tch of the
    // shard's planes (chunks: more columns in flight than the 307 k of one full march, at the
    // cost of re-reading the t-field of two planes per chunk); the t-field w_t = mu_t - r q_t
    // of planes t-1, t, t+1 stays in registers (loaded one plane ahead), the x / y fields'
    // neighbours are same-row / adjacent-row loads (L1 / L2 hits).
    const int ntx = (g.Nx + TX - 1) / TX, ntiles = ntx * ((g.Ny + RHS_TY - 1) / RHS_TY);
    const int lin = xcd_tile(blockIdx.x);
    const int ch = lin / ntiles, tile = lin - ch * ntiles;
    const int l0 = ch * tch, l1 = min(g.nloc, l0 + tch);
    const int x = (tile % ntx) * TX + (threadIdx.x & (TX - 1));
    const int y = (tile / ntx) * RHS_TY + threadIdx.x / TX;
    const bool in = x < g.Nx && y < g.Ny && l0 < g.nloc;
    const int64_t nxy = g.nxy, off = in ? (int64_t)y * g.Nx + x : 0;
    const bool has_lo = g.t0 > 0, has_hi = g.t0 + g.nloc < g.Nt;
    auto wt = [&](int l) { const int64_t i = l * nxy + off; return mut[i] - r * qt[i]; };
    auto wx = [&](int64_t i) { return mux[i] - r * qx[i]; };
    auto wy = [&](int64_t i) { return muy[i] - r * qy[i]; };
    double ff = 0.0;
    if (in) {
        double tm = (l0 > 0 || has_lo) ? wt(l0 - 1) : 0.0, tc = wt(l0);
        double tp = (l0 + 1 < g.nloc || has_hi) ? wt(l0 + 1) : 0.0;
        for (int l = l0; l < l1; ++l) {
            const int t = g.t0 + l;
            const double tpp =
                (l + 1 < l1 && (l + 2 < g.nloc || (l + 2 == g.nloc && has_hi))) ? wt(l + 2) : 0.0;
            const int64_t i = l * nxy + off;
            double s = 0.0;
            acc_d1w(s, t, g.Nt, tm, tc, tp);
            acc_d1w(s, x, g.Nx, x > 0 ? wx(i - 1) : 0.0, wx(i), x < g.Nx - 1 ? wx(i + 1) : 0.0);
            acc_d1w(s, y, g.Ny, y > 0 ? wy(i - g.Nx) : 0.0, wy(i), y < g.Ny - 1 ? wy(i + g.Nx) : 0.0);
            if (t == 0) s -= (rho0[off] - mut[i]) + r * qt[i];
            if (t == g.Nt - 1) s += (rhoT[off] - mut[i]) + r * qt[i];
            F[i] = s;
            ff += s * s;
            tm = tc;
            tc = tp;
            tp = tpp;
        }
    }
    if (!gath) return;   // F.F only feeds the stencil CG's stopping rule (the spectral CG takes it from b^)
    double v[1] = {ff}, tot[1];
    if (grid_reduce_last<1, RHS_NT>(v, rb, tot) && threadIdx.x == 0) gath[rank] = tot[0];
}

hipError_t launch_rhs(const Geo& g, const double* mut, const double* mux, const double* muy, const double* qt,
                      const double* qx, const double* qy, const double* rho0, const double* rhoT, double r,
                      double* F, RedBuf rb, double* gath, int rank, hipStream_t s) {
    // planes per chunk (FOTO_RHS_TCH; default 8: four chunks at Nt = 32)
    static const int tch = [] {
        const char* e = getenv("FOTO_RHS_TCH");
        const int v = e ? atoi(e) : 8;
        return v > 0 ? v : 8;
    }();
    const int nch = (g.nloc + tch - 1) / tch;
    const int nb = ((g.Nx + TX - 1) / TX) * ((g.Ny + RHS_TY - 1) / RHS_TY) * nch;
    k_rhs<<<nb, RHS_NT, 0, s>>>(g, mut, mux, muy, qt, qx, qy, rho0, rhoT, r, F, rb, gath, rank, tch);
    return hipGetLastError();
}

// mu_rho[n] = (1 - n/(Nt-1)) rho0 + (n/(Nt-1)) rhoT, m = 0, q = 0 (benamou_brenier.py:191-194)
__global__ __launch_bounds__(NT) void k_init_mu(Geo g, const double* __restrict__ rho0,
                                                const double* __restrict__ rhoT, double* mut, double* mux,
                                                double* muy, double* qt, double* qx, double* qy) {
    const int64_t n = (int64_t)g.nloc * g.nxy;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const int l = (int)(i / g.nxy);
    const int64_t off = i - (int64_t)l * g.nxy;
    const double s = (double)(g.t0 + l) / (double)(g.Nt - 1);
    mut[i] = (1.0 - s) * rho0[off] + s * rhoT[off];
    mux[i] = 0.0;
    muy[i] = 0.0;
    qt[i] = 0.0;
    qx[i] = 0.0;
    qy[i] = 0.0;
}

hipError_t launch_init_mu(const Geo& g, const double* rho0, const double* rhoT, double* mut, double* mux,
                          double* muy, double* qt, double* qx, double* qy, hipStream_t s) {
    k_init_mu<<<flat_blocks((int64_t)g.nloc * g.nxy), NT, 0, s>>>(g, rho0, rhoT, mut, mux, muy, qt, qx, qy);
    return hipGetLastError();
}

// ============================================================================ stepB (A8)

// The projection of benamou_brenier.py:123-148 with the reference's branch tests and
// closed forms, in an algebraically identical but cheaper form: (cos, sin)(atan2(b2, b1))
// = (b1, b2) / |b|, x^(1/3) -> cbrt(x), (a+1)^3 and m^(3/2) by products.  Each changes a
// result by at most an ulp or two (checked to 1e-12 against the reference's stepB in
// tests/golden/stepb.npz, including both branches and the boundary); stepB runs once per
// outer iteration on every voxel, and atan2 / cos / sin / pow would dominate it.
// rare branch (a < -1, small |b|): kept out of line so its acos / cos do not inflate the
// register allocation of the kernels that inline project_K
__device__ __noinline__ double proj_trig_z(double al, double rho) {
    const double m = -al - 1.0;
    const double sm = sqrt(m);
    return 1.632993161855452 * sm * cos(0.3333333333333333 * acos(1.8371173070873836 * rho / (m * sm)));
}

// S^(1/3) and S^(-1/3) for finite S > 0 without the library cbrt and a division: S = m 2^e
// (m in [0.5, 1)), e = 3q + s (s in {0, 1, 2}), S' = m 2^s in [0.5, 4); y ~ S'^(-1/3) from the
// fp32 log2 / exp2 (~1e-7 relative), two Newton steps y <- y (4 - S' y^3) / 3 (quadratic:
// rounding level), then S^(1/3) = S' y^2 2^q and S^(-1/3) = y 2^-q.  Within 2-3 ulp of the
// rounded values (the reference's x ** (1/3) is itself within an ulp of them).
#ifndef FOTO_PROJ_FAST
#define FOTO_PROJ_FAST 1
#endif
__device__ __forceinline__ void cbrt_pair(double S, double& c, double& ic) {
    const int e = __builtin_amdgcn_frexp_exp(S);
    const double m = __builtin_amdgcn_frexp_mant(S);
    const int q = (e >= 0) ? e / 3 : -((2 - e) / 3);   // floor(e / 3)
    const double Sp = __builtin_amdgcn_ldexp(m, e - 3 * q);
    const float yf = __builtin_amdgcn_exp2f(-0.3333333333f * __builtin_amdgcn_logf((float)Sp));
    double y = (double)yf;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double y3 = (y * y) * y;
        y = (y * fma(-Sp, y3, 4.0)) * 0.3333333333333333;
    }
    c = __builtin_amdgcn_ldexp((Sp * y) * y, q);
    ic = __builtin_amdgcn_ldexp(y, -q);
}

__device__ __forceinline__ void project_K(double al, double b1, double b2, double& oa, double& o1, double& o2) {
    if (2.0 * al + b1 * b1 + b2 * b2 <= 0.0) {
        oa = al; o1 = b1; o2 = b2;
        return;
    }
    const double SQRT2 = 1.4142135623730951;
    const double rho = sqrt(b1 * b1 + b2 * b2);
    const double ap1 = al + 1.0;
    double aH, rH;
    if (-32.0 * (ap1 * ap1 * ap1) - 108.0 * (rho * rho) < 0.0) {
        const double S = 0.3535533905932738 * rho +
                         0.16666666666666666 * sqrt(1.3333333333333333 * (al * al * al) + 4.0 * (al * al) +
                                                    4.5 * (rho * rho) + 4.0 * al + 1.3333333333333333);
#if FOTO_PROJ_FAST
        double c, ic;
        if (S > 0.0 && S <= 1.7976931348623157e308) {
            cbrt_pair(S, c, ic);
        } else {
            c = cbrt(S);
            ic = 1.0 / c;
        }
        const double zh = fma(-0.3333333333333333 * ap1, ic, c);
#else
        const double c = cbrt(S);
        const double zh = (-0.3333333333333333 * ap1) / c + c;
#endif
        aH = -(zh * zh);
        rH = SQRT2 * zh;
    } else {
        const double zh = proj_trig_z(al, rho);
        aH = -0.5 * (zh * zh);
        rH = zh;
    }
    oa = aH;
    if (rho > 0.0) {
#if FOTO_PROJ_FAST
        const double ir = 1.0 / rho;
        o1 = rH * (b1 * ir);
        o2 = rH * (b2 * ir);
#else
        o1 = rH * (b1 / rho);
        o2 = rH * (b2 / rho);
#endif
    } else {   // atan2(+-0, +0) = +-0, atan2(+-0, -0) = +-pi
        o1 = signbit(b1) ? -rH : rH;
        o2 = 0.0;
    }
}

__global__ __launch_bounds__(NT) void k_stepB(int64_t M, const double* __restrict__ pa, const double* __restrict__ p1,
                                              const double* __restrict__ p2, double* __restrict__ qa,
                                              double* __restrict__ q1, double* __restrict__ q2) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= M) return;
    double a, b, c;
    project_K(pa[i], p1[i], p2[i], a, b, c);
    qa[i] = a;
    q1[i] = b;
    q2[i] = c;
}

hipError_t launch_stepB(int64_t M, const double* pa, const double* p1, const double* p2, double* qa, double* q1,
                        double* q2, hipStream_t s) {
    k_stepB<<<flat_blocks(M), NT, 0, s>>>(M, pa, p1, p2, qa, q1, q2);
    return hipGetLastError();
}

// ============================================================================ stepB + stepC + crit (fused)

// g = grad_st phi; q = Proj_K(g + (1/r) mu); mu += r (g - q); mu_rho = max(mu_rho, 0);
// num += mu_rho |g_t + (g_x^2 + g_y^2)/2|, den += mu_rho (g_x^2 + g_y^2)
// (benamou_brenier.py:213-248).
__global__ __launch_bounds__(NT) void k_prox(Geo g, const double* __restrict__ phi, double* __restrict__ mut,
                                             double* __restrict__ mux, double* __restrict__ muy,
                                             double* __restrict__ qt, double* __restrict__ qx,
                                             double* __restrict__ qy, double r, double inv_r, RedBuf rb,
                                             double* gath, int rank, const int* __restrict__ guard) {
    // 2.5-D march over phi (64 x 4 LDS tile + halo, t-neighbours in registers), then the
    // pointwise stepB / stepC / criterion terms of each voxel.
    // guard: the CG's done flag when the host enqueued this without waiting for the solve; an
    // unfinished solve leaves mu, q untouched and the host re-runs prox after finishing it.
    if (guard && *guard == 0) return;
    const int64_t nxy = g.nxy;
    double num = 0.0, den = 0.0;
    march(g, blockIdx.x, [&](int l, int64_t off) { return phi[l * nxy + off]; },
          [&](int l, int t, int64_t off, int x, int y, double c, double xm, double xp, double ym, double yp,
              double tm, double tp) {
              const int64_t i = l * nxy + off;
              const double gt = d1w(t, g.Nt, tm, c, tp);
              const double gx = d1w(x, g.Nx, xm, c, xp);
              const double gy = d1w(y, g.Ny, ym, c, yp);
              const double m0 = mut[i], m1 = mux[i], m2 = muy[i];
              double a, b1, b2;
              project_K(gt + inv_r * m0, gx + inv_r * m1, gy + inv_r * m2, a, b1, b2);
              qt[i] = a;
              qx[i] = b1;
              qy[i] = b2;
              double n0 = m0 + r * (gt - a);
              n0 = (n0 < 0.0) ? 0.0 : n0;   // np.maximum(mu, 0) (NaN propagates)
              mut[i] = n0;
              mux[i] = m1 + r * (gx - b1);
              muy[i] = m2 + r * (gy - b2);
              const double gg = gx * gx + gy * gy;
              num += n0 * fabs(gt + 0.5 * gg);
              den += n0 * gg;
          });
    double v[2] = {num, den}, tot[2];
    if (grid_reduce_last<2>(v, rb, tot) && threadIdx.x == 0) {
        gath[2 * rank] = tot[0];
        gath[2 * rank + 1] = tot[1];
    }
}

hipError_t launch_prox(const Geo& g, const double* phi, double* mut, double* mux, double* muy, double* qt,
                       double* qx, double* qy, double r, RedBuf rb, double* gath, int rank, hipStream_t s,
                       const int* guard) {
    k_prox<<<march_blocks(g), NT, 0, s>>>(g, phi, mut, mux, muy, qt, qx, qy, r, 1.0 / r, rb, gath, rank, guard);
    return hipGetLastError();
}

// q = Proj_K(grad_st phi + mu / r) alone (k_prox's formulas; mu untouched): the stepB output of
// the last outer iteration, recomputed on demand where the fused kernel below never stores it.
__global__ __launch_bounds__(NT) void k_q_from_phi(Geo g, const double* __restrict__ phi,
                                                   const double* __restrict__ mut, const double* __restrict__ mux,
                                                   const double* __restrict__ muy, double* __restrict__ qt,
                                                   double* __restrict__ qx, double* __restrict__ qy, double inv_r) {
    const int64_t nxy = g.nxy;
    march(g, blockIdx.x, [&](int l, int64_t off) { return phi[l * nxy + off]; },
          [&](int l, int t, int64_t off, int x, int y, double c, double xm, double xp, double ym, double yp,
              double tm, double tp) {
              const int64_t i = l * nxy + off;
              double a, b1, b2;
              project_K(d1w(t, g.Nt, tm, c, tp) + inv_r * mut[i], d1w(x, g.Nx, xm, c, xp) + inv_r * mux[i],
                        d1w(y, g.Ny, ym, c, yp) + inv_r * muy[i], a, b1, b2);
              qt[i] = a;
              qx[i] = b1;
              qy[i] = b2;
          });
}

hipError_t launch_q_from_phi(const Geo& g, const double* phi, const double* mut, const double* mux,
                             const double* muy, double* qt, double* qx, double* qy, double r, hipStream_t s) {
    k_q_from_phi<<<march_blocks(g), NT, 0, s>>>(g, phi, mut, mux, muy, qt, qx, qy, 1.0 / r);
    return hipGetLastError();
}

// ============================================================================ prox + next RHS (fused)
//
// One outer iteration's stepB / stepC / criterion (k_prox) fused with the NEXT iteration's
// right-hand side (k_rhs): F = div_st(mu' - r q) + BC needs only the new mu' and q of a voxel
// and its six neighbours, so the kernel that produces them can finish F itself -- q is never
// stored and mu' is never re-read (k_prox + k_rhs move 80 + 56 B per voxel, this kernel
// 8 (phi) + 24 (mu) + 24 (mu') + 8 (F) = 64 B).  The price is the neighbours' stepB: a block
// owns a 64 x 8 tile of F over a chunk of planes [l0, l1) and computes stepB on the tile plus
// a one-voxel ring (66 x 10: the x / y neighbours F needs) and on the planes l0 - 1 and l1
// (the t neighbours), which needs phi on a two-voxel ring (68 x 12) and planes l0 - 2 .. l1 + 1.
// mu' goes to a second buffer (neighbouring blocks still read the old mu of their ring voxels).
// Time-sharded there are two ways across a slab boundary.  EDGE RECOMPUTE (FOTO_PR_EDGE=0): a
// shard's first and last chunks recompute stepB on the neighbouring ranks' boundary planes
// exactly as the chunk seams do -- phi needs two halo planes and mu one on each side, five
// planes per neighbour on the wire.  EDGE DEFER (default): stepB stays on the own planes, F of a
// plane next to another rank is deferred -- the kernel stores w_t of its two outermost planes on
// each deferred side and (w_x, w_y, mu'_t, q_t) of the edge plane itself, one w_t plane is
// exchanged with each neighbour, and k_rhs_edge finishes F there with the same operations in the
// same order: phi one halo plane, w_t one -- two planes per neighbour.  Plane indices p are local
// (memory: p * nxy); t = t0 + p is global (boundary conditions).  Per voxel the arithmetic is k_prox's and k_rhs's, in the same order:
// mu', F and the crit terms are bit-identical to the unfused kernels; only the crit / F.F sums
// are grouped differently.
//
// Iteration p of the march (p = max(l0 - 1, 0) .. l1): store phi(p + 2) (loaded during the
// previous iteration) into a 4-plane LDS ring, issue the loads of phi(p + 3) and mu(p + 1),
// stepB on plane p (phi planes p - 1 .. p + 1 from the ring) -> w = mu' - r q of plane p into
// a double-buffered LDS image (x, y parts; the own voxel's t part stays in registers), then
// F(p - 1) from w of planes p - 2 .. p; one barrier per iteration.  Threads 0..147 (waves
// 0-2) also take the 148 ring voxels.  Chunks of FOTO_PR_TCH planes (default 16) give the
// grid more blocks than resident slots (a full-length march leaves a one-sixth-full second
// round at 640 x 480).
#ifndef FOTO_PR_Y
#define FOTO_PR_Y 8
#endif
// mu' is read again only by the next outer iteration's prox, ~1.5 GB of other traffic later:
// stored non-temporal it does not displace the lines the next kernels read (F, phi) --
// 1646 -> 1655 it/s, the prox launch itself +1 us (A/B, profiles/r04n_ab_prox_nt.txt);
// 2: F non-temporal too (the x-DCT reads it next: no better); 0: plain stores
#ifndef FOTO_PR_NT
#define FOTO_PR_NT 1
#endif
// The old mu is dead after this kernel: its loads are non-temporal.  Own voxels only (1):
// 1675-1688 -> 1708-1719 it/s, the DCT chain after it 130 -> 124 us (F stays cached for the
// x-DCT); the ring voxels' loads too (2, default): 1690-1716 -> 1703-1740, the prox launch
// unchanged (A/B, profiles/r04n_ab_nt_loads.txt).  0: plain loads.
#ifndef FOTO_PR_NTLD
#define FOTO_PR_NTLD 2
#endif
#ifndef FOTO_PR_NTPHI
#define FOTO_PR_NTPHI 0  // 1: phi loaded non-temporal (prox 165 -> 173 us: its halo is re-read)
#endif
#ifndef FOTO_PR_X
#define FOTO_PR_X 64
#endif
// own voxels per thread (FOTO_PR_VPT=2 with FOTO_PR_Y=16: a 64 x 16 tile on 512 threads, rows y and
// y + 8 per thread, the ring 164 voxels for 1024 instead of 148 for 512; 81.5 KB of LDS, so one
// block per CU at up to 256 VGPRs)
#ifndef FOTO_PR_VPT
#define FOTO_PR_VPT 1
#endif
// 1: tiles whose phi region lies inside the plane run a copy of the march without bound tests
// (prox_rhs_body<.., true>); 0: every tile runs the general one (A/B builds)
#ifndef FOTO_PR_CHFAST
#define FOTO_PR_CHFAST 0   // 1: block order tile-major with the chunks fastest (A/B builds)
#endif
#ifndef FOTO_PR_INTERIOR
#define FOTO_PR_INTERIOR 1
#endif
constexpr int PR_X = FOTO_PR_X, PR_Y = FOTO_PR_Y, PR_VPT = FOTO_PR_VPT;
constexpr int PR_NT = PR_X * PR_Y / PR_VPT;                 // 512 threads (64 x 8)
constexpr int PR_YV = PR_Y / PR_VPT;                        // rows between a thread's own voxels
constexpr int PR_PW = PR_X + 2, PR_PH = PR_Y + 2;         // stepB region
constexpr int PR_FW = PR_X + 4, PR_FH = PR_Y + 4;         // phi region
constexpr int PR_HALO = 2 * PR_PW + 2 * PR_Y;             // 148 ring voxels (64 x 8)
constexpr int PR_FN = PR_FW * PR_FH;                      // 816 phi values per plane
constexpr int PR_FR = (PR_FN + PR_NT - 1) / PR_NT;        // phi loads per thread per plane
static_assert(PR_X == 64 && PR_NT <= 1024 && PR_HALO <= PR_NT && PR_Y % PR_VPT == 0,   // (32 x 16, 16 x 32, 32 x 8: slower, r03)
              "whole rows per thread, ring voxels on the first threads");
constexpr int PR_WPE = PR_VPT == 1 ? 4 : 2;               // waves per SIMD (VGPR budget 128 / 256)

// EDGE: the deferred-edge variant (sharded); the single-shard instantiation carries none of its
// code (its extra registers spilled the kernel at the 128-VGPR cap: 171 -> 184 us)
// INTERIOR (round 6): the block's whole phi region (the tile plus a two-voxel ring) lies inside
// the plane, so every own voxel, ring voxel and phi load is in the grid and every x / y
// neighbour F reads exists -- the per-lane bound tests and the branches around the loads they
// guard fold away (77 % of the blocks at 640 x 480).  The same arithmetic in the same order.
template <bool EDGE, bool INTERIOR>
__device__ __forceinline__ void prox_rhs_body(
        Geo g, const double* __restrict__ phi, const double* __restrict__ mut, const double* __restrict__ mux,
        const double* __restrict__ muy, double* __restrict__ nut, double* __restrict__ nux, double* __restrict__ nuy,
        const double* __restrict__ rho0, const double* __restrict__ rhoT, double r, double inv_r,
        double* __restrict__ F, int tch, int defer_lo, int defer_hi, double* __restrict__ wt_out,
        double* __restrict__ edge, int wt_pre, double (*fr)[PR_FN], double (*wb)[2][PR_PH * PR_PW], int ch, int x0,
        int y0, double& num_out, double& den_out, double& ff_out) {
    const int Nt = g.Nt, Nx = g.Nx, Ny = g.Ny, t0 = g.t0;
    const int64_t nxy = g.nxy;
    const int l0 = ch * tch, l1 = min(g.nloc, l0 + tch);   // own planes of this chunk (local)
    const int tid = threadIdx.x;
    // own voxels: stepB region positions (1 + tid % 64, 1 + tid / 64 + v PR_YV)
    const int opx = 1 + (tid & (PR_X - 1));
    const int ox = x0 - 1 + opx;
    int opy[PR_VPT], oy[PR_VPT], ooff[PR_VPT];
    bool own[PR_VPT];
#pragma unroll
    for (int v = 0; v < PR_VPT; ++v) {
        opy[v] = 1 + tid / PR_X + v * PR_YV;
        oy[v] = y0 - 1 + opy[v];
        own[v] = INTERIOR || (ox < Nx && oy[v] < Ny);
        ooff[v] = own[v] ? oy[v] * Nx + ox : 0;   // in-plane offsets fit 32 bits
    }
    // ring voxel of threads 0..PR_HALO-1
    int hpx = 0, hpy = 0;
    if (tid < PR_PW) { hpx = tid; hpy = 0; }
    else if (tid < 2 * PR_PW) { hpx = tid - PR_PW; hpy = PR_PH - 1; }
    else if (tid < 2 * PR_PW + PR_Y) { hpx = 0; hpy = 1 + tid - 2 * PR_PW; }
    else { hpx = PR_PW - 1; hpy = 1 + tid - 2 * PR_PW - PR_Y; }
    const int hx = x0 - 1 + hpx, hy = y0 - 1 + hpy;
    const bool hal = tid < PR_HALO && (INTERIOR || (hx >= 0 && hx < Nx && hy >= 0 && hy < Ny));
    const int hoff = hal ? hy * Nx + hx : 0;
    // phi region loads of this thread
    int foff[PR_FR];
    bool fin[PR_FR];
#pragma unroll
    for (int j = 0; j < PR_FR; ++j) {
        const int idx = tid + j * PR_NT;
        const int fy = idx / PR_FW, fx = idx - fy * PR_FW;
        const int xx = x0 - 2 + fx, yy = y0 - 2 + fy;
        fin[j] = idx < PR_FN && (INTERIOR || (xx >= 0 && xx < Nx && yy >= 0 && yy < Ny));
        foff[j] = fin[j] ? yy * Nx + xx : 0;
    }
    // stepB planes (local): one beyond the chunk on each side, within the grid and, where an edge
    // is deferred, within the shard
    if (!EDGE) defer_lo = defer_hi = 0;
    const int pa = max(l0 - 1, defer_lo ? 0 : -t0), pz = min(l1, defer_hi ? g.nloc - 1 : Nt - 1 - t0);
    const int nl = g.nloc;
    double fv[PR_FR];
    auto load_phi_to = [&](int p, double (&v)[PR_FR]) {   // planes beyond pz + 1 are never read
        const bool ok = t0 + p >= 0 && p <= pz + 1 && t0 + p < Nt;
#pragma unroll
        for (int j = 0; j < PR_FR; ++j)
#if FOTO_PR_NTPHI == 1
            v[j] = (ok && fin[j]) ? __builtin_nontemporal_load(&phi[p * nxy + foff[j]]) : 0.0;
#else
            v[j] = (ok && fin[j]) ? phi[p * nxy + foff[j]] : 0.0;
#endif
    };
    auto store_phi_from = [&](int p, const double (&v)[PR_FR]) {
#pragma unroll
        for (int j = 0; j < PR_FR; ++j)
            if (tid + j * PR_NT < PR_FN) fr[p & 3][tid + j * PR_NT] = v[j];
    };
    auto load_phi = [&](int p) { load_phi_to(p, fv); };
    auto store_phi = [&](int p) { store_phi_from(p, fv); };
    // mu of the own and the ring voxels, one plane ahead
    double om[PR_VPT][3], hm[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int v = 0; v < PR_VPT; ++v) om[v][0] = om[v][1] = om[v][2] = 0.0;
    auto load_mu = [&](int p) {
        if (p > pz) return;
#pragma unroll
        for (int v = 0; v < PR_VPT; ++v) {
#if FOTO_PR_NTLD
            if (own[v]) {   // (the old mu is dead after this kernel)
                om[v][0] = __builtin_nontemporal_load(&mut[p * nxy + ooff[v]]);
                om[v][1] = __builtin_nontemporal_load(&mux[p * nxy + ooff[v]]);
                om[v][2] = __builtin_nontemporal_load(&muy[p * nxy + ooff[v]]);
            }
#else
            if (own[v]) { om[v][0] = mut[p * nxy + ooff[v]]; om[v][1] = mux[p * nxy + ooff[v]]; om[v][2] = muy[p * nxy + ooff[v]]; }
#endif
        }
#if FOTO_PR_NTLD >= 2
        if (hal) {
            hm[0] = __builtin_nontemporal_load(&mut[p * nxy + hoff]);
            hm[1] = __builtin_nontemporal_load(&mux[p * nxy + hoff]);
            hm[2] = __builtin_nontemporal_load(&muy[p * nxy + hoff]);
        }
#else
        if (hal) { hm[0] = mut[p * nxy + hoff]; hm[1] = mux[p * nxy + hoff]; hm[2] = muy[p * nxy + hoff]; }
#endif
    };
    // stepB / stepC at stepB-region position (px, py) of local plane p (k_prox's body)
    auto stepb = [&](int p, int px, int py, int xg, int yg, const double (&m)[3], double (&w)[3], double& n0o,
                     double& ao, double& gto, double& gxo, double& gyo, double (&nu)[3]) {
        const int t = t0 + p;
        const int fi = (py + 1) * PR_FW + px + 1;
        const double* P = fr[p & 3];
        const double c = P[fi];
        const double tm = t > 0 ? fr[(p - 1) & 3][fi] : 0.0, tp = t < Nt - 1 ? fr[(p + 1) & 3][fi] : 0.0;
        const double gt = d1w(t, Nt, tm, c, tp);
        const double gx = d1w(xg, Nx, P[fi - 1], c, P[fi + 1]);
        const double gy = d1w(yg, Ny, P[fi - PR_FW], c, P[fi + PR_FW]);
        double a, b1, b2;
        project_K(gt + inv_r * m[0], gx + inv_r * m[1], gy + inv_r * m[2], a, b1, b2);
        double n0 = m[0] + r * (gt - a);
        n0 = (n0 < 0.0) ? 0.0 : n0;   // np.maximum(mu, 0) (NaN propagates)
        nu[0] = n0;
        nu[1] = m[1] + r * (gx - b1);
        nu[2] = m[2] + r * (gy - b2);
        w[0] = nu[0] - r * a;   // k_rhs: mu_t - r q_t, from the stored mu', q
        w[1] = nu[1] - r * b1;
        w[2] = nu[2] - r * b2;
        n0o = n0;
        ao = a;
        gto = gt;
        gxo = gx;
        gyo = gy;
    };
    double num = 0.0, den = 0.0, ff = 0.0;
    // own voxels: w_t of planes p-2, p-1, p; (mu'_t, q_t) of plane p-1 (bcm, bcq) and p (_n)
    double wtm[PR_VPT], wtc[PR_VPT], wtn[PR_VPT], bcm[PR_VPT], bcq[PR_VPT], bcm_n[PR_VPT], bcq_n[PR_VPT];
#pragma unroll
    for (int v = 0; v < PR_VPT; ++v) wtm[v] = wtc[v] = wtn[v] = bcm[v] = bcq[v] = bcm_n[v] = bcq_n[v] = 0.0;
    // plane p's stepB for the own and the ring voxels: mu' out (own planes only), w into
    // wb[p & 1], crit terms (own planes only)
    auto plane = [&](int p, const double (&mo)[PR_VPT][3], const double (&mh)[3]) {
        const bool mine = p >= l0 && p < l1;
#pragma unroll
        for (int v = 0; v < PR_VPT; ++v) {
            if (own[v]) {
                double w[3], nu[3], n0, a, gt, gx, gy;
                stepb(p, opx, opy[v], ox, oy[v], mo[v], w, n0, a, gt, gx, gy, nu);
                if (mine) {
                    const int64_t i = p * nxy + ooff[v];
#if FOTO_PR_NT
                    __builtin_nontemporal_store(nu[0], &nut[i]);
                    __builtin_nontemporal_store(nu[1], &nux[i]);
                    __builtin_nontemporal_store(nu[2], &nuy[i]);
#else
                    nut[i] = nu[0];
                    nux[i] = nu[1];
                    nuy[i] = nu[2];
#endif
                    const double gg = gx * gx + gy * gy;
                    num += n0 * fabs(gt + 0.5 * gg);
                    den += n0 * gg;
                }
                wb[p & 1][0][opy[v] * PR_PW + opx] = w[1];
                wb[p & 1][1][opy[v] * PR_PW + opx] = w[2];
                wtn[v] = w[0];
                bcm_n[v] = n0;
                bcq_n[v] = a;
            }
        }
        if (hal) {
            double w[3], nu[3], n0, a, gt, gx, gy;
            stepb(p, hpx, hpy, hx, hy, mh, w, n0, a, gt, gx, gy, nu);
            wb[p & 1][0][hpy * PR_PW + hpx] = w[1];
            wb[p & 1][1][hpy * PR_PW + hpx] = w[2];
        }
    };
    // prologue: phi planes pa-1 .. pa+1 in the ring, phi(pa+2) and mu(pa) in flight
    {   // every prologue load in flight before the first LDS store
        double f0[PR_FR], f1[PR_FR], f2[PR_FR];
        load_phi_to(pa - 1, f0);
        load_phi_to(pa, f1);
        load_phi_to(pa + 1, f2);
        load_phi(pa + 2);
        load_mu(pa);
        store_phi_from(pa - 1, f0);   // (pa = 0: plane -1 is never read)
        store_phi_from(pa, f1);
        store_phi_from(pa + 1, f2);
    }
    __syncthreads();
    for (int p = pa; p <= l1; ++p) {
        store_phi(p + 2);   // slot (p+2) & 3 = (p-2) & 3: last read by iteration p-1
        load_phi(p + 3);
        double cm[PR_VPT][3];
#pragma unroll
        for (int v = 0; v < PR_VPT; ++v) { cm[v][0] = om[v][0]; cm[v][1] = om[v][1]; cm[v][2] = om[v][2]; }
        const double chm[3] = {hm[0], hm[1], hm[2]};   // mu(p)
        load_mu(p + 1);
        if (p <= pz) plane(p, cm, chm);
        else {
#pragma unroll
            for (int v = 0; v < PR_VPT; ++v) wtn[v] = 0.0;   // t0 + p = Nt: F(Nt - 1) reads no w_t(Nt)
        }
        const int n = p - 1, tn = t0 + n;
        const bool deferred = (defer_lo && n == 0) || (defer_hi && n == nl - 1);   // k_rhs_edge's
#pragma unroll
        for (int v = 0; v < PR_VPT; ++v) {
            if (EDGE && own[v] && n >= l0) {
                // what k_rhs_edge needs next to a deferred edge, from the values F(n) would use: w_t
                // of the two outermost planes, and (w_x, w_y, mu'_t, q_t) of the edge plane itself
                // (wt_pre: k_wt_pre wrote the edge planes' w_t, which may be on the wire already)
                if (((defer_lo && n <= 1) || (defer_hi && n >= nl - 2)) && !(wt_pre && deferred))
                    wt_out[n * nxy + ooff[v]] = wtc[v];
                if (deferred) {   // slot 0: plane 0, slot 1: plane nloc - 1 (nloc = 1: both)
                    const int ci = opy[v] * PR_PW + opx;
                    double* E = edge + ooff[v] + ((defer_lo && n == 0) ? 0 : 4 * nxy);
                    E[0] = wb[n & 1][0][ci];
                    E[nxy] = wb[n & 1][1][ci];
                    E[2 * nxy] = bcm[v];
                    E[3 * nxy] = bcq[v];
                    if (defer_lo && defer_hi && nl == 1) {
                        E[4 * nxy] = E[0];
                        E[5 * nxy] = E[nxy];
                        E[6 * nxy] = bcm[v];
                        E[7 * nxy] = bcq[v];
                    }
                }
            }
            if (own[v] && n >= l0 && !deferred) {
                // F(n) (k_rhs's order: t, x, y terms, then the boundary-plane corrections)
                const double* WX = wb[n & 1][0];
                const double* WY = wb[n & 1][1];
                const int ci = opy[v] * PR_PW + opx;
                const int oo = ooff[v], yv = oy[v];
                double s = 0.0;
                acc_d1w(s, tn, Nt, wtm[v], wtc[v], wtn[v]);
                acc_d1w(s, ox, Nx, (INTERIOR || ox > 0) ? WX[ci - 1] : 0.0, WX[ci],
                        (INTERIOR || ox < Nx - 1) ? WX[ci + 1] : 0.0);
                acc_d1w(s, yv, Ny, (INTERIOR || yv > 0) ? WY[ci - PR_PW] : 0.0, WY[ci],
                        (INTERIOR || yv < Ny - 1) ? WY[ci + PR_PW] : 0.0);
                if (tn == 0) s -= (rho0[oo] - bcm[v]) + r * bcq[v];
                if (tn == Nt - 1) s += (rhoT[oo] - bcm[v]) + r * bcq[v];
#if FOTO_PR_NT >= 2
                __builtin_nontemporal_store(s, &F[n * nxy + oo]);
#else
                F[n * nxy + oo] = s;
#endif
                ff += s * s;
            }
            wtm[v] = wtc[v];
            wtc[v] = wtn[v];
            bcm[v] = bcm_n[v];
            bcq[v] = bcq_n[v];
        }
        __syncthreads();
    }
    num_out = num;
    den_out = den;
    ff_out = ff;
}

template <bool EDGE>
__global__ __launch_bounds__(PR_NT) __attribute__((amdgpu_waves_per_eu(PR_WPE))) void k_prox_rhs(
        Geo g, const double* __restrict__ phi, const double* __restrict__ mut, const double* __restrict__ mux,
        const double* __restrict__ muy, double* __restrict__ nut, double* __restrict__ nux, double* __restrict__ nuy,
        const double* __restrict__ rho0, const double* __restrict__ rhoT, double r, double inv_r,
        double* __restrict__ F, RedBuf rb, double* gath_crit, double* gath_rr, const int* __restrict__ guard, int tch,
        int defer_lo, int defer_hi, double* __restrict__ wt_out, double* __restrict__ edge, double* hcrit,
        int wt_pre) {
    if (guard && *guard == 0) return;
    __shared__ double fr[4][PR_FN];                  // phi ring (plane p in slot p & 3)
    __shared__ double wb[2][2][PR_PH * PR_PW];       // [plane & 1][x | y part] of w
    const int Nx = g.Nx, Ny = g.Ny;
    const int ntx = (Nx + PR_X - 1) / PR_X, ntiles = ntx * ((Ny + PR_Y - 1) / PR_Y);
    const int lin = xcd_tile(blockIdx.x);
#if FOTO_PR_CHFAST
    // a tile's chunks adjacent in the block order (one XCD, resident together)
    const int nch = (g.nloc + tch - 1) / tch;
    const int tile = lin / nch, ch = lin - tile * nch;
#else
    const int ch = lin / ntiles, tile = lin - ch * ntiles;
#endif
    const int x0 = (tile % ntx) * PR_X, y0 = (tile / ntx) * PR_Y;
    double num, den, ff;
#if FOTO_PR_INTERIOR
    if (x0 >= 2 && x0 + PR_X + 2 <= Nx && y0 >= 2 && y0 + PR_Y + 2 <= Ny)
        prox_rhs_body<EDGE, true>(g, phi, mut, mux, muy, nut, nux, nuy, rho0, rhoT, r, inv_r, F, tch, defer_lo,
                                  defer_hi, wt_out, edge, wt_pre, fr, wb, ch, x0, y0, num, den, ff);
    else
#endif
        prox_rhs_body<EDGE, false>(g, phi, mut, mux, muy, nut, nux, nuy, rho0, rhoT, r, inv_r, F, tch, defer_lo,
                                   defer_hi, wt_out, edge, wt_pre, fr, wb, ch, x0, y0, num, den, ff);
    double v[3] = {num, den, ff}, tot[3];
    if (grid_reduce_last<3, PR_NT>(v, rb, tot) && threadIdx.x == 0) {   // (this rank's slots)
        gath_crit[0] = tot[0];
        gath_crit[1] = tot[1];
        if (gath_rr) gath_rr[0] = tot[2];
        if (hcrit) {   // (pinned, coherent host slot: the crit readback without a copy launch)
            hcrit[0] = tot[0];
            hcrit[1] = tot[1];
            __threadfence_system();
        }
    }
}

// planes per chunk (FOTO_PR_TCH, read per call for A/B tests).  Measured at 640x480x32
// (MI355X, 2 blocks of 512 threads per CU): 4 / 8 / 16 / 32 planes -> 232 / 195 / 173 / 193 us
// (more chunks: more recomputed boundary planes; fewer: a partly filled last round of blocks).
int prox_rhs_tch(const Geo& g) {
    const char* e = getenv("FOTO_PR_TCH");
    const int v = e ? atoi(e) : 16;
    return std::min(v > 0 ? v : 16, g.nloc);
}

int prox_rhs_blocks(const Geo& g) {
    const int tch = prox_rhs_tch(g);
    return ((g.Nx + PR_X - 1) / PR_X) * ((g.Ny + PR_Y - 1) / PR_Y) * ((g.nloc + tch - 1) / tch);
}

hipError_t launch_prox_rhs(const Geo& g, const double* phi, const double* mut, const double* mux, const double* muy,
                           double* nut, double* nux, double* nuy, const double* rho0, const double* rhoT, double r,
                           double* F, RedBuf rb, double* gath_crit, double* gath_rr, hipStream_t s, const int* guard,
                           int defer_lo, int defer_hi, double* wt_out, double* edge, double* hcrit, int wt_pre) {
    const int nb = prox_rhs_blocks(g);
    if (rb.cap < 3 * nb) return hipErrorInvalidValue;
    if ((defer_lo || defer_hi) && (!wt_out || !edge)) return hipErrorInvalidValue;
    if (defer_lo || defer_hi)
        k_prox_rhs<true><<<nb, PR_NT, 0, s>>>(g, phi, mut, mux, muy, nut, nux, nuy, rho0, rhoT, r, 1.0 / r, F, rb,
                                              gath_crit, gath_rr, guard, prox_rhs_tch(g), defer_lo, defer_hi, wt_out, edge,
                                              hcrit, wt_pre);
    else
        k_prox_rhs<false><<<nb, PR_NT, 0, s>>>(g, phi, mut, mux, muy, nut, nux, nuy, rho0, rhoT, r, 1.0 / r, F, rb,
                                               gath_crit, gath_rr, guard, prox_rhs_tch(g), 0, 0, nullptr, nullptr,
                                               hcrit, 0);
    return hipGetLastError();
}

// (round 5) w_t of a shard's deferred edge planes before k_prox_rhs: per voxel k_prox's stepB
// (the fused kernel's stepb, same operations in the same order, out-of-grid neighbours 0.0 as
// its LDS image holds them), so the w_t plane each neighbour needs can be on the wire while
// k_prox_rhs runs (foto_bb.cpp prox_rhs / wt_overlap).  blockIdx.y: plane pa, then pb.
__global__ __launch_bounds__(NT) void k_wt_pre(Geo g, int pa, int pb, const double* __restrict__ phi,
                                               const double* __restrict__ mut, const double* __restrict__ mux,
                                               const double* __restrict__ muy, double r, double inv_r,
                                               double* __restrict__ wt, const int* __restrict__ guard) {
    if (guard && *guard == 0) return;
    const int64_t nxy = g.nxy;
    const int64_t off = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (off >= nxy) return;
    const int p = blockIdx.y == 0 ? pa : pb;
    const int y = (int)(off / g.Nx), x = (int)(off - (int64_t)y * g.Nx), t = g.t0 + p;
    const int64_t i = (int64_t)p * nxy + off;
    const double c = phi[i];
    const double tm = t > 0 ? phi[i - nxy] : 0.0, tp = t < g.Nt - 1 ? phi[i + nxy] : 0.0;
    const double gt = d1w(t, g.Nt, tm, c, tp);
    const double gx = d1w(x, g.Nx, x > 0 ? phi[i - 1] : 0.0, c, x < g.Nx - 1 ? phi[i + 1] : 0.0);
    const double gy = d1w(y, g.Ny, y > 0 ? phi[i - g.Nx] : 0.0, c, y < g.Ny - 1 ? phi[i + g.Nx] : 0.0);
    const double m0 = mut[i], m1 = mux[i], m2 = muy[i];
    double a, b1, b2;
    project_K(gt + inv_r * m0, gx + inv_r * m1, gy + inv_r * m2, a, b1, b2);
    double n0 = m0 + r * (gt - a);
    n0 = (n0 < 0.0) ? 0.0 : n0;
    wt[i] = n0 - r * a;
}

hipError_t launch_wt_pre(const Geo& g, const double* phi, const double* mut, const double* mux, const double* muy,
                         double r, double* wt, int defer_lo, int defer_hi, hipStream_t s, const int* guard) {
    if (!defer_lo && !defer_hi) return hipSuccess;
    const int pa = defer_lo ? 0 : g.nloc - 1, pb = g.nloc - 1;
    const int np = (defer_lo && defer_hi && g.nloc > 1) ? 2 : 1;
    k_wt_pre<<<dim3((unsigned)flat_blocks(g.nxy), np), NT, 0, s>>>(g, pa, pb, phi, mut, mux, muy, r, 1.0 / r, wt,
                                                                  guard);
    return hipGetLastError();
}

// F on a deferred edge plane of a shard (local plane n = 0 or nloc - 1) from what k_prox_rhs
// stored there and the neighbour's w_t plane (exchanged into wt's halo): k_prox_rhs's F code
// -- t, x, y terms, then the boundary corrections, in the same order -- so F is bit-identical
// to the single-shard kernel's.  F.F of the plane is added to gath_rr[0] (stencil CG).
__global__ __launch_bounds__(NT) void k_rhs_edge(Geo g, int n, const double* __restrict__ wt,
                                                 const double* __restrict__ E, const double* __restrict__ rho0,
                                                 const double* __restrict__ rhoT, double r, double* __restrict__ F,
                                                 RedBuf rb, double* gath_rr, const int* __restrict__ guard) {
    if (guard && *guard == 0) return;
    const int64_t nxy = g.nxy;
    const int64_t off = (int64_t)blockIdx.x * NT + threadIdx.x;
    double ff = 0.0;
    if (off < nxy) {
        const int y = (int)(off / g.Nx), x = (int)(off - (int64_t)y * g.Nx), tn = g.t0 + n;
        const double* WX = E;
        const double* WY = E + nxy;
        const int64_t i = (int64_t)n * nxy + off;
        double s = 0.0;
        acc_d1w(s, tn, g.Nt, wt[i - nxy], wt[i], wt[i + nxy]);
        acc_d1w(s, x, g.Nx, x > 0 ? WX[off - 1] : 0.0, WX[off], x < g.Nx - 1 ? WX[off + 1] : 0.0);
        acc_d1w(s, y, g.Ny, y > 0 ? WY[off - g.Nx] : 0.0, WY[off], y < g.Ny - 1 ? WY[off + g.Nx] : 0.0);
        const double bcm = E[2 * nxy + off], bcq = E[3 * nxy + off];
        if (tn == 0) s -= (rho0[off] - bcm) + r * bcq;
        if (tn == g.Nt - 1) s += (rhoT[off] - bcm) + r * bcq;
        F[i] = s;
        ff = s * s;
    }
    if (!gath_rr) return;
    double v[1] = {ff}, tot[1];
    if (grid_reduce_last<1>(v, rb, tot) && threadIdx.x == 0) gath_rr[0] += tot[0];
}

hipError_t launch_rhs_edge(const Geo& g, int n, const double* wt, const double* edge, const double* rho0,
                           const double* rhoT, double r, double* F, RedBuf rb, double* gath_rr, hipStream_t s,
                           const int* guard) {
    if (n < 0 || n >= g.nloc) return hipErrorInvalidValue;
    k_rhs_edge<<<flat_blocks(g.nxy), NT, 0, s>>>(g, n, wt, edge, rho0, rhoT, r, F, rb, gath_rr, guard);
    return hipGetLastError();
}

// ============================================================================ 2-D operators

// grad_1d_central (operators.py:52-65): bc 'N' end rows zero; bc 'D' zero extension.
__device__ __forceinline__ double d1c(int k, int n, double m, double p, int bcD) {
    if (k == 0) return bcD ? 0.5 * p : 0.0;
    if (k == n - 1) return bcD ? -0.5 * m : 0.0;
    return 0.5 * (p - m);
}

__global__ __launch_bounds__(NT) void k_grad2(int Nx, int Ny, const double* __restrict__ f, double* __restrict__ gx,
                                              double* __restrict__ gy, int bcD) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= (int64_t)Nx * Ny) return;
    const int y = (int)(i / Nx), x = (int)(i - (int64_t)y * Nx);
    gx[i] = d1c(x, Nx, x > 0 ? f[i - 1] : 0.0, x < Nx - 1 ? f[i + 1] : 0.0, bcD);
    gy[i] = d1c(y, Ny, y > 0 ? f[i - Nx] : 0.0, y < Ny - 1 ? f[i + Nx] : 0.0, bcD);
}

hipError_t launch_grad2(int Nx, int Ny, const double* f, double* gx, double* gy, int bcD, hipStream_t s) {
    k_grad2<<<flat_blocks((int64_t)Nx * Ny), NT, 0, s>>>(Nx, Ny, f, gx, gy, bcD);
    return hipGetLastError();
}

// operators.div (operators.py:182-191) row, COO order: x-block terms then y-block terms.
__device__ __forceinline__ void acc_d1c(double& s, int k, int n, double m, double p, int bcD) {
    if (k == 0) { if (bcD) s += 0.5 * p; }
    else if (k == n - 1) { if (bcD) s += -0.5 * m; }
    else { s += -0.5 * m; s += 0.5 * p; }
}

__global__ __launch_bounds__(NT) void k_div2(int Nx, int Ny, const double* __restrict__ u, const double* __restrict__ v,
                                             double* __restrict__ out, int bcD, double sign) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= (int64_t)Nx * Ny) return;
    const int y = (int)(i / Nx), x = (int)(i - (int64_t)y * Nx);
    double s = 0.0;
    acc_d1c(s, x, Nx, x > 0 ? u[i - 1] : 0.0, x < Nx - 1 ? u[i + 1] : 0.0, bcD);
    acc_d1c(s, y, Ny, y > 0 ? v[i - Nx] : 0.0, y < Ny - 1 ? v[i + Nx] : 0.0, bcD);
    out[i] = sign * s;
}

hipError_t launch_div2(int Nx, int Ny, const double* u, const double* v, double* out, int bcD, double sign,
                       hipStream_t s) {
    k_div2<<<flat_blocks((int64_t)Nx * Ny), NT, 0, s>>>(Nx, Ny, u, v, out, bcD, sign);
    return hipGetLastError();
}

// grad_forward bc 'N' (operators.py:67-79, 171-180): z[k+1] - z[k], last row 0.
__global__ __launch_bounds__(NT) void k_grad2_fwd(int Nx, int Ny, const double* __restrict__ f,
                                                  double* __restrict__ gx, double* __restrict__ gy) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= (int64_t)Nx * Ny) return;
    const int y = (int)(i / Nx), x = (int)(i - (int64_t)y * Nx);
    gx[i] = (x < Nx - 1) ? -1.0 * f[i] + 1.0 * f[i + 1] : 0.0;
    gy[i] = (y < Ny - 1) ? -1.0 * f[i] + 1.0 * f[i + Nx] : 0.0;
}

hipError_t launch_grad2_forward(int Nx, int Ny, const double* f, double* gx, double* gy, hipStream_t s) {
    k_grad2_fwd<<<flat_blocks((int64_t)Nx * Ny), NT, 0, s>>>(Nx, Ny, f, gx, gy);
    return hipGetLastError();
}

// ============================================================================ flow extraction (A13/A14)

// un[n] = G_x phi_n, vn[n] = G_y phi_n (bc 'N': zero on the edge columns / rows).
__device__ __forceinline__ double un_at(const double* P, int Nx, int yy, int xx) {
    if (xx == 0 || xx == Nx - 1) return 0.0;
    return 0.5 * (P[(int64_t)yy * Nx + xx + 1] - P[(int64_t)yy * Nx + xx - 1]);
}
__device__ __forceinline__ double vn_at(const double* P, int Nx, int Ny, int yy, int xx) {
    if (yy == 0 || yy == Ny - 1) return 0.0;
    return 0.5 * (P[(int64_t)(yy + 1) * Nx + xx] - P[(int64_t)(yy - 1) * Nx + xx]);
}

__device__ __forceinline__ int trunc_clamp(double v, int hi) {
    double t = trunc(v);               // int() truncates toward zero
    if (!(t >= 0.0)) t = 0.0;          // also maps NaN to 0
    if (t > (double)hi) t = (double)hi;
    return (int)t;
}

// reconstructTrajectory (utils.py:44-99) for steps n in [n_lo, n_hi), one thread per pixel.
__global__ __launch_bounds__(NT) void k_traj(Geo g, const double* __restrict__ phi, int n_lo, int n_hi,
                                             double* __restrict__ px, double* __restrict__ py, int init) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= g.nxy) return;
    const int Nx = g.Nx, Ny = g.Ny;
    const int j = (int)(i / Nx), ii = (int)(i - (int64_t)j * Nx);
    double x = init ? (double)ii : px[i];
    double y = init ? (double)j : py[i];
    for (int n = n_lo; n < n_hi; ++n) {
        const double* P = phi + (int64_t)(n - g.t0) * g.nxy;
        const int tx = trunc_clamp(x, Nx - 2), ty = trunc_clamp(y, Ny - 2);
        const double dX = x - tx, dY = y - ty;
        const double w1 = (1 - dY) * (1 - dX), w2 = dX * (1 - dY), w3 = dY * dX, w4 = (1 - dX) * dY;
        const double u00 = un_at(P, Nx, ty, tx), u01 = un_at(P, Nx, ty, tx + 1);
        const double u11 = un_at(P, Nx, ty + 1, tx + 1), u10 = un_at(P, Nx, ty + 1, tx);
        const double v00 = vn_at(P, Nx, Ny, ty, tx), v01 = vn_at(P, Nx, Ny, ty, tx + 1);
        const double v11 = vn_at(P, Nx, Ny, ty + 1, tx + 1), v10 = vn_at(P, Nx, Ny, ty + 1, tx);
        x += w1 * u00 + w2 * u01 + w3 * u11 + w4 * u10;
        y += w1 * v00 + w2 * v01 + w3 * v11 + w4 * v10;
    }
    px[i] = x;
    py[i] = y;
}

hipError_t launch_traj(const Geo& g, const double* phi, int n_lo, int n_hi, double* px, double* py, int init,
                       hipStream_t s) {
    k_traj<<<flat_blocks(g.nxy), NT, 0, s>>>(g, phi, n_lo, n_hi, px, py, init);
    return hipGetLastError();
}

__global__ __launch_bounds__(NT) void k_flow_uv(int Nx, int Ny, const double* __restrict__ px,
                                                const double* __restrict__ py, double* __restrict__ u,
                                                double* __restrict__ v) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= (int64_t)Nx * Ny) return;
    const int j = (int)(i / Nx), ii = (int)(i - (int64_t)j * Nx);
    u[i] = px[i] - (double)ii;
    v[i] = py[i] - (double)j;
}

hipError_t launch_flow_finish(int Nx, int Ny, const double* px, const double* py, double* u, double* v, double* m,
                              hipStream_t s) {
    k_flow_uv<<<flat_blocks((int64_t)Nx * Ny), NT, 0, s>>>(Nx, Ny, px, py, u, v);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_div2(Nx, Ny, u, v, m, 1, -1.0, s);   // m = -div(bc 'D') [u; v]
}

}  // namespace foto

namespace foto {

// x.x partial sums -> gath[rank] (used to seed CG with b.b when b comes from the host)
__global__ __launch_bounds__(NT) void k_dot_self(int64_t n, const double* __restrict__ x, RedBuf rb, double* gath,
                                                 int rank) {
    double acc = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) acc += x[i] * x[i];
    double v[1] = {acc}, tot[1];
    if (grid_reduce_last<1>(v, rb, tot) && threadIdx.x == 0) gath[rank] = tot[0];
}

hipError_t launch_dot_self(int64_t n, const double* x, RedBuf rb, double* gath, int rank, hipStream_t s) {
    int nb = (int)std::min<int64_t>((n + NT - 1) / NT, 2048);
    k_dot_self<<<nb, NT, 0, s>>>(n, x, rb, gath, rank);
    return hipGetLastError();
}

}  // namespace foto
