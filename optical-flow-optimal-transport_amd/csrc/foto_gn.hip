// libfoto: Gennert-Negahdaripour variational baseline (classical.GLLOpticalFlow,
// classical.py:25-130) on gfx950.
//
// The reference assembles a 3wh x 3wh sparse SPD system
//   [[-a L + fx^2, fx fy, -fx f2], [fy fx, -a L + fy^2, -fy f2], [-f2 fx, -f2 fy, -l L + f2^2]]
// (L = 5-point Neumann Laplacian = -G^T G with G = grad_forward) and solves it with SuperLU.
// Here the operator is applied matrix-free (one thread per pixel, all three fields) and
// solved with CG preconditioned by one symmetric multigrid V-cycle (damped block-Jacobi
// smoothing with the per-pixel 3x3 block D + v v^T, v = (fx, fy, -f2); FOTO_GN_MG=0 keeps
// plain block-Jacobi PCG), driven on the device with the same last-block reductions as
// the BB CG and replayed as a hipGraph.
#include <chrono>

#include "foto_internal.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace foto {

// reductions shared with foto_kernels.hip (re-declared here: header-only templates)
__device__ __forceinline__ double gn_wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

template <int K>
__device__ __forceinline__ void gn_block_sum(double (&v)[K], double* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v[k] = gn_wave_sum(v[k]);
        if (lane == 0) sh[k * (NT / 64) + w] = v[k];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            double s = sh[k * (NT / 64)];
#pragma unroll
            for (int j = 1; j < NT / 64; ++j) s += sh[k * (NT / 64) + j];
            v[k] = s;
        }
    }
}

template <int K>
__device__ bool gn_reduce_last(double (&v)[K], RedBuf rb, double (&tot)[K]) {
    __shared__ double sh[K * (NT / 64)];
    __shared__ int is_last;
    gn_block_sum<K>(v, sh);
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
    for (int i = threadIdx.x; i < nb; i += NT) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            acc[k] += __hip_atomic_load(&rb.partials[(int64_t)k * nb + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    gn_block_sum<K>(acc, sh);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) tot[k] = acc[k];
        __hip_atomic_store(rb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// PCG kernels run a grid-stride loop over pixels on at most two blocks per CU: each block
// adds one agent-scope ticket per launch, and 1200 tickets on one address (one block per
// 256 pixels at 640x480) serialised at the memory side (~28 us per kernel, rocprofv3); with
// 512 blocks and a 512-entry gather the kernels are bandwidth-bound.
static int gn_grid(int64_t n) {
    static int cap = 0;
    if (cap == 0) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            cus = 256;
        cap = 2 * cus;
    }
    return (int)std::min<int64_t>(flat_blocks(n), cap);
}

// ----------------------------------------------------------------------------- coefficients

// classical.py:90-100
__global__ __launch_bounds__(NT) void k_gn_coeffs(int w, int h, const double* __restrict__ f1,
                                                  const double* __restrict__ f2, double* __restrict__ fx,
                                                  double* __restrict__ fy, double* __restrict__ ft) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= (int64_t)w * h) return;
    const int y = (int)(i / w), x = (int)(i - (int64_t)y * w);
    fx[i] = (x >= 1 && x <= w - 2) ? 0.5 * (f2[i + 1] - f2[i - 1]) : 0.0;
    fy[i] = (y >= 1 && y <= h - 2) ? 0.5 * (f2[i + w] - f2[i - w]) : 0.0;
    ft[i] = f2[i] - f1[i];
}

hipError_t launch_gn_coeffs(int w, int h, const double* f1, const double* f2, double* fx, double* fy, double* ft,
                            hipStream_t s) {
    k_gn_coeffs<<<flat_blocks((int64_t)w * h), NT, 0, s>>>(w, h, f1, f2, fx, fy, ft);
    return hipGetLastError();
}

// b = [-fx ft; -fy ft; f2 ft] (classical.py:110)
__global__ __launch_bounds__(NT) void k_gn_rhs(int64_t n, const double* __restrict__ fx, const double* __restrict__ fy,
                                               const double* __restrict__ f2, const double* __restrict__ ft,
                                               double* __restrict__ b) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    b[i] = -fx[i] * ft[i];
    b[n + i] = -fy[i] * ft[i];
    b[2 * n + i] = f2[i] * ft[i];
}

hipError_t launch_gn_rhs(int w, int h, const double* fx, const double* fy, const double* f2, const double* ft,
                         double* b, hipStream_t s) {
    const int64_t n = (int64_t)w * h;
    k_gn_rhs<<<flat_blocks(n), NT, 0, s>>>(n, fx, fy, f2, ft, b);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------- operator

struct GNPix {
    int x, y;
    bool hy, hx, hX, hY;
    double c;   // neighbour count = diagonal of G^T G
};

__device__ __forceinline__ GNPix gn_pix(int w, int h, int64_t i) {
    GNPix P;
    // 32-bit division (w h < 2^31): the 64-bit one is a long software sequence per pixel
    P.y = (int)((unsigned)i / (unsigned)w);
    P.x = (int)i - P.y * w;
    P.hy = P.y > 0; P.hY = P.y < h - 1; P.hx = P.x > 0; P.hX = P.x < w - 1;
    P.c = (double)((int)P.hy + (int)P.hY + (int)P.hx + (int)P.hX);
    return P;
}

// one field's Laplacian block row in CSR order: (y-1), (x-1), diag, (x+1), (y+1)
// The five values are fetched unconditionally (clamped indices) and the missing neighbours
// skipped by selects: with the fetches behind branches every neighbour was its own memory
// round trip (~25 us per PCG kernel at 640x480).  Same additions in the same order.
template <class F>
__device__ __forceinline__ double gn_lap_row(const GNPix& P, int w, int64_t i, double coef, double dg, F val,
                                             double s) {
    const double m = -coef;
    const double vym = val(P.hy ? i - w : i), vxm = val(P.hx ? i - 1 : i), vc = val(i);
    const double vxp = val(P.hX ? i + 1 : i), vyp = val(P.hY ? i + w : i);
    s = P.hy ? s + m * vym : s;
    s = P.hx ? s + m * vxm : s;
    s += dg * vc;
    s = P.hX ? s + m * vxp : s;
    s = P.hY ? s + m * vyp : s;
    return s;
}

// (A z)_i for all three fields; F(field, index) -> value of the vector being multiplied.
template <class F>
__device__ __forceinline__ void gn_row(const GNPix& P, int w, int64_t n, int64_t i, double fx, double fy, double f2,
                                       double a, double l, F val, double& yu, double& yv, double& ym) {
    auto U = [&](int64_t j) { return val(0, j); };
    auto V = [&](int64_t j) { return val(1, j); };
    auto Mm = [&](int64_t j) { return val(2, j); };
    const double ui = val(0, i), vi = val(1, i), mi = val(2, i);
    double s = gn_lap_row(P, w, i, a, a * P.c + fx * fx, U, 0.0);
    s += (fx * fy) * vi;
    s += (-fx * f2) * mi;
    yu = s;
    s = 0.0;
    s += (fy * fx) * ui;   // CSR order: the u column precedes the v block
    s = gn_lap_row(P, w, i, a, a * P.c + fy * fy, V, s);
    s += (-fy * f2) * mi;
    yv = s;
    s = 0.0;
    s += (-f2 * fx) * ui;
    s += (-f2 * fy) * vi;
    s = gn_lap_row(P, w, i, l, l * P.c + f2 * f2, Mm, s);
    ym = s;
    (void)n;
}

// gn_row with the five stencil values of each field already fetched: V(f, k), k in CSR order
// (y-1, x-1, centre, x+1, y+1; missing neighbours fetched at the centre's index, as gn_lap_row
// does) -- the same additions in the same order
template <class F>
__device__ __forceinline__ double gn_lap_row_v(const GNPix& P, double coef, double dg, F val, double s) {
    const double m = -coef;
    s = P.hy ? s + m * val(0) : s;
    s = P.hx ? s + m * val(1) : s;
    s += dg * val(2);
    s = P.hX ? s + m * val(3) : s;
    s = P.hY ? s + m * val(4) : s;
    return s;
}

template <class F>
__device__ __forceinline__ void gn_row_v(const GNPix& P, double fx, double fy, double f2, double a, double l, F val,
                                         double& yu, double& yv, double& ym) {
    const double ui = val(0, 2), vi = val(1, 2), mi = val(2, 2);
    double s = gn_lap_row_v(P, a, a * P.c + fx * fx, [&](int k) { return val(0, k); }, 0.0);
    s += (fx * fy) * vi;
    s += (-fx * f2) * mi;
    yu = s;
    s = 0.0;
    s += (fy * fx) * ui;
    s = gn_lap_row_v(P, a, a * P.c + fy * fy, [&](int k) { return val(1, k); }, s);
    s += (-fy * f2) * mi;
    yv = s;
    s = 0.0;
    s += (-f2 * fx) * ui;
    s += (-f2 * fy) * vi;
    s = gn_lap_row_v(P, l, l * P.c + f2 * f2, [&](int k) { return val(2, k); }, s);
    ym = s;
}

__global__ __launch_bounds__(NT) void k_gn_apply(int w, int h, const double* __restrict__ fx,
                                                 const double* __restrict__ fy, const double* __restrict__ f2,
                                                 double a, double l, const double* __restrict__ x,
                                                 double* __restrict__ y) {
    const int64_t n = (int64_t)w * h;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const GNPix P = gn_pix(w, h, i);
    double yu, yv, ym;
    gn_row(P, w, n, i, fx[i], fy[i], f2[i], a, l, [&](int f, int64_t j) { return x[f * n + j]; }, yu, yv, ym);
    y[i] = yu;
    y[n + i] = yv;
    y[2 * n + i] = ym;
}

hipError_t launch_gn_apply(int w, int h, const double* fx, const double* fy, const double* f2, double alpha,
                           double lam, const double* x, double* y, hipStream_t s) {
    k_gn_apply<<<flat_blocks((int64_t)w * h), NT, 0, s>>>(w, h, fx, fy, f2, alpha, lam, x, y);
    return hipGetLastError();
}

// ----------------------------------------------------------------------------- preconditioner

// z = (D + v v^T)^{-1} r with D = diag(a c, a c, l c), v = (fx, fy, -f2) (Sherman-Morrison)
__device__ __forceinline__ void gn_precond(double c, double fx, double fy, double f2, double a, double l, double ru,
                                           double rv, double rm, double& zu, double& zv, double& zm) {
    const double du = 1.0 / (a * c), dm = 1.0 / (l * c);
    const double wu = fx * du, wv = fy * du, wm = -f2 * dm;            // D^-1 v
    const double den = 1.0 + fx * wu + fy * wv + (-f2) * wm;          // 1 + v^T D^-1 v
    const double yu = ru * du, yv = rv * du, ym = rm * dm;            // D^-1 r
    const double t = (fx * yu + fy * yv + (-f2) * ym) / den;          // v^T D^-1 r / den
    zu = yu - wu * t;
    zv = yv - wv * t;
    zm = ym - wm * t;
}

// r = b, z = M r, partials (r.r, r.z) -> gath[0], gath[1]
__global__ __launch_bounds__(NT) void k_gn_pcg_init(int w, int h, const double* __restrict__ fx,
                                                    const double* __restrict__ fy, const double* __restrict__ f2,
                                                    double a, double l, const double* __restrict__ b,
                                                    double* __restrict__ r, double* __restrict__ z, RedBuf rb,
                                                    double* gath) {
    const int64_t n = (int64_t)w * h;
    double rr = 0.0, rz = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const GNPix P = gn_pix(w, h, i);
        const double ru = b[i], rv = b[n + i], rm = b[2 * n + i];
        r[i] = ru; r[n + i] = rv; r[2 * n + i] = rm;
        double zu, zv, zm;
        gn_precond(P.c, fx[i], fy[i], f2[i], a, l, ru, rv, rm, zu, zv, zm);
        z[i] = zu; z[n + i] = zv; z[2 * n + i] = zm;
        rr += ru * ru + rv * rv + rm * rm;
        rz += ru * zu + rv * zv + rm * zm;
    }
    double v[2] = {rr, rz}, tot[2];
    if (gn_reduce_last<2>(v, rb, tot) && threadIdx.x == 0) { gath[0] = tot[0]; gath[1] = tot[1]; }
}

hipError_t launch_gn_pcg_init(int w, int h, const double* fx, const double* fy, const double* f2, double alpha,
                              double lam, const double* b, double* r, double* z, RedBuf rb, double* gath,
                              hipStream_t s) {
    k_gn_pcg_init<<<gn_grid((int64_t)w * h), NT, 0, s>>>(w, h, fx, fy, f2, alpha, lam, b, r, z, rb, gath);
    return hipGetLastError();
}

// Iteration k, first half: stop test on ||r||, beta = rz / rz_prev, p = z + beta p (computed
// for the pixel and its 4 neighbours), q = A p, partial p.q; writes p.
// gath_rz = {r.r, r.z} of r_k; gath_pq = {p.q}.
__global__ __launch_bounds__(NT) void k_gn_pcg_dir(int w, int h, int k_arg, const double* __restrict__ fx,
                                                   const double* __restrict__ fy, const double* __restrict__ f2,
                                                   double a, double l, const double* __restrict__ z,
                                                   const double* __restrict__ po, double* __restrict__ pn, CGScal* S,
                                                   RedBuf rb, const double* __restrict__ gath_rz,
                                                   double* __restrict__ gath_pq, double rtol) {
    if (S->done) return;
    const int k = k_arg >= 0 ? k_arg : S->pad[0];   // k < 0: iteration index kept on the device (MG path)
    const double rr = gath_rz[0], rz = gath_rz[1];
    const double atol = (k == 0) ? fmax(0.0, rtol * sqrt(rr)) : S->atol;
    if (rr == 0.0 || sqrt(rr) < atol) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { S->done = 1; S->iters = k; }
        return;
    }
    const double beta = (k > 0) ? rz / S->rho : 0.0;
    const int64_t n = (int64_t)w * h;
    double pq = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const GNPix P = gn_pix(w, h, i);
        auto pv = [&](int f, int64_t j) -> double {
            const int64_t o = f * n + j;
            return (k == 0) ? z[o] : beta * po[o] + z[o];
        };
        double qu, qv, qm;
        gn_row(P, w, n, i, fx[i], fy[i], f2[i], a, l, pv, qu, qv, qm);
        const double pu = pv(0, i), pvv = pv(1, i), pm = pv(2, i);
        pn[i] = pu; pn[n + i] = pvv; pn[2 * n + i] = pm;
        pq += pu * qu + pvv * qv + pm * qm;
    }
    double v[1] = {pq}, tot[1];
    if (gn_reduce_last<1>(v, rb, tot) && threadIdx.x == 0) {
        S->rho = rz;
        if (k == 0) { S->bb = rr; S->atol = atol; }
        gath_pq[0] = tot[0];
    }
}

hipError_t launch_gn_pcg_dir(int w, int h, int k, const double* fx, const double* fy, const double* f2, double alpha,
                             double lam, const double* z, const double* pold, double* pnew, CGScal* S, RedBuf rb,
                             const double* gath_rz, double* gath_pq, double rtol, hipStream_t s) {
    k_gn_pcg_dir<<<gn_grid((int64_t)w * h), NT, 0, s>>>(w, h, k, fx, fy, f2, alpha, lam, z, pold, pnew, S, rb,
                                                            gath_rz, gath_pq, rtol);
    return hipGetLastError();
}

// second half: alpha = rz / p.q; x += alpha p; r -= alpha A p; z = M r; partials (r.r, r.z)
__global__ __launch_bounds__(NT) void k_gn_pcg_upd(int w, int h, int k, const double* __restrict__ fx,
                                                   const double* __restrict__ fy, const double* __restrict__ f2,
                                                   double a, double l, const double* __restrict__ p,
                                                   double* __restrict__ x, double* __restrict__ r,
                                                   double* __restrict__ z, CGScal* S, RedBuf rb,
                                                   const double* __restrict__ gath_pq, double* __restrict__ gath_rz) {
    if (S->done) return;
    const double alpha = S->rho / gath_pq[0];
    const int64_t n = (int64_t)w * h;
    double rr = 0.0, rz = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * NT) {
        const GNPix P = gn_pix(w, h, i);
        const double cfx = fx[i], cfy = fy[i], cf2 = f2[i];
        double qu, qv, qm;
        gn_row(P, w, n, i, cfx, cfy, cf2, a, l, [&](int f, int64_t j) { return p[f * n + j]; }, qu, qv, qm);
        const double q3[3] = {qu, qv, qm};
        double rn[3];
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const int64_t o = f * n + i;
            const double ap = alpha * p[o];
            x[o] = (k == 0) ? 0.0 + ap : x[o] + ap;
            rn[f] = r[o] - alpha * q3[f];
            r[o] = rn[f];
        }
        double zu, zv, zm;
        gn_precond(P.c, cfx, cfy, cf2, a, l, rn[0], rn[1], rn[2], zu, zv, zm);
        z[i] = zu; z[n + i] = zv; z[2 * n + i] = zm;
        rr += rn[0] * rn[0] + rn[1] * rn[1] + rn[2] * rn[2];
        rz += rn[0] * zu + rn[1] * zv + rn[2] * zm;
    }
    double v[2] = {rr, rz}, tot[2];
    if (gn_reduce_last<2>(v, rb, tot) && threadIdx.x == 0) {
        gath_rz[0] = tot[0];
        gath_rz[1] = tot[1];
    }
}

hipError_t launch_gn_pcg_upd(int w, int h, int k, const double* fx, const double* fy, const double* f2, double alpha,
                             double lam, const double* p, double* x, double* r, double* z, CGScal* S, RedBuf rb,
                             const double* gath_pq, double* gath_rz, hipStream_t s) {
    k_gn_pcg_upd<<<gn_grid((int64_t)w * h), NT, 0, s>>>(w, h, k, fx, fy, f2, alpha, lam, p, x, r, z, S, rb,
                                                            gath_pq, gath_rz);
    return hipGetLastError();
}



// ============================================================================ multigrid-preconditioned CG
//
// PCG on the GN system (classical.py:68-130) preconditioned by one symmetric V-cycle:
// cell-centred levels (w, h) -> (ceil(w/2), ceil(h/2)) down to at most MG_COARSE cells;
// operator on level l: s_f (-Lambda) x_f + B x per cell, s = (alpha, alpha, lambda) / 4^l (the
// h^2 scaling of a 5-point Neumann Laplacian rediscretised on a grid twice as coarse),
// B = the pointwise 3x3 coupling v v^T (v = (fx, fy, -f2)) on level 0 and the average of the
// children's B (weighted like R B P) below; prolongation P = cell-centred bilinear (weights
// 3/4, 1/4 per axis, indices clamped at the Neumann boundary), restriction R = P^T / 4;
// one damped (omega = 0.8) block-Jacobi sweep before and after the coarse correction, the
// coarsest level smoothed MG_CSWEEPS times from zero in one block.  Every piece is a fixed
// symmetric linear operator, so the V-cycle is a valid CG preconditioner.  Any approximation
// here only changes the preconditioner: the PCG applies the exact operator (gn_row, CSR
// order) and stops on the exact residual norm.
//
// Launch structure (13 kernels per PCG iteration at 640x480, replayed as a hipGraph):
//   k_gnp_dir   stop test, beta, p = z + beta p, q = A p, partial p.q
//   k_gnp_upd   alpha, x += alpha p, r -= alpha A p, partial r.r
//   k_mg_down2  per level: pre-smoothing from zero, residual and restriction in one LDS tile
//   k_mg_coarse the coarsest level in one block
//   k_mg_up2    per level: prolongation of the coarse correction and post-smoothing in one
//               LDS tile (level 0: z and the partial r.z)
// Global sums are consumer-side: every reducing kernel stores one partial per block (no
// atomics, no ticket), and every kernel that needs the sum adds the partials in the same
// fixed order in each of its blocks, so all blocks take identical decisions.

#ifndef FOTO_MG_COARSE
#define FOTO_MG_COARSE 1024
#endif
#ifndef FOTO_MG_CSWEEPS
#define FOTO_MG_CSWEEPS 12   // 48 -> 12: same PCG counts at 640x480, 584x388, 320x240 (r02 A/B), 12 % less PCG time
#endif
constexpr int MG_COARSE = FOTO_MG_COARSE;   // cells of the coarsest level (one block, one cell per thread)
constexpr int MG_CSWEEPS = FOTO_MG_CSWEEPS;
constexpr double MG_OMEGA = 0.8;
constexpr int GT_X = 32, GT_Y = 16;   // fine tile of the level kernels (256 threads, 2 cells each)

struct MGLev {
    int w, h;
    double s0, s1, s2;
    const double* B;      // 6 planes: bxx bxy bxm byy bym bmm
    const double* Dinv;   // 6 planes: inverse of the cell's 3x3 diagonal block (symmetric)
};

static inline int mg_tiles(int w, int h) { return ((w + GT_X - 1) / GT_X) * ((h + GT_Y - 1) / GT_Y); }

__device__ __forceinline__ int mg_ncount(int x, int y, int w, int h) {
    return (x > 0) + (x < w - 1) + (y > 0) + (y < h - 1);
}

// 1-D prolongation weight of coarse index I for fine index i (nc coarse cells), clamped
__device__ __forceinline__ double mg_w1(int i, int I, int nc) {
    const int I0 = i >> 1;
    int I1 = (i & 1) ? I0 + 1 : I0 - 1;
    I1 = I1 < 0 ? 0 : (I1 > nc - 1 ? nc - 1 : I1);
    return (I0 == I ? 0.75 : 0.0) + (I1 == I ? 0.25 : 0.0);
}

__device__ __forceinline__ void mg_dinv(const MGLev& L, int64_t i, double r0, double r1, double r2, double& z0,
                                        double& z1, double& z2) {
    const int64_t n = (int64_t)L.w * L.h;
    const double* D = L.Dinv;
    const double d00 = D[i], d01 = D[n + i], d02 = D[2 * n + i], d11 = D[3 * n + i], d12 = D[4 * n + i],
                 d22 = D[5 * n + i];
    z0 = d00 * r0 + d01 * r1 + d02 * r2;
    z1 = d01 * r0 + d11 * r1 + d12 * r2;
    z2 = d02 * r0 + d12 * r1 + d22 * r2;
}

// the cell's 6 coefficient planes (B or Dinv: xx xy xm yy ym mm) into registers
__device__ __forceinline__ void mg_load6(const double* __restrict__ P, int64_t n, int64_t i, double (&c)[6]) {
#pragma unroll
    for (int k = 0; k < 6; ++k) c[k] = P[k * n + i];
}

// mg_dinv with the cell's inverse block already in registers (the same arithmetic)
__device__ __forceinline__ void mg_dinv_v(const double (&d)[6], double r0, double r1, double r2, double& z0,
                                          double& z1, double& z2) {
    z0 = d[0] * r0 + d[1] * r1 + d[2] * r2;
    z1 = d[1] * r0 + d[3] * r1 + d[4] * r2;
    z2 = d[2] * r0 + d[4] * r1 + d[5] * r2;
}

// (A x) of cell (x, y) with the cell's B in registers (mg_apply_t's arithmetic)
template <class F>
__device__ __forceinline__ void mg_apply_b(const MGLev& L, int x, int y, const double (&B)[6], F X, double& a0,
                                           double& a1, double& a2, double& v0, double& v1, double& v2) {
    const bool hxm = x > 0, hxp = x < L.w - 1, hym = y > 0, hyp = y < L.h - 1;
    const double c = (double)((int)hxm + (int)hxp + (int)hym + (int)hyp);
    double v[3], nb[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        v[f] = X(f, 0, 0);
        nb[f] = (hxm ? X(f, 0, -1) : 0.0) + (hxp ? X(f, 0, 1) : 0.0) + (hym ? X(f, -1, 0) : 0.0) +
                (hyp ? X(f, 1, 0) : 0.0);
    }
    a0 = L.s0 * (c * v[0] - nb[0]) + B[0] * v[0] + B[1] * v[1] + B[2] * v[2];
    a1 = L.s1 * (c * v[1] - nb[1]) + B[1] * v[0] + B[3] * v[1] + B[4] * v[2];
    a2 = L.s2 * (c * v[2] - nb[2]) + B[2] * v[0] + B[4] * v[1] + B[5] * v[2];
    v0 = v[0]; v1 = v[1]; v2 = v[2];
}

// (A x) of cell (x, y) = global index i, with the vector in an LDS tile: X(f, dy, dx) is the
// value at the neighbour offset (dy, dx) in {-1, 0, 1}; neighbours outside the grid are skipped
template <class F>
__device__ __forceinline__ void mg_apply_t(const MGLev& L, int x, int y, int64_t i, F X, double& a0, double& a1,
                                           double& a2, double& v0, double& v1, double& v2) {
    const int64_t n = (int64_t)L.w * L.h;
    const bool hxm = x > 0, hxp = x < L.w - 1, hym = y > 0, hyp = y < L.h - 1;
    const double c = (double)((int)hxm + (int)hxp + (int)hym + (int)hyp);
    double v[3], nb[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        v[f] = X(f, 0, 0);
        nb[f] = (hxm ? X(f, 0, -1) : 0.0) + (hxp ? X(f, 0, 1) : 0.0) + (hym ? X(f, -1, 0) : 0.0) +
                (hyp ? X(f, 1, 0) : 0.0);
    }
    const double* B = L.B;
    const double bxx = B[i], bxy = B[n + i], bxm = B[2 * n + i], byy = B[3 * n + i], bym = B[4 * n + i],
                 bmm = B[5 * n + i];
    a0 = L.s0 * (c * v[0] - nb[0]) + bxx * v[0] + bxy * v[1] + bxm * v[2];
    a1 = L.s1 * (c * v[1] - nb[1]) + bxy * v[0] + byy * v[1] + bym * v[2];
    a2 = L.s2 * (c * v[2] - nb[2]) + bxm * v[0] + bym * v[1] + bmm * v[2];
    v0 = v[0]; v1 = v[1]; v2 = v[2];
}

// ----------------------------------------------------------------------------- consumer-side sums

// sum of the nb partials of each of K arrays, in the same fixed order in every block
// (thread t adds t, t + NT, ...; then a fixed shuffle tree and the 4 wave sums in order)
template <int K>
__device__ __forceinline__ void mg_sum_partials(const double* const (&src)[K], int nb, double (&out)[K]) {
    __shared__ double sh[K][NT / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double v = 0.0;
        for (int i = threadIdx.x; i < nb; i += NT) v += src[k][i];
        v = gn_wave_sum(v);
        if (lane == 0) sh[k][wv] = v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double s = sh[k][0];
#pragma unroll
        for (int j = 1; j < NT / 64; ++j) s += sh[k][j];
        out[k] = s;
    }
}

// this block's partial of v -> dst[block] (fixed order)
__device__ __forceinline__ void mg_block_partial(double v, double* dst) {
    __shared__ double sh[NT / 64];
    v = gn_wave_sum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = sh[0];
#pragma unroll
        for (int j = 1; j < NT / 64; ++j) s += sh[j];
        dst[blockIdx.x] = s;
    }
}

// ----------------------------------------------------------------------------- PCG kernels

// r = b, partial r.r
__global__ __launch_bounds__(NT) void k_gnp_init(int64_t n, const double* __restrict__ b, double* __restrict__ r,
                                                 double* __restrict__ rr_part) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    double rr = 0.0;
    if (i < n) {
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const double v = b[f * n + i];
            r[f * n + i] = v;
            rr += v * v;
        }
    }
    mg_block_partial(rr, rr_part);
}

// iteration k (S->pad[0]): stop test on ||r_k|| (atol = rtol ||b|| fixed at k = 0), beta =
// rz_k / rz_{k-1}, p_k = z_k + beta p_{k-1} (for the pixel and its 4 neighbours), q = A p_k,
// partial p.q; writes p_k.
__global__ __launch_bounds__(NT) void k_gnp_dir(int w, int h, const double* __restrict__ fx,
                                                const double* __restrict__ fy, const double* __restrict__ f2,
                                                double a, double l, const double* __restrict__ z,
                                                const double* __restrict__ po, double* __restrict__ pn, CGScal* S,
                                                const double* rr_part, int nb_rr, const double* rz_cur,
                                                const double* rz_prev, int nb_rz, double* __restrict__ pq_part,
                                                double rtol, double* __restrict__ qout, const double* rr_part2,
                                                int nb_rr2) {
    // (round 5) the stencil values of z and p_{k-1} and the pixel's coefficients are loaded before
    // the partial sums that give beta, so the two waits overlap
    const int k = S->pad[0];
    const int done = S->done;
    const int64_t n = (int64_t)w * h;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    const bool in = i < n;
    const GNPix P = gn_pix(w, h, in ? i : 0);
    double zv[3][5], pv5[3][5], cfx = 0.0, cfy = 0.0, cf2 = 0.0;
    {
        const int64_t j5[5] = {P.hy ? i - w : i, P.hx ? i - 1 : i, i, P.hX ? i + 1 : i, P.hY ? i + w : i};
#pragma unroll
        for (int f = 0; f < 3; ++f)
#pragma unroll
            for (int q = 0; q < 5; ++q) {
                zv[f][q] = in ? z[f * n + j5[q]] : 0.0;
                pv5[f][q] = (in && k > 0) ? po[f * n + j5[q]] : 0.0;
            }
        if (in) { cfx = fx[i]; cfy = fy[i]; cf2 = f2[i]; }
    }
    double rr, rzc, rzp;
    {
        const double* src[2] = {rz_cur, rz_prev};
        double o[2];
        mg_sum_partials<2>(src, nb_rz, o);
        rzc = o[0];
        rzp = o[1];
        // r.r of r_k: k_gnp_init's partials at k = 0, then the update's (k_gnp_upd, or the level-0
        // down leg with the update folded in: rr_part2, one partial per tile)
        const bool second = rr_part2 && k > 0;
        const double* s1[1] = {second ? rr_part2 : rr_part};
        double o1[1];
        __syncthreads();   // mg_sum_partials' LDS is reused
        mg_sum_partials<1>(s1, second ? nb_rr2 : nb_rr, o1);
        rr = o1[0];
    }
    if (done) return;
    const double atol = (k == 0) ? fmax(0.0, rtol * sqrt(rr)) : S->atol;
    if (rr == 0.0 || sqrt(rr) < atol) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { S->done = 1; S->iters = k; }
        return;
    }
    if (k == 0 && blockIdx.x == 0 && threadIdx.x == 0) { S->bb = rr; S->atol = atol; }
    const double beta = (k > 0) ? rzc / rzp : 0.0;
    double pq = 0.0;
    if (in) {
        auto pv = [&](int f, int q) -> double { return (k == 0) ? zv[f][q] : beta * pv5[f][q] + zv[f][q]; };
        double qu, qv, qm;
        gn_row_v(P, cfx, cfy, cf2, a, l, pv, qu, qv, qm);
        const double pu = pv(0, 2), pvv = pv(1, 2), pm = pv(2, 2);
        pn[i] = pu; pn[n + i] = pvv; pn[2 * n + i] = pm;
        if (qout) { qout[i] = qu; qout[n + i] = qv; qout[2 * n + i] = qm; }   // (the folded update's A p)
        pq = pu * qu + pvv * qv + pm * qm;
    }
    mg_block_partial(pq, pq_part);
}

// alpha = rz_k / p.q; x += alpha p (x starts at 0); r -= alpha A p; partial r.r; k += 1
__global__ __launch_bounds__(NT) void k_gnp_upd(int w, int h, const double* __restrict__ fx,
                                                const double* __restrict__ fy, const double* __restrict__ f2,
                                                double a, double l, const double* __restrict__ p,
                                                double* __restrict__ x, double* __restrict__ r, CGScal* S,
                                                const double* rz_cur, int nb_rz, const double* pq_part, int nb_pq,
                                                double* __restrict__ rr_part) {
    if (S->done) return;
    double alpha;
    {
        const double* s1[1] = {rz_cur};
        double o1[1];
        mg_sum_partials<1>(s1, nb_rz, o1);
        const double* s2[1] = {pq_part};
        double o2[1];
        __syncthreads();
        mg_sum_partials<1>(s2, nb_pq, o2);
        alpha = o1[0] / o2[0];
    }
    const int64_t n = (int64_t)w * h;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    double rr = 0.0;
    if (i < n) {
        const GNPix P = gn_pix(w, h, i);
        double qu, qv, qm;
        gn_row(P, w, n, i, fx[i], fy[i], f2[i], a, l, [&](int f, int64_t j) { return p[f * n + j]; }, qu, qv, qm);
        const double q3[3] = {qu, qv, qm};
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const int64_t o = f * n + i;
            x[o] = x[o] + alpha * p[o];
            const double rn = r[o] - alpha * q3[f];
            r[o] = rn;
            rr += rn * rn;
        }
    }
    mg_block_partial(rr, rr_part);
    // the iteration index: read by k_gnp_dir only, so no block of this launch races with it
    if (blockIdx.x == 0 && threadIdx.x == 0) S->pad[0] = S->pad[0] + 1;
}

// device -> mapped pinned host memory, 8 B per lane (writes cross PCIe as the kernel runs)
__global__ __launch_bounds__(NT) void k_gn_download(int64_t n, const double* __restrict__ x, double* host) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i < n) host[i] = x[i];
}

// ----------------------------------------------------------------------------- V-cycle kernels

__global__ __launch_bounds__(NT) void k_mg_b0(int64_t n, const double* __restrict__ fx, const double* __restrict__ fy,
                                              const double* __restrict__ f2, double* __restrict__ B) {
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const double a = fx[i], b = fy[i], m = f2[i];
    B[i] = a * a;
    B[n + i] = a * b;
    B[2 * n + i] = -a * m;
    B[3 * n + i] = b * b;
    B[4 * n + i] = -b * m;
    B[5 * n + i] = m * m;
}

// coarse B = (sum of children B weighted by the P weights) / (sum of those weights)
// (FOTO_GN_SETUP_FUSE=0: this form and k_mg_dinv; default: k_mg_coarsen_d)
__global__ __launch_bounds__(NT) void k_mg_coarsen(int w, int h, const double* __restrict__ B, int wc, int hc,
                                                   double* __restrict__ Bc) {
    const int64_t nc = (int64_t)wc * hc, n = (int64_t)w * h;
    const int64_t I = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (I >= nc) return;
    const int J = (int)(I / wc), K = (int)(I - (int64_t)J * wc);
    double acc[6] = {0, 0, 0, 0, 0, 0}, ws = 0.0;
    for (int y = max(0, 2 * J - 1); y <= min(h - 1, 2 * J + 2); ++y) {
        const double wy = mg_w1(y, J, hc);
        for (int x = max(0, 2 * K - 1); x <= min(w - 1, 2 * K + 2); ++x) {
            const double wgt = wy * mg_w1(x, K, wc);
            if (wgt == 0.0) continue;
            const int64_t i = (int64_t)y * w + x;
#pragma unroll
            for (int f = 0; f < 6; ++f) acc[f] += wgt * B[f * n + i];
            ws += wgt;
        }
    }
#pragma unroll
    for (int f = 0; f < 6; ++f) Bc[f * nc + I] = acc[f] / ws;
}

// inverse of the 3x3 diagonal block diag(s c) + B (symmetric positive definite), cofactors, of
// cell (x, y) of level L from its B values
__device__ __forceinline__ void mg_dinv_vals(const MGLev& L, int x, int y, const double* Bv, double (&D)[6]) {
    const double c = (double)mg_ncount(x, y, L.w, L.h);
    const double a = L.s0 * c + Bv[0], b = Bv[1], d = Bv[2], e = L.s1 * c + Bv[3], f = Bv[4], g = L.s2 * c + Bv[5];
    // [[a b d] [b e f] [d f g]]
    const double c00 = e * g - f * f, c01 = d * f - b * g, c02 = b * f - d * e;
    const double c11 = a * g - d * d, c12 = b * d - a * f, c22 = a * e - b * b;
    const double det = a * c00 + b * c01 + d * c02, id = 1.0 / det;
    D[0] = c00 * id;
    D[1] = c01 * id;
    D[2] = c02 * id;
    D[3] = c11 * id;
    D[4] = c12 * id;
    D[5] = c22 * id;
}

__device__ __forceinline__ void mg_dinv_cell(const MGLev& L, int x, int y, int64_t i, const double* Bv,
                                             double* __restrict__ Dinv) {
    const int64_t n = (int64_t)L.w * L.h;
    double D[6];
    mg_dinv_vals(L, x, y, Bv, D);
#pragma unroll
    for (int k = 0; k < 6; ++k) Dinv[k * n + i] = D[k];
}

// level 0's B of a cell from the GN coefficients (fx, fy, f2) there: v v^T, v = (fx, fy, -f2)
__device__ __forceinline__ void mg_b_from(double a, double b, double m, double (&B)[6]) {
    B[0] = a * a;
    B[1] = a * b;
    B[2] = -a * m;
    B[3] = b * b;
    B[4] = -b * m;
    B[5] = m * m;
}

// the GN coefficient planes level 0's B and D^-1 are made of (round 6: the PCG's level-0 legs
// form both per cell from these 24 B instead of loading the stored 96 B; FOTO_GN_RECOMP=0: load)
struct MGCoef {
    const double* fx;
    const double* fy;
    const double* f2;
};

__global__ __launch_bounds__(NT) void k_mg_dinv(MGLev L, double* __restrict__ Dinv) {
    const int64_t n = (int64_t)L.w * L.h;
    const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    const int y = (int)(i / L.w), x = (int)(i - (int64_t)y * L.w);
    const double Bv[6] = {L.B[i], L.B[n + i], L.B[2 * n + i], L.B[3 * n + i], L.B[4 * n + i], L.B[5 * n + i]};
    mg_dinv_cell(L, x, y, i, Bv, Dinv);
}

// Round 6 (setup of a solve, 0.3 ms at 640x480 of which the coarsening was ~95 us over five
// launches and the block inverses six more): level 0's B with its block inverses in one pass, and
// each coarse level's B with its block inverses in one pass over a fixed 4 x 4 window (clamped
// addresses, every load issued at once; positions of weight 0 are skipped as before, so the sums
// are the same in the same order: bit-identical to k_mg_b0 / k_mg_coarsen + k_mg_dinv)
__global__ __launch_bounds__(NT) void k_mg_b0_d(MGLev L, const double* __restrict__ fx, const double* __restrict__ fy,
                                                const double* __restrict__ f2, double* __restrict__ B,
                                                double* __restrict__ Dinv) {
    const int n = L.w * L.h;
    const int i = blockIdx.x * NT + threadIdx.x;
    if (i >= n) return;
    double Bv[6];
    mg_b_from(fx[i], fy[i], f2[i], Bv);
#pragma unroll
    for (int f = 0; f < 6; ++f) B[(int64_t)f * n + i] = Bv[f];
    const int y = i / L.w;
    mg_dinv_cell(L, i - y * L.w, y, i, Bv, Dinv);
}

__global__ __launch_bounds__(NT) void k_mg_coarsen_d(int w, int h, const double* __restrict__ B, MGLev C,
                                                     double* __restrict__ Bc, double* __restrict__ Dinv) {
    const int nc = C.w * C.h, n = w * h;
    const int I = blockIdx.x * NT + threadIdx.x;
    if (I >= nc) return;
    const int J = I / C.w, K = I - J * C.w;
    double wy[4], wx[4];
    int ro[4], co[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int y = 2 * J - 1 + t, x = 2 * K - 1 + t;
        wy[t] = (y >= 0 && y < h) ? mg_w1(y, J, C.h) : 0.0;
        wx[t] = (x >= 0 && x < w) ? mg_w1(x, K, C.w) : 0.0;
        ro[t] = min(max(y, 0), h - 1) * w;
        co[t] = min(max(x, 0), w - 1);
    }
    double acc[6] = {0, 0, 0, 0, 0, 0}, ws = 0.0;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double wgt = wy[t] * wx[u];
            const int i = ro[t] + co[u];
            double v[6];
#pragma unroll
            for (int f = 0; f < 6; ++f) v[f] = B[(int64_t)f * n + i];
            if (wgt != 0.0) {
#pragma unroll
                for (int f = 0; f < 6; ++f) acc[f] += wgt * v[f];
                ws += wgt;
            }
        }
    double Bv[6];
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        Bv[f] = acc[f] / ws;
        Bc[(int64_t)f * nc + I] = Bv[f];
    }
    mg_dinv_cell(C, K, J, I, Bv, Dinv);
}

// k_gnp_upd folded into the level-0 down leg (round 5; FOTO_GN_FOLD=0: the separate kernel):
// alpha = rz_k / p.q from the same consumer-side sums, r' = r - alpha q on the tile and its halo
// (q = A p as k_gnp_dir computed it -- the values k_gnp_upd recomputes, bit for bit), x += alpha p
// and r' stored on the tile, and the partial r'.r' per tile.  r is double-buffered by iteration
// parity: the neighbouring tiles still read the old r of their halo cells.
struct MGUpd {
    const double* rold;
    double* rnew;
    const double* q;
    const double* p;
    double* x;
    const double* rz_cur;
    const double* pq_part;
    double* rr_part;
    CGScal* S;
    int nb_rz, nb_pq;
    MGCoef cf;   // (RC: level 0's B and D^-1 from these)
};

// Down leg of one level, one GT_Y x GT_X fine tile per block:
//   x = omega D^-1 f (pre-smoothing from zero) over the tile + 2 halo cells   -> LDS
//   r = f - A x over the tile + 1 halo cell                                   -> LDS; x -> xg
//   fc = R r = P^T r / 4 for the tile's GT_Y/2 x GT_X/2 coarse cells (4 x 4 taps) -> fc
// UPD (level 0 of a PCG iteration): f is r' = r - alpha q, formed here (MGUpd above)
#ifndef FOTO_MG_B2LATE
#define FOTO_MG_B2LATE 1
#endif
#ifndef FOTO_MG_RSALIAS
#define FOTO_MG_RSALIAS 1
#endif
template <bool UPD, bool RC = false>
__global__ __launch_bounds__(NT) void k_mg_down2(MGLev L, int wc, int hc, const CGScal* S,
                                                 const double* __restrict__ f, double* __restrict__ xg,
                                                 double* __restrict__ fc, MGUpd U) {
    // Every global load of the first two stages is issued up front (round 5): a small level's
    // launch was three dependent memory round trips (the done flag, f and D^-1, then B and f
    // again) at 7-8 us for 1-40 tiles.  f of the region goes to LDS for the second stage.
    constexpr int XW = GT_X + 4, XH = GT_Y + 4, RW = GT_X + 2, RH = GT_Y + 2;
    constexpr int C1 = (XH * XW + NT - 1) / NT, C2 = (RH * RW + NT - 1) / NT;
    __shared__ double xs[3][XH][XW];
    __shared__ double fs[3][XH][XW];
#if FOTO_MG_RSALIAS
    // r lives in fs's space (fs is dead once stage 2 has read it; one barrier more): 49 -> 35 KB
    // of LDS per block, four blocks per CU instead of three
    static_assert(3 * RH * RW <= 3 * XH * XW, "r fits f's space");
    double (*rs)[RH][RW] = reinterpret_cast<double (*)[RH][RW]>(&fs[0][0][0]);
#else
    __shared__ double rs[3][RH][RW];
#endif
    const int done = S->done;
    const int w = L.w, h = L.h;
    const int64_t n = (int64_t)w * h;
    const int tiles_x = (w + GT_X - 1) / GT_X;
    const int x0 = (blockIdx.x % tiles_x) * GT_X, y0 = (blockIdx.x / tiles_x) * GT_Y;
    // stage-2 cells' B (tile + 1 halo); level 0 of a PCG iteration (UPD, FOTO_MG_B2LATE=1): after
    // stage 1 -- held from the start beside the stage-1 loads it took 150 VGPRs (3 waves per SIMD)
    static_assert(!RC || UPD, "RC: the level-0 leg of a PCG iteration");
    constexpr int NB = RC ? 3 : 6;   // per stage-2 cell: (fx, fy, f2) or B
    double b2[C2][NB];
    auto load_b2 = [&]() {
#pragma unroll
        for (int k = 0; k < C2; ++k) {
            const int c = threadIdx.x + k * NT;
            const int ly = c / RW, lx = c - ly * RW, gy = y0 - 1 + ly, gx = x0 - 1 + lx;
            if (c < RH * RW && gx >= 0 && gx < w && gy >= 0 && gy < h) {
                const int64_t i = (int64_t)gy * w + gx;
                if constexpr (RC) {
                    b2[k][0] = U.cf.fx[i]; b2[k][1] = U.cf.fy[i]; b2[k][2] = U.cf.f2[i];
                } else {
                    for (int q = 0; q < 6; ++q) b2[k][q] = L.B[q * n + i];
                }
            } else {
                for (int q = 0; q < NB; ++q) b2[k][q] = 0.0;
            }
        }
    };
    constexpr bool B2LATE = UPD && FOTO_MG_B2LATE;
    if constexpr (!B2LATE) load_b2();
    // stage-1 cells' f (UPD: r and q) and D^-1 (tile + 2 halo; RC: the coefficients it is made of)
    constexpr int ND = RC ? 3 : 6;
    double f1[C1][3], d1[C1][ND];
#pragma unroll
    for (int k = 0; k < C1; ++k) {
        const int c = threadIdx.x + k * NT;
        const int ly = c / XW, lx = c - ly * XW, gy = y0 - 2 + ly, gx = x0 - 2 + lx;
        if (c < XH * XW && gx >= 0 && gx < w && gy >= 0 && gy < h) {
            const int64_t i = (int64_t)gy * w + gx;
            if constexpr (UPD) {
                f1[k][0] = U.rold[i]; f1[k][1] = U.rold[n + i]; f1[k][2] = U.rold[2 * n + i];
            } else {
                f1[k][0] = f[i]; f1[k][1] = f[n + i]; f1[k][2] = f[2 * n + i];
            }
            if constexpr (RC) {
                d1[k][0] = U.cf.fx[i]; d1[k][1] = U.cf.fy[i]; d1[k][2] = U.cf.f2[i];
            } else {
                for (int q = 0; q < 6; ++q) d1[k][q] = L.Dinv[q * n + i];
            }
        } else {
            f1[k][0] = f1[k][1] = f1[k][2] = 0.0;
            for (int q = 0; q < ND; ++q) d1[k][q] = 0.0;
        }
    }
    double alpha = 0.0;
    if constexpr (UPD) {   // r' = r - alpha q (k_gnp_upd's expression); alpha = rz_k / p.q
        double qv[C1][3];
#pragma unroll
        for (int k = 0; k < C1; ++k) {
            const int c = threadIdx.x + k * NT;
            const int ly = c / XW, lx = c - ly * XW, gy = y0 - 2 + ly, gx = x0 - 2 + lx;
            const bool in = c < XH * XW && gx >= 0 && gx < w && gy >= 0 && gy < h;
            const int64_t i = in ? (int64_t)gy * w + gx : 0;
#pragma unroll
            for (int fl = 0; fl < 3; ++fl) qv[k][fl] = in ? U.q[fl * n + i] : 0.0;
        }
        const double* s1[1] = {U.rz_cur};
        double o1[1];
        mg_sum_partials<1>(s1, U.nb_rz, o1);
        const double* s2[1] = {U.pq_part};
        double o2[1];
        __syncthreads();
        mg_sum_partials<1>(s2, U.nb_pq, o2);
        alpha = o1[0] / o2[0];
#pragma unroll
        for (int k = 0; k < C1; ++k)
#pragma unroll
            for (int fl = 0; fl < 3; ++fl) f1[k][fl] = f1[k][fl] - alpha * qv[k][fl];
    }
    if (done) return;   // (uniform; the loads above were issued before this wait)
#pragma unroll
    for (int k = 0; k < C1; ++k) {
        const int c = threadIdx.x + k * NT;
        if (c >= XH * XW) continue;
        const int ly = c / XW, lx = c - ly * XW, gy = y0 - 2 + ly, gx = x0 - 2 + lx;
        double z0 = 0.0, z1 = 0.0, z2 = 0.0;
        if (gx >= 0 && gx < w && gy >= 0 && gy < h) {
            if constexpr (RC) {
                double Bv[6], D[6];
                mg_b_from(d1[k][0], d1[k][1], d1[k][2], Bv);
                mg_dinv_vals(L, gx, gy, Bv, D);
                mg_dinv_v(D, f1[k][0], f1[k][1], f1[k][2], z0, z1, z2);
            } else {
                mg_dinv_v(d1[k], f1[k][0], f1[k][1], f1[k][2], z0, z1, z2);
            }
            z0 *= MG_OMEGA; z1 *= MG_OMEGA; z2 *= MG_OMEGA;
        }
        xs[0][ly][lx] = z0; xs[1][ly][lx] = z1; xs[2][ly][lx] = z2;
        fs[0][ly][lx] = f1[k][0]; fs[1][ly][lx] = f1[k][1]; fs[2][ly][lx] = f1[k][2];
    }
    if constexpr (B2LATE) load_b2();
    __syncthreads();
    double rr = 0.0;
    double rv[C2][3];
#pragma unroll
    for (int k = 0; k < C2; ++k) {
        const int c = threadIdx.x + k * NT;
        rv[k][0] = rv[k][1] = rv[k][2] = 0.0;
        if (c >= RH * RW) continue;
        const int ly = c / RW, lx = c - ly * RW, gy = y0 - 1 + ly, gx = x0 - 1 + lx;
        double r0 = 0.0, r1 = 0.0, r2 = 0.0;
        if (gx >= 0 && gx < w && gy >= 0 && gy < h) {
            const int64_t i = (int64_t)gy * w + gx;
            double a0, a1, a2, v0, v1, v2;
            double Bv[6];
            if constexpr (RC) mg_b_from(b2[k][0], b2[k][1], b2[k][2], Bv);
            else for (int q = 0; q < 6; ++q) Bv[q] = b2[k][q];
            mg_apply_b(L, gx, gy, Bv, [&](int fl, int dy, int dx) { return xs[fl][ly + 1 + dy][lx + 1 + dx]; }, a0,
                       a1, a2, v0, v1, v2);
            const double fa = fs[0][ly + 1][lx + 1], fb = fs[1][ly + 1][lx + 1], fcv = fs[2][ly + 1][lx + 1];
            r0 = fa - a0; r1 = fb - a1; r2 = fcv - a2;
            if (ly >= 1 && ly <= GT_Y && lx >= 1 && lx <= GT_X) {
                xg[i] = v0; xg[n + i] = v1; xg[2 * n + i] = v2;
                if constexpr (UPD) {   // k_gnp_upd's stores and its r.r terms, field order
                    const double fr[3] = {fa, fb, fcv};
#pragma unroll
                    for (int fl = 0; fl < 3; ++fl) {
                        const int64_t o = fl * n + i;
                        U.x[o] = U.x[o] + alpha * U.p[o];
                        U.rnew[o] = fr[fl];
                        rr += fr[fl] * fr[fl];
                    }
                }
            }
        }
        rv[k][0] = r0; rv[k][1] = r1; rv[k][2] = r2;
    }
#if FOTO_MG_RSALIAS
    __syncthreads();   // (every read of fs done)
#endif
#pragma unroll
    for (int k = 0; k < C2; ++k) {
        const int c = threadIdx.x + k * NT;
        if (c >= RH * RW) continue;
        const int ly = c / RW, lx = c - ly * RW;
        rs[0][ly][lx] = rv[k][0]; rs[1][ly][lx] = rv[k][1]; rs[2][ly][lx] = rv[k][2];
    }
    __syncthreads();
    const int64_t nc = (int64_t)wc * hc;
    for (int c = threadIdx.x; c < (GT_Y / 2) * (GT_X / 2); c += NT) {
        const int cy = c / (GT_X / 2), cx = c - cy * (GT_X / 2);
        const int J = y0 / 2 + cy, K = x0 / 2 + cx;
        if (J >= hc || K >= wc) continue;
        double wy[4], wx[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int y = 2 * J - 1 + d, x = 2 * K - 1 + d;
            wy[d] = (y >= 0 && y < h) ? mg_w1(y, J, hc) : 0.0;
            wx[d] = (x >= 0 && x < w) ? mg_w1(x, K, wc) : 0.0;
        }
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int dy = 0; dy < 4; ++dy) {
            double b0 = 0.0, b1 = 0.0, bb = 0.0;
#pragma unroll
            for (int dx = 0; dx < 4; ++dx) {
                const int ly = 2 * cy + dy, lx = 2 * cx + dx;   // (2J - 1 + dy) - (y0 - 1)
                b0 += wx[dx] * rs[0][ly][lx];
                b1 += wx[dx] * rs[1][ly][lx];
                bb += wx[dx] * rs[2][ly][lx];
            }
            a0 += wy[dy] * b0; a1 += wy[dy] * b1; a2 += wy[dy] * bb;
        }
        const int64_t I = (int64_t)J * wc + K;
        fc[I] = 0.25 * a0;
        fc[nc + I] = 0.25 * a1;
        fc[2 * nc + I] = 0.25 * a2;
    }
    if constexpr (UPD) {
        mg_block_partial(rr, U.rr_part);
        // the iteration index: read by k_gnp_dir only, so no block of this launch races with it
        if (blockIdx.x == 0 && threadIdx.x == 0) U.S->pad[0] = U.S->pad[0] + 1;
    }
}

// Up leg of one level, one GT_Y x GT_X fine tile per block:
//   x' = x + P ec over the tile + 1 halo cell -> LDS
//   out = x' + omega D^-1 (f - A x') on the tile; RZ: partial f . out -> rz_part[block]
// (Round 5: this kernel's B, f and D^-1 loaded before the prolongation stage, as k_mg_down2 does,
// measured 0.2-1.2 us slower per launch at every level -- not kept.)
template <bool RZ, bool RC = false>
__global__ __launch_bounds__(NT) void k_mg_up2(MGLev L, int wc, int hc, const CGScal* S,
                                               const double* __restrict__ ec, const double* __restrict__ f,
                                               const double* __restrict__ xg, double* __restrict__ out,
                                               double* __restrict__ rz_part, MGCoef cf = MGCoef{}) {
    if (S->done) return;
    constexpr int RW = GT_X + 2, RH = GT_Y + 2;
    __shared__ double xs[3][RH][RW];
    const int w = L.w, h = L.h;
    const int64_t n = (int64_t)w * h, nc = (int64_t)wc * hc;
    const int tiles_x = (w + GT_X - 1) / GT_X;
    const int x0 = (blockIdx.x % tiles_x) * GT_X, y0 = (blockIdx.x / tiles_x) * GT_Y;
    for (int c = threadIdx.x; c < RH * RW; c += NT) {
        const int ly = c / RW, lx = c - ly * RW, gy = y0 - 1 + ly, gx = x0 - 1 + lx;
        double v[3] = {0.0, 0.0, 0.0};
        if (gx >= 0 && gx < w && gy >= 0 && gy < h) {
            const int64_t i = (int64_t)gy * w + gx;
            const int X0 = gx >> 1, Y0 = gy >> 1;
            int X1 = (gx & 1) ? X0 + 1 : X0 - 1, Y1 = (gy & 1) ? Y0 + 1 : Y0 - 1;
            X1 = X1 < 0 ? 0 : (X1 > wc - 1 ? wc - 1 : X1);
            Y1 = Y1 < 0 ? 0 : (Y1 > hc - 1 ? hc - 1 : Y1);
            const int64_t c00 = (int64_t)Y0 * wc + X0, c01 = (int64_t)Y0 * wc + X1, c10 = (int64_t)Y1 * wc + X0,
                          c11 = (int64_t)Y1 * wc + X1;
#pragma unroll
            for (int fl = 0; fl < 3; ++fl) {
                const double* e = ec + fl * nc;
                v[fl] = xg[fl * n + i] + (0.5625 * e[c00] + 0.1875 * e[c01] + 0.1875 * e[c10] + 0.0625 * e[c11]);
            }
        }
        xs[0][ly][lx] = v[0]; xs[1][ly][lx] = v[1]; xs[2][ly][lx] = v[2];
    }
    __syncthreads();
    double rz = 0.0;
    for (int c = threadIdx.x; c < GT_Y * GT_X; c += NT) {
        const int ly = c / GT_X, lx = c - ly * GT_X, gy = y0 + ly, gx = x0 + lx;
        if (gx >= w || gy >= h) continue;
        const int64_t i = (int64_t)gy * w + gx;
        double a0, a1, a2, v0, v1, v2, z0, z1, z2;
        const auto X = [&](int fl, int dy, int dx) { return xs[fl][ly + 1 + dy][lx + 1 + dx]; };
        if constexpr (RC) {
            double Bv[6], D[6];
            mg_b_from(cf.fx[i], cf.fy[i], cf.f2[i], Bv);
            mg_apply_b(L, gx, gy, Bv, X, a0, a1, a2, v0, v1, v2);
            mg_dinv_vals(L, gx, gy, Bv, D);
            mg_dinv_v(D, f[i] - a0, f[n + i] - a1, f[2 * n + i] - a2, z0, z1, z2);
        } else {
            mg_apply_t(L, gx, gy, i, X, a0, a1, a2, v0, v1, v2);
            mg_dinv(L, i, f[i] - a0, f[n + i] - a1, f[2 * n + i] - a2, z0, z1, z2);
        }
        const double f0 = f[i], f1 = f[n + i], f2v = f[2 * n + i];
        const double o0 = v0 + MG_OMEGA * z0, o1 = v1 + MG_OMEGA * z1, o2 = v2 + MG_OMEGA * z2;
        out[i] = o0;
        out[n + i] = o1;
        out[2 * n + i] = o2;
        rz += f0 * o0 + f1 * o1 + f2v * o2;
    }
    if constexpr (RZ) mg_block_partial(rz, rz_part);
}

// coarsest level: MG_CSWEEPS damped block-Jacobi sweeps from zero in one block (x in LDS, each
// thread's cell coefficients in registers: a sweep touches no global memory), up to MG_CPT cells
// per thread (MG_COARSE > 1024: a coarsest level above 1024 cells, one V-cycle level less);
// RZ (single-level hierarchy): also the partial f . x -> rz_part[0]
constexpr int MG_CPT = (MG_COARSE + 1023) / 1024;
template <bool RZ>
__global__ __launch_bounds__(1024) void k_mg_coarse(MGLev L, const CGScal* S, const double* __restrict__ f,
                                                     double* __restrict__ xout, double* rz_part) {
    if (S->done) return;
    __shared__ double xs[2][3 * MG_COARSE];
    __shared__ double red[16];
    const int n = L.w * L.h;
    double f0[MG_CPT], f1[MG_CPT], f2v[MG_CPT], b[MG_CPT][6], d[MG_CPT][6], c[MG_CPT];
    int ci[MG_CPT];
    bool in[MG_CPT], hxm[MG_CPT], hxp[MG_CPT], hym[MG_CPT], hyp[MG_CPT];
#pragma unroll
    for (int q = 0; q < MG_CPT; ++q) {
        const int i = threadIdx.x + q * (int)blockDim.x;
        ci[q] = i;
        in[q] = i < n;
        const int y = in[q] ? i / L.w : 0, xx = in[q] ? i - y * L.w : 0;
        hxm[q] = xx > 0; hxp[q] = xx < L.w - 1; hym[q] = y > 0; hyp[q] = y < L.h - 1;
        c[q] = (double)mg_ncount(xx, y, L.w, L.h);
        f0[q] = f1[q] = f2v[q] = 0.0;
        for (int k = 0; k < 6; ++k) { b[q][k] = 0.0; d[q][k] = 0.0; }
        if (in[q]) {
            f0[q] = f[i]; f1[q] = f[n + i]; f2v[q] = f[2 * n + i];
#pragma unroll
            for (int k = 0; k < 6; ++k) { b[q][k] = L.B[k * n + i]; d[q][k] = L.Dinv[k * n + i]; }
            const double z0 = d[q][0] * f0[q] + d[q][1] * f1[q] + d[q][2] * f2v[q],
                         z1 = d[q][1] * f0[q] + d[q][3] * f1[q] + d[q][4] * f2v[q],
                         z2 = d[q][2] * f0[q] + d[q][4] * f1[q] + d[q][5] * f2v[q];
            xs[0][i] = MG_OMEGA * z0; xs[0][n + i] = MG_OMEGA * z1; xs[0][2 * n + i] = MG_OMEGA * z2;
        }
    }
    __syncthreads();
    const double sc[3] = {L.s0, L.s1, L.s2};
    int cur = 0;
    for (int sweep = 1; sweep < MG_CSWEEPS; ++sweep) {
#pragma unroll
        for (int q = 0; q < MG_CPT; ++q) {
            if (!in[q]) continue;
            const int i = ci[q];
            const double* xc = xs[cur];
            double v[3], a[3];
#pragma unroll
            for (int fl = 0; fl < 3; ++fl) {
                const double* qq = xc + fl * n;
                v[fl] = qq[i];
                const double nb = (hxm[q] ? qq[i - 1] : 0.0) + (hxp[q] ? qq[i + 1] : 0.0) +
                                  (hym[q] ? qq[i - L.w] : 0.0) + (hyp[q] ? qq[i + L.w] : 0.0);
                a[fl] = sc[fl] * (c[q] * v[fl] - nb);
            }
            const double r0 = f0[q] - (a[0] + b[q][0] * v[0] + b[q][1] * v[1] + b[q][2] * v[2]);
            const double r1 = f1[q] - (a[1] + b[q][1] * v[0] + b[q][3] * v[1] + b[q][4] * v[2]);
            const double r2 = f2v[q] - (a[2] + b[q][2] * v[0] + b[q][4] * v[1] + b[q][5] * v[2]);
            xs[cur ^ 1][i] = v[0] + MG_OMEGA * (d[q][0] * r0 + d[q][1] * r1 + d[q][2] * r2);
            xs[cur ^ 1][n + i] = v[1] + MG_OMEGA * (d[q][1] * r0 + d[q][3] * r1 + d[q][4] * r2);
            xs[cur ^ 1][2 * n + i] = v[2] + MG_OMEGA * (d[q][2] * r0 + d[q][4] * r1 + d[q][5] * r2);
        }
        cur ^= 1;
        __syncthreads();
    }
    double rz = 0.0;
#pragma unroll
    for (int q = 0; q < MG_CPT; ++q) {
        if (!in[q]) continue;
        const int i = ci[q];
        xout[i] = xs[cur][i]; xout[n + i] = xs[cur][n + i]; xout[2 * n + i] = xs[cur][2 * n + i];
        rz += f0[q] * xs[cur][i] + f1[q] * xs[cur][n + i] + f2v[q] * xs[cur][2 * n + i];
    }
    if constexpr (RZ) {
        rz = gn_wave_sum(rz);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = rz;
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = 0.0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
            rz_part[0] = s;
        }
    }
}

// The small levels in one block (FOTO_MG_TAIL=1; off by default -- measured slower): below ~80x60
// cells a level kernel is a few blocks whose launch and drain look costlier than its work (6-9 us
// each, five of the 13 launches of a PCG iteration at 640x480).  k_mg_tail runs the down legs of
// levels l0 .. c-1, the coarsest solve and the up legs back to l0 in one 1024-thread block, level
// arrays in global memory (L2-resident), a barrier between stages, every cell with the level
// kernels' formulas in their order (the same preconditioner bit for bit).  Replayed from the
// hipGraph the separate launches are cheap, and one CU's stages are latency-bound: 180 us per
// PCG iteration with the tail from 80x60 down, 137.6 from 40x30, 133.5-133.8 without (r03, A/B on
// one box).
constexpr int MG_TAIL_MAX = 6;
constexpr int MG_TAIL_CELLS = 1300;   // levels at most this many cells join the tail (5000: slower)
struct MGTail {
    int nl;                            // levels in the tail; the last one is the coarsest
    MGLev L[MG_TAIL_MAX];
    double* f[MG_TAIL_MAX];
    double* x[MG_TAIL_MAX];
    double* y[MG_TAIL_MAX];
};

__global__ __launch_bounds__(1024) void k_mg_tail(MGTail T, const CGScal* S) {
    if (S->done) return;
    const int tid = threadIdx.x;
    const int nl = T.nl;
    for (int l = 0; l + 1 < nl; ++l) {   // down legs (k_mg_down2's three stages, level-wide)
        const MGLev L = T.L[l];
        const int w = L.w, h = L.h;
        const int64_t n = (int64_t)w * h;
        const double* f = T.f[l];
        double* x = T.x[l];
        double* rr = T.y[l];   // the residual; y is the up leg's output, free until then
        for (int64_t i = tid; i < n; i += 1024) {
            double z0, z1, z2;
            mg_dinv(L, i, f[i], f[n + i], f[2 * n + i], z0, z1, z2);
            x[i] = z0 * MG_OMEGA; x[n + i] = z1 * MG_OMEGA; x[2 * n + i] = z2 * MG_OMEGA;
        }
        __syncthreads();
        for (int64_t i = tid; i < n; i += 1024) {
            const int gy = (int)(i / w), gx = (int)(i - (int64_t)gy * w);
            double a0, a1, a2, v0, v1, v2;
            mg_apply_t(L, gx, gy, i, [&](int fl, int dy, int dx) { return x[fl * n + i + (int64_t)dy * w + dx]; }, a0,
                       a1, a2, v0, v1, v2);
            rr[i] = f[i] - a0; rr[n + i] = f[n + i] - a1; rr[2 * n + i] = f[2 * n + i] - a2;
        }
        __syncthreads();
        const int wc = T.L[l + 1].w, hc = T.L[l + 1].h;
        const int64_t nc = (int64_t)wc * hc;
        double* fc = T.f[l + 1];
        for (int64_t I0 = tid; I0 < nc; I0 += 1024) {
            const int J = (int)(I0 / wc), K = (int)(I0 - (int64_t)J * wc);
            double wy[4], wx[4];
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                const int y = 2 * J - 1 + d, xx = 2 * K - 1 + d;
                wy[d] = (y >= 0 && y < h) ? mg_w1(y, J, hc) : 0.0;
                wx[d] = (xx >= 0 && xx < w) ? mg_w1(xx, K, wc) : 0.0;
            }
            double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
            for (int dy = 0; dy < 4; ++dy) {
                double b0 = 0.0, b1 = 0.0, b2 = 0.0;
                const int y = 2 * J - 1 + dy;
#pragma unroll
                for (int dx = 0; dx < 4; ++dx) {
                    const int xx = 2 * K - 1 + dx;
                    const bool in = y >= 0 && y < h && xx >= 0 && xx < w;
                    const int64_t i = in ? (int64_t)y * w + xx : 0;
                    b0 += wx[dx] * (in ? rr[i] : 0.0);
                    b1 += wx[dx] * (in ? rr[n + i] : 0.0);
                    b2 += wx[dx] * (in ? rr[2 * n + i] : 0.0);
                }
                a0 += wy[dy] * b0; a1 += wy[dy] * b1; a2 += wy[dy] * b2;
            }
            fc[I0] = 0.25 * a0;
            fc[nc + I0] = 0.25 * a1;
            fc[2 * nc + I0] = 0.25 * a2;
        }
        __syncthreads();
    }
    {   // the coarsest level: k_mg_coarse<false>'s sweeps
        const MGLev L = T.L[nl - 1];
        __shared__ double xs[2][3 * MG_COARSE];
        const int n = L.w * L.h, i = tid;
        const bool in = i < n;
        const int y = in ? i / L.w : 0, xx = in ? i - y * L.w : 0;
        const double* f = T.f[nl - 1];
        double f0 = 0, f1 = 0, f2v = 0;
        double b[6] = {0, 0, 0, 0, 0, 0}, d[6] = {0, 0, 0, 0, 0, 0};
        const bool hxm = xx > 0, hxp = xx < L.w - 1, hym = y > 0, hyp = y < L.h - 1;
        const double c = (double)mg_ncount(xx, y, L.w, L.h);
        if (in) {
            f0 = f[i]; f1 = f[n + i]; f2v = f[2 * n + i];
#pragma unroll
            for (int k = 0; k < 6; ++k) { b[k] = L.B[k * n + i]; d[k] = L.Dinv[k * n + i]; }
            const double z0 = d[0] * f0 + d[1] * f1 + d[2] * f2v, z1 = d[1] * f0 + d[3] * f1 + d[4] * f2v,
                         z2 = d[2] * f0 + d[4] * f1 + d[5] * f2v;
            xs[0][i] = MG_OMEGA * z0; xs[0][n + i] = MG_OMEGA * z1; xs[0][2 * n + i] = MG_OMEGA * z2;
        }
        __syncthreads();
        const double sc[3] = {L.s0, L.s1, L.s2};
        int cur = 0;
        for (int sweep = 1; sweep < MG_CSWEEPS; ++sweep) {
            if (in) {
                const double* xc = xs[cur];
                double v[3], a[3];
#pragma unroll
                for (int fl = 0; fl < 3; ++fl) {
                    const double* q = xc + fl * n;
                    v[fl] = q[i];
                    const double nb = (hxm ? q[i - 1] : 0.0) + (hxp ? q[i + 1] : 0.0) + (hym ? q[i - L.w] : 0.0) +
                                      (hyp ? q[i + L.w] : 0.0);
                    a[fl] = sc[fl] * (c * v[fl] - nb);
                }
                const double r0 = f0 - (a[0] + b[0] * v[0] + b[1] * v[1] + b[2] * v[2]);
                const double r1 = f1 - (a[1] + b[1] * v[0] + b[3] * v[1] + b[4] * v[2]);
                const double r2 = f2v - (a[2] + b[2] * v[0] + b[4] * v[1] + b[5] * v[2]);
                xs[cur ^ 1][i] = v[0] + MG_OMEGA * (d[0] * r0 + d[1] * r1 + d[2] * r2);
                xs[cur ^ 1][n + i] = v[1] + MG_OMEGA * (d[1] * r0 + d[3] * r1 + d[4] * r2);
                xs[cur ^ 1][2 * n + i] = v[2] + MG_OMEGA * (d[2] * r0 + d[4] * r1 + d[5] * r2);
            }
            cur ^= 1;
            __syncthreads();
        }
        if (in) {
            double* xo = T.x[nl - 1];
            xo[i] = xs[cur][i]; xo[n + i] = xs[cur][n + i]; xo[2 * n + i] = xs[cur][2 * n + i];
        }
        __syncthreads();
    }
    for (int l = nl - 2; l >= 0; --l) {   // up legs (k_mg_up2<false>'s two stages, level-wide)
        const MGLev L = T.L[l];
        const int w = L.w, h = L.h;
        const int64_t n = (int64_t)w * h;
        const int wc = T.L[l + 1].w, hc = T.L[l + 1].h;
        const int64_t nc = (int64_t)wc * hc;
        const double* ec = (l + 1 == nl - 1) ? T.x[nl - 1] : T.y[l + 1];
        double* x = T.x[l];   // x' = x + P ec, in place
        for (int64_t i = tid; i < n; i += 1024) {
            const int gy = (int)(i / w), gx = (int)(i - (int64_t)gy * w);
            const int X0 = gx >> 1, Y0 = gy >> 1;
            int X1 = (gx & 1) ? X0 + 1 : X0 - 1, Y1 = (gy & 1) ? Y0 + 1 : Y0 - 1;
            X1 = X1 < 0 ? 0 : (X1 > wc - 1 ? wc - 1 : X1);
            Y1 = Y1 < 0 ? 0 : (Y1 > hc - 1 ? hc - 1 : Y1);
            const int64_t c00 = (int64_t)Y0 * wc + X0, c01 = (int64_t)Y0 * wc + X1, c10 = (int64_t)Y1 * wc + X0,
                          c11 = (int64_t)Y1 * wc + X1;
#pragma unroll
            for (int fl = 0; fl < 3; ++fl) {
                const double* e = ec + fl * nc;
                x[fl * n + i] = x[fl * n + i] + (0.5625 * e[c00] + 0.1875 * e[c01] + 0.1875 * e[c10] + 0.0625 * e[c11]);
            }
        }
        __syncthreads();
        const double* f = T.f[l];
        double* out = T.y[l];
        for (int64_t i = tid; i < n; i += 1024) {
            const int gy = (int)(i / w), gx = (int)(i - (int64_t)gy * w);
            double a0, a1, a2, v0, v1, v2, z0, z1, z2;
            mg_apply_t(L, gx, gy, i, [&](int fl, int dy, int dx) { return x[fl * n + i + (int64_t)dy * w + dx]; }, a0,
                       a1, a2, v0, v1, v2);
            const double f0 = f[i], f1 = f[n + i], f2v = f[2 * n + i];
            mg_dinv(L, i, f0 - a0, f1 - a1, f2v - a2, z0, z1, z2);
            out[i] = v0 + MG_OMEGA * z0;
            out[n + i] = v1 + MG_OMEGA * z1;
            out[2 * n + i] = v2 + MG_OMEGA * z2;
        }
        __syncthreads();
    }
}

// ----------------------------------------------------------------------------- persistent small levels
// The levels from l0 down (each at most MG_PT_TILES tiles), the coarsest solve and the up legs
// back to l0 in ONE launch of tiles(l0) blocks (round 5, opt-in FOTO_MG_PTAIL=1): every small
// level kernel sat at a ~5.5 us launch floor.  Measured slower (profiles/r05_gn_ptail.txt): at
// 640x480 the launch takes 55 us for the 7 stages that the level kernels run in 43 -- a stage
// here is ~8 us, its `sc1` loads of the previous stage's tiles (dropped from the L2 by the `sc1`
// stores, served across the XCDs) plus the barrier cost as much as a kernel boundary does; the
// polls' s_sleep is not it (the same without).  Stage s's blocks hand their tiles to
// stage s + 1's through a grid barrier: every wave waits for its stores, the block joins a
// workgroup barrier, one lane adds to an agent-scope arrival counter and polls it with `sc1`
// loads until the whole grid has arrived.  Every load and store of the handed-off level arrays
// (f, x, y) is an `sc1` access (agent-scope relaxed atomics: L2-served, coherent across the
// XCDs without cache flushes -- MI355X_MICROARCH.md's hand-off table, row 1); B and D^-1 are
// read-only here.  Each cell's arithmetic is the level kernels' in their order (the same
// preconditioner bit for bit).  The counter only grows: launch i of a solve waits for
// (i * syncs + s + 1) * blocks arrivals (i = the PCG iteration index, S->pad[0]); the host zeroes
// it with the solve's scalars.  A poll that never completes (blocks not co-resident -- 64 small
// blocks on a 256-CU device) gives up after ~1 s and flags S->pad[1] instead of hanging.
#ifndef FOTO_PT_SLEEP
#define FOTO_PT_SLEEP 2   // s_sleep between two polls of the arrival counter (A/B builds)
#endif
constexpr int MG_PT_TILES = 64;     // a level joins the tail when it has at most this many tiles
constexpr int MG_PT_MAX = 8;
struct MGPTail {
    int nl;                         // levels l0 .. c (the last is the coarsest)
    MGLev L[MG_PT_MAX];
    double* f[MG_PT_MAX];
    double* x[MG_PT_MAX];
    double* y[MG_PT_MAX];
    unsigned* counter;
    int syncs;                      // grid barriers per launch
};

__device__ __forceinline__ double pt_ld(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pt_st(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void pt_grid_sync(unsigned* counter, unsigned target, CGScal* S) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int spins = 0;
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
#if FOTO_PT_SLEEP
            __builtin_amdgcn_s_sleep(FOTO_PT_SLEEP);
#endif
            if (++spins > (1 << 20)) {   // (~1 s: a barrier normally completes in microseconds)   // never co-resident: flag it, do not hang the device
                __hip_atomic_store(&S->pad[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
    }
    __syncthreads();
}

__global__ __launch_bounds__(NT) void k_mg_ptail(MGPTail T, CGScal* S) {
    if (S->done) return;
    constexpr int XW = GT_X + 4, XH = GT_Y + 4, RW = GT_X + 2, RH = GT_Y + 2;
    // one LDS pool: the level stages' x / r tiles, or the coarsest solve's two 3n buffers
    constexpr int PT_POOL = (3 * XH * XW + 3 * RH * RW) > 6 * MG_COARSE ? (3 * XH * XW + 3 * RH * RW) : 6 * MG_COARSE;
    __shared__ double pool[PT_POOL];
    auto xs = reinterpret_cast<double(*)[XH][XW]>(pool);
    auto rs = reinterpret_cast<double(*)[RH][RW]>(pool + 3 * XH * XW);
    const unsigned nb = gridDim.x;
    unsigned target = (unsigned)S->pad[0] * (unsigned)T.syncs * nb;
    const int nl = T.nl, c = nl - 1;
    // ---- down legs: k_mg_down2<false>'s three stages, tile = blockIdx.x
    for (int l = 0; l < c; ++l) {
        const MGLev L = T.L[l];
        const int w = L.w, h = L.h, wc = T.L[l + 1].w, hc = T.L[l + 1].h;
        const int tiles_x = (w + GT_X - 1) / GT_X, ntiles = tiles_x * ((h + GT_Y - 1) / GT_Y);
        if ((int)blockIdx.x < ntiles) {
            const int64_t n = (int64_t)w * h, nc = (int64_t)wc * hc;
            const double* f = T.f[l];
            double* xg = T.x[l];
            double* fc = T.f[l + 1];
            const int x0 = (blockIdx.x % tiles_x) * GT_X, y0 = (blockIdx.x / tiles_x) * GT_Y;
            for (int cc = threadIdx.x; cc < XH * XW; cc += NT) {
                const int ly = cc / XW, lx = cc - ly * XW, gy = y0 - 2 + ly, gx = x0 - 2 + lx;
                double z0 = 0.0, z1 = 0.0, z2 = 0.0;
                if (gx >= 0 && gx < w && gy >= 0 && gy < h) {
                    const int64_t i = (int64_t)gy * w + gx;
                    mg_dinv(L, i, pt_ld(&f[i]), pt_ld(&f[n + i]), pt_ld(&f[2 * n + i]), z0, z1, z2);
                    z0 *= MG_OMEGA; z1 *= MG_OMEGA; z2 *= MG_OMEGA;
                }
                xs[0][ly][lx] = z0; xs[1][ly][lx] = z1; xs[2][ly][lx] = z2;
            }
            __syncthreads();
            for (int cc = threadIdx.x; cc < RH * RW; cc += NT) {
                const int ly = cc / RW, lx = cc - ly * RW, gy = y0 - 1 + ly, gx = x0 - 1 + lx;
                double r0 = 0.0, r1 = 0.0, r2 = 0.0;
                if (gx >= 0 && gx < w && gy >= 0 && gy < h) {
                    const int64_t i = (int64_t)gy * w + gx;
                    double a0, a1, a2, v0, v1, v2;
                    mg_apply_t(L, gx, gy, i, [&](int fl, int dy, int dx) { return xs[fl][ly + 1 + dy][lx + 1 + dx]; },
                               a0, a1, a2, v0, v1, v2);
                    r0 = pt_ld(&f[i]) - a0; r1 = pt_ld(&f[n + i]) - a1; r2 = pt_ld(&f[2 * n + i]) - a2;
                    if (ly >= 1 && ly <= GT_Y && lx >= 1 && lx <= GT_X) {
                        pt_st(&xg[i], v0); pt_st(&xg[n + i], v1); pt_st(&xg[2 * n + i], v2);
                    }
                }
                rs[0][ly][lx] = r0; rs[1][ly][lx] = r1; rs[2][ly][lx] = r2;
            }
            __syncthreads();
            for (int cc = threadIdx.x; cc < (GT_Y / 2) * (GT_X / 2); cc += NT) {
                const int cy = cc / (GT_X / 2), cx = cc - cy * (GT_X / 2);
                const int J = y0 / 2 + cy, K = x0 / 2 + cx;
                if (J >= hc || K >= wc) continue;
                double wy[4], wx[4];
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const int y = 2 * J - 1 + d, x = 2 * K - 1 + d;
                    wy[d] = (y >= 0 && y < h) ? mg_w1(y, J, hc) : 0.0;
                    wx[d] = (x >= 0 && x < w) ? mg_w1(x, K, wc) : 0.0;
                }
                double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
                for (int dy = 0; dy < 4; ++dy) {
                    double b0 = 0.0, b1 = 0.0, b2 = 0.0;
#pragma unroll
                    for (int dx = 0; dx < 4; ++dx) {
                        const int ly = 2 * cy + dy, lx = 2 * cx + dx;
                        b0 += wx[dx] * rs[0][ly][lx];
                        b1 += wx[dx] * rs[1][ly][lx];
                        b2 += wx[dx] * rs[2][ly][lx];
                    }
                    a0 += wy[dy] * b0; a1 += wy[dy] * b1; a2 += wy[dy] * b2;
                }
                const int64_t I = (int64_t)J * wc + K;
                pt_st(&fc[I], 0.25 * a0);
                pt_st(&fc[nc + I], 0.25 * a1);
                pt_st(&fc[2 * nc + I], 0.25 * a2);
            }
        }
        target += nb;
        pt_grid_sync(T.counter, target, S);
    }
    // ---- the coarsest level: k_mg_coarse<false>'s sweeps in block 0, up to 4 cells per thread
    if (blockIdx.x == 0) {
        constexpr int CP = (MG_COARSE + NT - 1) / NT;
        const MGLev L = T.L[c];
        const int n = L.w * L.h;
        auto xb = [&](int i) { return pool + i * (3 * MG_COARSE); };   // the two sweep buffers
        const double* f = T.f[c];
        double f0[CP], f1[CP], f2v[CP], b[CP][6], d[CP][6], cn[CP];
        int ci[CP];
        bool in[CP], hxm[CP], hxp[CP], hym[CP], hyp[CP];
#pragma unroll
        for (int q = 0; q < CP; ++q) {
            const int i = threadIdx.x + q * NT;
            ci[q] = i;
            in[q] = i < n;
            const int y = in[q] ? i / L.w : 0, xx = in[q] ? i - y * L.w : 0;
            hxm[q] = xx > 0; hxp[q] = xx < L.w - 1; hym[q] = y > 0; hyp[q] = y < L.h - 1;
            cn[q] = (double)mg_ncount(xx, y, L.w, L.h);
            f0[q] = f1[q] = f2v[q] = 0.0;
            for (int k = 0; k < 6; ++k) { b[q][k] = 0.0; d[q][k] = 0.0; }
            if (in[q]) {
                f0[q] = pt_ld(&f[i]); f1[q] = pt_ld(&f[n + i]); f2v[q] = pt_ld(&f[2 * n + i]);
#pragma unroll
                for (int k = 0; k < 6; ++k) { b[q][k] = L.B[k * n + i]; d[q][k] = L.Dinv[k * n + i]; }
                const double z0 = d[q][0] * f0[q] + d[q][1] * f1[q] + d[q][2] * f2v[q],
                             z1 = d[q][1] * f0[q] + d[q][3] * f1[q] + d[q][4] * f2v[q],
                             z2 = d[q][2] * f0[q] + d[q][4] * f1[q] + d[q][5] * f2v[q];
                xb(0)[i] = MG_OMEGA * z0; xb(0)[n + i] = MG_OMEGA * z1; xb(0)[2 * n + i] = MG_OMEGA * z2;
            }
        }
        __syncthreads();
        const double sc[3] = {L.s0, L.s1, L.s2};
        int cur = 0;
        for (int sweep = 1; sweep < MG_CSWEEPS; ++sweep) {
#pragma unroll
            for (int q = 0; q < CP; ++q) {
                if (!in[q]) continue;
                const int i = ci[q];
                const double* xc = xb(cur);
                double v[3], a[3];
#pragma unroll
                for (int fl = 0; fl < 3; ++fl) {
                    const double* qq = xc + fl * n;
                    v[fl] = qq[i];
                    const double nbv = (hxm[q] ? qq[i - 1] : 0.0) + (hxp[q] ? qq[i + 1] : 0.0) +
                                       (hym[q] ? qq[i - L.w] : 0.0) + (hyp[q] ? qq[i + L.w] : 0.0);
                    a[fl] = sc[fl] * (cn[q] * v[fl] - nbv);
                }
                const double r0 = f0[q] - (a[0] + b[q][0] * v[0] + b[q][1] * v[1] + b[q][2] * v[2]);
                const double r1 = f1[q] - (a[1] + b[q][1] * v[0] + b[q][3] * v[1] + b[q][4] * v[2]);
                const double r2 = f2v[q] - (a[2] + b[q][2] * v[0] + b[q][4] * v[1] + b[q][5] * v[2]);
                xb(cur ^ 1)[i] = v[0] + MG_OMEGA * (d[q][0] * r0 + d[q][1] * r1 + d[q][2] * r2);
                xb(cur ^ 1)[n + i] = v[1] + MG_OMEGA * (d[q][1] * r0 + d[q][3] * r1 + d[q][4] * r2);
                xb(cur ^ 1)[2 * n + i] = v[2] + MG_OMEGA * (d[q][2] * r0 + d[q][4] * r1 + d[q][5] * r2);
            }
            cur ^= 1;
            __syncthreads();
        }
        double* xo = T.x[c];
#pragma unroll
        for (int q = 0; q < CP; ++q) {
            if (!in[q]) continue;
            const int i = ci[q];
            pt_st(&xo[i], xb(cur)[i]); pt_st(&xo[n + i], xb(cur)[n + i]); pt_st(&xo[2 * n + i], xb(cur)[2 * n + i]);
        }
    }
    target += nb;
    pt_grid_sync(T.counter, target, S);
    // ---- up legs: k_mg_up2<false>'s two stages
    for (int l = c - 1; l >= 0; --l) {
        const MGLev L = T.L[l];
        const int w = L.w, h = L.h, wc = T.L[l + 1].w, hc = T.L[l + 1].h;
        const int tiles_x = (w + GT_X - 1) / GT_X, ntiles = tiles_x * ((h + GT_Y - 1) / GT_Y);
        if ((int)blockIdx.x < ntiles) {
            const int64_t n = (int64_t)w * h, nc = (int64_t)wc * hc;
            const double* ec = (l + 1 == c) ? T.x[c] : T.y[l + 1];
            const double* f = T.f[l];
            const double* xg = T.x[l];
            double* outp = T.y[l];
            const int x0 = (blockIdx.x % tiles_x) * GT_X, y0 = (blockIdx.x / tiles_x) * GT_Y;
            for (int cc = threadIdx.x; cc < RH * RW; cc += NT) {
                const int ly = cc / RW, lx = cc - ly * RW, gy = y0 - 1 + ly, gx = x0 - 1 + lx;
                double v[3] = {0.0, 0.0, 0.0};
                if (gx >= 0 && gx < w && gy >= 0 && gy < h) {
                    const int64_t i = (int64_t)gy * w + gx;
                    const int X0 = gx >> 1, Y0 = gy >> 1;
                    int X1 = (gx & 1) ? X0 + 1 : X0 - 1, Y1 = (gy & 1) ? Y0 + 1 : Y0 - 1;
                    X1 = X1 < 0 ? 0 : (X1 > wc - 1 ? wc - 1 : X1);
                    Y1 = Y1 < 0 ? 0 : (Y1 > hc - 1 ? hc - 1 : Y1);
                    const int64_t c00 = (int64_t)Y0 * wc + X0, c01 = (int64_t)Y0 * wc + X1,
                                  c10 = (int64_t)Y1 * wc + X0, c11 = (int64_t)Y1 * wc + X1;
#pragma unroll
                    for (int fl = 0; fl < 3; ++fl) {
                        const double* e = ec + fl * nc;
                        v[fl] = pt_ld(&xg[fl * n + i]) + (0.5625 * pt_ld(&e[c00]) + 0.1875 * pt_ld(&e[c01]) +
                                                          0.1875 * pt_ld(&e[c10]) + 0.0625 * pt_ld(&e[c11]));
                    }
                }
                xs[0][ly][lx] = v[0]; xs[1][ly][lx] = v[1]; xs[2][ly][lx] = v[2];
            }
            __syncthreads();
            for (int cc = threadIdx.x; cc < GT_Y * GT_X; cc += NT) {
                const int ly = cc / GT_X, lx = cc - ly * GT_X, gy = y0 + ly, gx = x0 + lx;
                if (gx >= w || gy >= h) continue;
                const int64_t i = (int64_t)gy * w + gx;
                double a0, a1, a2, v0, v1, v2, z0, z1, z2;
                mg_apply_t(L, gx, gy, i, [&](int fl, int dy, int dx) { return xs[fl][ly + 1 + dy][lx + 1 + dx]; }, a0,
                           a1, a2, v0, v1, v2);
                const double f0 = pt_ld(&f[i]), f1 = pt_ld(&f[n + i]), f2v = pt_ld(&f[2 * n + i]);
                mg_dinv(L, i, f0 - a0, f1 - a1, f2v - a2, z0, z1, z2);
                pt_st(&outp[i], v0 + MG_OMEGA * z0);
                pt_st(&outp[n + i], v1 + MG_OMEGA * z1);
                pt_st(&outp[2 * n + i], v2 + MG_OMEGA * z2);
            }
        }
        if (l > 0) {
            target += nb;
            pt_grid_sync(T.counter, target, S);
        }
    }
}

// ----------------------------------------------------------------------------- last level + coarsest in LDS
// The down leg of the level above the coarsest, the coarsest solve and that level's up leg in one
// block whose vectors never leave the LDS (round 5, default where the level has at most
// MG_LT_CELLS cells: 40x30 at 640x480 and 320x240; FOTO_MG_LTAIL=0: the three level kernels).
// The one-block tail of round 3 kept its level arrays in global memory and was slower; here
// f, x, r and the coarse vectors sit in ~94 KB of LDS, each cell's B and D^-1 in registers, and
// the stages are separated by workgroup barriers only.  Every cell's arithmetic is the level
// kernels' (k_mg_down2, k_mg_coarse, k_mg_up2) in their order: the same preconditioner bit for
// bit.  Reads f of the level (the down leg above wrote it), writes only the up leg's output y.
constexpr int MG_LT_CELLS = 1536;
constexpr int MG_LT_NTH = 512;    // (1024 threads: 128 VGPRs, the cells' coefficients spilled)
constexpr int MG_LT_CPT = (MG_LT_CELLS + MG_LT_NTH - 1) / MG_LT_NTH;   // fine cells per thread
__host__ __device__ constexpr size_t mg_lt_lds(int n, int nc) {   // doubles of dynamic LDS
    return 3 * (size_t)n + 3 * (size_t)n + (3 * (size_t)n > 6 * (size_t)nc ? 3 * (size_t)n : 6 * (size_t)nc) +
           3 * (size_t)nc;
}
__global__ __launch_bounds__(MG_LT_NTH) void k_mg_ltail(MGLev L, MGLev C, const CGScal* S,
                                                        const double* __restrict__ f, double* __restrict__ y) {
    if (S->done) return;
    extern __shared__ double lds[];
    const int w = L.w, h = L.h, n = w * h, wc = C.w, hc = C.h, nc = wc * hc;
    double* fL = lds;               // f of the level
    double* xL = fL + 3 * n;        // the down leg's x, then x' = x + P e
    double* rL = xL + 3 * n;        // r, then the coarse solve's two sweep buffers
    double* fcL = rL + (3 * n > 6 * nc ? 3 * n : 6 * nc);   // f of the coarsest level
    const int tid = threadIdx.x;
    // the coarsest cell's coefficients first (they were a dependent round trip mid-kernel)
    double cb[6], cd[6];
    {
        const bool cin = tid < nc;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            cb[k] = cin ? C.B[k * nc + tid] : 0.0;
            cd[k] = cin ? C.Dinv[k * nc + tid] : 0.0;
        }
    }
    // the fine cells' coefficients in registers; f into LDS
    double bq[MG_LT_CPT][6], dq[MG_LT_CPT][6];
#pragma unroll
    for (int q = 0; q < MG_LT_CPT; ++q) {
        const int i = tid + q * MG_LT_NTH;
        if (i < n) {
            for (int k = 0; k < 6; ++k) { bq[q][k] = L.B[k * n + i]; dq[q][k] = L.Dinv[k * n + i]; }
            for (int fl = 0; fl < 3; ++fl) fL[fl * n + i] = f[fl * n + i];
        } else {
            for (int k = 0; k < 6; ++k) { bq[q][k] = 0.0; dq[q][k] = 0.0; }
        }
    }
    __syncthreads();
    // down leg, stage 1: x = omega D^-1 f
#pragma unroll
    for (int q = 0; q < MG_LT_CPT; ++q) {
        const int i = tid + q * MG_LT_NTH;
        if (i >= n) continue;
        double z0, z1, z2;
        mg_dinv_v(dq[q], fL[i], fL[n + i], fL[2 * n + i], z0, z1, z2);
        xL[i] = z0 * MG_OMEGA; xL[n + i] = z1 * MG_OMEGA; xL[2 * n + i] = z2 * MG_OMEGA;
    }
    __syncthreads();
    // stage 2: r = f - A x
#pragma unroll
    for (int q = 0; q < MG_LT_CPT; ++q) {
        const int i = tid + q * MG_LT_NTH;
        if (i >= n) continue;
        const int gy = i / w, gx = i - gy * w;
        double a0, a1, a2, v0, v1, v2;
        mg_apply_b(L, gx, gy, bq[q], [&](int fl, int dy, int dx) { return xL[fl * n + i + dy * w + dx]; }, a0, a1,
                   a2, v0, v1, v2);
        rL[i] = fL[i] - a0; rL[n + i] = fL[n + i] - a1; rL[2 * n + i] = fL[2 * n + i] - a2;
    }
    __syncthreads();
    // stage 3: fc = R r (4 x 4 taps; taps outside the grid weigh 0 and read 0, as the tile's halo)
    for (int I0 = tid; I0 < nc; I0 += MG_LT_NTH) {
        const int J = I0 / wc, K = I0 - J * wc;
        double wy[4], wx[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const int yy = 2 * J - 1 + d, xx = 2 * K - 1 + d;
            wy[d] = (yy >= 0 && yy < h) ? mg_w1(yy, J, hc) : 0.0;
            wx[d] = (xx >= 0 && xx < w) ? mg_w1(xx, K, wc) : 0.0;
        }
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
        for (int dy = 0; dy < 4; ++dy) {
            double b0 = 0.0, b1 = 0.0, b2 = 0.0;
            const int yy = 2 * J - 1 + dy;
#pragma unroll
            for (int dx = 0; dx < 4; ++dx) {
                const int xx = 2 * K - 1 + dx;
                const bool in = yy >= 0 && yy < h && xx >= 0 && xx < w;
                const int i = in ? yy * w + xx : 0;
                b0 += wx[dx] * (in ? rL[i] : 0.0);
                b1 += wx[dx] * (in ? rL[n + i] : 0.0);
                b2 += wx[dx] * (in ? rL[2 * n + i] : 0.0);
            }
            a0 += wy[dy] * b0; a1 += wy[dy] * b1; a2 += wy[dy] * b2;
        }
        fcL[I0] = 0.25 * a0;
        fcL[nc + I0] = 0.25 * a1;
        fcL[2 * nc + I0] = 0.25 * a2;
    }
    __syncthreads();
    // the coarsest level: k_mg_coarse<false>'s sweeps (one cell per thread: the host checks nc <= MG_LT_NTH)
    {
        double* xb0 = rL;
        double* xb1 = rL + 3 * nc;
        const int i = tid;
        const bool in = i < nc;
        const int yc = in ? i / wc : 0, xc = in ? i - yc * wc : 0;
        double f0 = 0, f1 = 0, f2v = 0, b[6], d[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) { b[k] = cb[k]; d[k] = cd[k]; }
        const bool hxm = xc > 0, hxp = xc < wc - 1, hym = yc > 0, hyp = yc < hc - 1;
        const double cn = (double)mg_ncount(xc, yc, wc, hc);
        if (in) {
            f0 = fcL[i]; f1 = fcL[nc + i]; f2v = fcL[2 * nc + i];
            const double z0 = d[0] * f0 + d[1] * f1 + d[2] * f2v, z1 = d[1] * f0 + d[3] * f1 + d[4] * f2v,
                         z2 = d[2] * f0 + d[4] * f1 + d[5] * f2v;
            xb0[i] = MG_OMEGA * z0; xb0[nc + i] = MG_OMEGA * z1; xb0[2 * nc + i] = MG_OMEGA * z2;
        }
        __syncthreads();
        const double sc[3] = {C.s0, C.s1, C.s2};
        int cur = 0;
        for (int sweep = 1; sweep < MG_CSWEEPS; ++sweep) {
            if (in) {
                const double* xcur = cur ? xb1 : xb0;
                double* xnext = cur ? xb0 : xb1;
                double v[3], a[3];
#pragma unroll
                for (int fl = 0; fl < 3; ++fl) {
                    const double* qq = xcur + fl * nc;
                    v[fl] = qq[i];
                    const double nbv = (hxm ? qq[i - 1] : 0.0) + (hxp ? qq[i + 1] : 0.0) + (hym ? qq[i - wc] : 0.0) +
                                       (hyp ? qq[i + wc] : 0.0);
                    a[fl] = sc[fl] * (cn * v[fl] - nbv);
                }
                const double r0 = f0 - (a[0] + b[0] * v[0] + b[1] * v[1] + b[2] * v[2]);
                const double r1 = f1 - (a[1] + b[1] * v[0] + b[3] * v[1] + b[4] * v[2]);
                const double r2 = f2v - (a[2] + b[2] * v[0] + b[4] * v[1] + b[5] * v[2]);
                xnext[i] = v[0] + MG_OMEGA * (d[0] * r0 + d[1] * r1 + d[2] * r2);
                xnext[nc + i] = v[1] + MG_OMEGA * (d[1] * r0 + d[3] * r1 + d[4] * r2);
                xnext[2 * nc + i] = v[2] + MG_OMEGA * (d[2] * r0 + d[4] * r1 + d[5] * r2);
            }
            cur ^= 1;
            __syncthreads();
        }
        // up leg, stage 1: x' = x + P e (pointwise: in place)
        const double* ec = cur ? xb1 : xb0;
#pragma unroll
        for (int q = 0; q < MG_LT_CPT; ++q) {
            const int ii = tid + q * MG_LT_NTH;
            if (ii >= n) continue;
            const int gy = ii / w, gx = ii - gy * w;
            const int X0 = gx >> 1, Y0 = gy >> 1;
            int X1 = (gx & 1) ? X0 + 1 : X0 - 1, Y1 = (gy & 1) ? Y0 + 1 : Y0 - 1;
            X1 = X1 < 0 ? 0 : (X1 > wc - 1 ? wc - 1 : X1);
            Y1 = Y1 < 0 ? 0 : (Y1 > hc - 1 ? hc - 1 : Y1);
            const int c00 = Y0 * wc + X0, c01 = Y0 * wc + X1, c10 = Y1 * wc + X0, c11 = Y1 * wc + X1;
#pragma unroll
            for (int fl = 0; fl < 3; ++fl) {
                const double* e = ec + fl * nc;
                xL[fl * n + ii] = xL[fl * n + ii] + (0.5625 * e[c00] + 0.1875 * e[c01] + 0.1875 * e[c10] + 0.0625 * e[c11]);
            }
        }
    }
    __syncthreads();
    // stage 2: y = x' + omega D^-1 (f - A x')
#pragma unroll
    for (int q = 0; q < MG_LT_CPT; ++q) {
        const int i = tid + q * MG_LT_NTH;
        if (i >= n) continue;
        const int gy = i / w, gx = i - gy * w;
        double a0, a1, a2, v0, v1, v2, z0, z1, z2;
        mg_apply_b(L, gx, gy, bq[q], [&](int fl, int dy, int dx) { return xL[fl * n + i + dy * w + dx]; }, a0, a1,
                   a2, v0, v1, v2);
        const double f0 = fL[i], f1 = fL[n + i], f2v = fL[2 * n + i];
        mg_dinv_v(dq[q], f0 - a0, f1 - a1, f2v - a2, z0, z1, z2);
        y[i] = v0 + MG_OMEGA * z0;
        y[n + i] = v1 + MG_OMEGA * z1;
        y[2 * n + i] = v2 + MG_OMEGA * z2;
    }
}

}  // namespace foto

// ============================================================================ GN plan (host)

using namespace foto;

namespace {

// The host side of a solve is two copies between the caller's pageable arrays and the plan's
// pinned staging: 5 MB in, 7.4 MB out at 640x480, 0.13 + 0.22 ms on one core against a 4.6 ms
// solve (FOTO_GN_TRACE).  A few workers made with the staging split them; the caller takes a
// share too.  FOTO_GN_HOST_THREADS (default 4) counts the workers; 0 copies on the caller alone.
class HostPool {
public:
    explicit HostPool(int workers) {
        for (int t = 0; t < workers; ++t) th_.emplace_back([this] { loop(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int workers() const { return (int)th_.size(); }
    // f(i) for every i < n, on the workers and the caller; returns when all have run
    void run(int n, const std::function<void(int)>& f) {
        if (th_.empty() || n <= 1) {
            for (int i = 0; i < n; ++i) f(i);
            return;
        }
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &f;
            n_ = n;
            next_.store(0);
            pending_ = (int)th_.size();
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> g(mu_);
        done_.wait(g, [this] { return pending_ == 0; });
        job_ = nullptr;
    }

private:
    void drain() {
        for (int i; (i = next_.fetch_add(1)) < n_;) (*job_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            drain();
            {
                std::lock_guard<std::mutex> g(mu_);
                --pending_;
            }
            done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    int n_ = 0, pending_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// memcpy in pieces of at least 256 KB over the pool
void pool_memcpy(HostPool* pool, void* dst, const void* src, size_t bytes) {
    const size_t piece = 256 << 10;
    const int parts = pool ? (int)std::min<size_t>((size_t)pool->workers() + 1, (bytes + piece - 1) / piece) : 1;
    if (parts <= 1) {
        memcpy(dst, src, bytes);
        return;
    }
    const size_t step = ((bytes + parts - 1) / parts + 4095) & ~(size_t)4095;
    pool->run(parts, [&](int i) {
        const size_t a = (size_t)i * step;
        if (a < bytes) memcpy((char*)dst + a, (const char*)src + a, std::min(step, bytes - a));
    });
}

}  // namespace

struct foto_gn_plan {
    int w = 0, h = 0, maxiter = 0, device = 0;
    double alpha = 0, lam = 0, rtol = 0;
    hipStream_t s = nullptr;
    double* base = nullptr;
    double *d1 = nullptr, *d2 = nullptr, *fx = nullptr, *fy = nullptr, *ft = nullptr, *b = nullptr, *x = nullptr,
           *r = nullptr, *z = nullptr, *p0 = nullptr, *p1 = nullptr;
    double *rr_part = nullptr, *pq_part = nullptr, *rz_part[2] = {nullptr, nullptr};
    double *r2 = nullptr, *q = nullptr, *rr_part2 = nullptr;   // the folded update (fold)
    bool recomp = true;              // level-0 legs form B, D^-1 from fx, fy, f2 (FOTO_GN_RECOMP=0: load them)
    bool exact_tail = true;          // launch the predicted count exactly (FOTO_GN_EXACT=0: whole graphs)
    bool setup_fuse = true;          // B and block inverses per level in one pass (FOTO_GN_SETUP_FUSE=0: not)
    bool fold = true;                // k_gnp_upd folded into the level-0 down leg (FOTO_GN_FOLD=0: not)
    size_t pt_l0 = 0;                // first level of the persistent small-level launch (0: none; FOTO_MG_PTAIL=1: on)
    bool lt = false;                 // the last level + coarsest in one LDS-resident block (k_mg_ltail)
    int graph_its = 4;               // PCG iterations per graph replay (FOTO_GN_GRAPH, even)
    unsigned* pt_counter = nullptr;  // its grid-barrier arrivals (zeroed per solve)
    int nb_pix = 0, nb_rz = 0;
    CGScal* dS = nullptr;
    CGScal* hS = nullptr;
    double* hbuf_dev = nullptr;   // hbuf as the device sees it (kernels write u, v, m there)
    double* hbuf = nullptr;   // pinned staging: f1, f2, u, v, m (pageable copies of ~2.5 MB were
                              // pinned on the fly by the runtime: 15-25 ms per solve at 640x480)
    struct Lev {
        int w = 0, h = 0;
        double s[3] = {0, 0, 0};
        double *B = nullptr, *Dinv = nullptr, *f = nullptr, *x = nullptr, *y = nullptr;
    };
    std::vector<Lev> lev;
    hipGraph_t graph = nullptr;
    hipGraphExec_t gexec = nullptr;
    hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
    hipEvent_t dl_ev[3] = {nullptr, nullptr, nullptr};   // u, v, m downloaded (the copy-out of one overlaps the next)
    std::unique_ptr<HostPool> pool;                        // host copies (made with the staging)
    int last_its = 0;
    double last[4] = {0, 0, 0, 0};   // ms setup+upload, ms PCG, iterations, iterations launched
    bool tail = false;               // small levels in one block (k_mg_tail, FOTO_MG_TAIL=1; measured slower)

    MGLev desc(size_t l) const {
        const Lev& L = lev[l];
        return MGLev{L.w, L.h, L.s[0], L.s[1], L.s[2], L.B, L.Dinv};
    }
    ~foto_gn_plan() {
        if (s) (void)hipStreamSynchronize(s);
        if (gexec) (void)hipGraphExecDestroy(gexec);
        if (graph) (void)hipGraphDestroy(graph);
        for (auto e : ev) if (e) (void)hipEventDestroy(e);
        for (auto e : dl_ev) if (e) (void)hipEventDestroy(e);
        pool.reset();
        if (base) (void)hipFree(base);
        if (hS) (void)hipHostFree(hS);
        if (hbuf) (void)hipHostFree(hbuf);
        stream_release(s);
    }
};

namespace foto {

// one thread per cell of the coarsest level, whole waves (fewer waves: cheaper barriers
// between the sweeps)
static int mg_coarse_threads(const foto_gn_plan::Lev& L) {
    const int n = L.w * L.h;
    const int per = (n + MG_CPT - 1) / MG_CPT;   // (MG_COARSE <= 1024: one cell per thread)
    return std::min(1024, ((per + 63) / 64) * 64);
}

// z = V(r) and the partials of r.z -> rz_out
// level 0's legs: B and D^-1 formed from the GN coefficients (P->recomp) or loaded
static void mg_down0(foto_gn_plan* P, int wc, int hc, double* x, double* fc, const MGUpd& upd) {
    const auto& L = P->lev[0];
    if (P->recomp)
        k_mg_down2<true, true><<<mg_tiles(L.w, L.h), NT, 0, P->s>>>(P->desc(0), wc, hc, P->dS, nullptr, x, fc, upd);
    else
        k_mg_down2<true, false><<<mg_tiles(L.w, L.h), NT, 0, P->s>>>(P->desc(0), wc, hc, P->dS, nullptr, x, fc, upd);
}

static void mg_up0(foto_gn_plan* P, int wc, int hc, const double* e, const double* r, const double* x, double* z,
                   double* rz_out) {
    const auto& L = P->lev[0];
    if (P->recomp)
        k_mg_up2<true, true><<<mg_tiles(L.w, L.h), NT, 0, P->s>>>(P->desc(0), wc, hc, P->dS, e, r, x, z, rz_out,
                                                                 MGCoef{P->fx, P->fy, P->d2});
    else
        k_mg_up2<true, false><<<mg_tiles(L.w, L.h), NT, 0, P->s>>>(P->desc(0), wc, hc, P->dS, e, r, x, z, rz_out);
}

static int gn_vcycle(foto_gn_plan* P, const double* r, double* z, double* rz_out, const MGUpd* upd = nullptr) {
    hipStream_t s = P->s;
    const size_t nl = P->lev.size();
    if (nl == 1) {
        k_mg_coarse<true><<<1, mg_coarse_threads(P->lev[0]), 0, s>>>(P->desc(0), P->dS, r, z, rz_out);
        FOTO_HIP_CHECK(hipGetLastError());
        return 0;
    }
    // the tail: the first level l0 >= 1 from which every level has at most MG_TAIL_CELLS cells
    size_t l0 = nl;
    if (P->tail) {
        for (size_t l = 1; l < nl; ++l)
            if ((int64_t)P->lev[l].w * P->lev[l].h <= MG_TAIL_CELLS && nl - l <= (size_t)MG_TAIL_MAX) { l0 = l; break; }
    }
    if (P->pt_l0 > 0) l0 = P->pt_l0;   // (the persistent launch replaces the one-block tail)
    if (P->lt) {   // level c - 1 and the coarsest in one block: the level kernels above and below it
        const size_t c = nl - 1;
        for (size_t l = 0; l + 1 < c; ++l) {
            const auto& L = P->lev[l];
            const auto& C = P->lev[l + 1];
            if (l == 0 && upd)
                mg_down0(P, C.w, C.h, L.x, C.f, *upd);
            else
                k_mg_down2<false><<<mg_tiles(L.w, L.h), NT, 0, s>>>(P->desc(l), C.w, C.h, P->dS, l == 0 ? r : L.f, L.x,
                                                                   C.f, MGUpd{});
            FOTO_HIP_CHECK(hipGetLastError());
        }
        const auto& L = P->lev[c - 1];
        const auto& C = P->lev[c];
        k_mg_ltail<<<1, MG_LT_NTH, mg_lt_lds(L.w * L.h, C.w * C.h) * sizeof(double), s>>>(P->desc(c - 1), P->desc(c),
                                                                                          P->dS, L.f, L.y);
        FOTO_HIP_CHECK(hipGetLastError());
        const double* e = L.y;
        for (size_t l = c - 1; l-- > 0;) {
            const auto& Lu = P->lev[l];
            const auto& Cu = P->lev[l + 1];
            if (l == 0) {
                mg_up0(P, Cu.w, Cu.h, e, r, Lu.x, z, rz_out);
            } else {
                k_mg_up2<false><<<mg_tiles(Lu.w, Lu.h), NT, 0, s>>>(P->desc(l), Cu.w, Cu.h, P->dS, e, Lu.f, Lu.x, Lu.y,
                                                                    nullptr);
                e = Lu.y;
            }
            FOTO_HIP_CHECK(hipGetLastError());
        }
        return 0;
    }
    const size_t ldown = std::min(l0, nl - 1);
    for (size_t l = 0; l < ldown; ++l) {
        const auto& L = P->lev[l];
        const auto& C = P->lev[l + 1];
        if (l == 0 && upd)
            mg_down0(P, C.w, C.h, L.x, C.f, *upd);
        else
            k_mg_down2<false><<<mg_tiles(L.w, L.h), NT, 0, s>>>(P->desc(l), C.w, C.h, P->dS, l == 0 ? r : L.f, L.x,
                                                               C.f, MGUpd{});
        FOTO_HIP_CHECK(hipGetLastError());
    }
    const size_t c = nl - 1;
    const double* e = nullptr;
    size_t lup = nl - 1;   // up legs below this level run as level kernels
    if (P->pt_l0 > 0) {
        MGPTail T{};
        T.nl = (int)(nl - l0);
        for (size_t l = l0; l < nl; ++l) {
            T.L[l - l0] = P->desc(l);
            T.f[l - l0] = P->lev[l].f;
            T.x[l - l0] = P->lev[l].x;
            T.y[l - l0] = P->lev[l].y;
        }
        T.counter = P->pt_counter;
        T.syncs = 2 * (T.nl - 1);   // a barrier after each down leg, the coarsest solve, each up leg but the last
        k_mg_ptail<<<mg_tiles(P->lev[l0].w, P->lev[l0].h), NT, 0, s>>>(T, P->dS);
        FOTO_HIP_CHECK(hipGetLastError());
        e = P->lev[l0].y;
        lup = l0;
    } else if (l0 < nl) {
        MGTail T{};
        T.nl = (int)(nl - l0);
        for (size_t l = l0; l < nl; ++l) {
            T.L[l - l0] = P->desc(l);
            T.f[l - l0] = P->lev[l].f;
            T.x[l - l0] = P->lev[l].x;
            T.y[l - l0] = P->lev[l].y;
        }
        k_mg_tail<<<1, 1024, 0, s>>>(T, P->dS);
        FOTO_HIP_CHECK(hipGetLastError());
        e = (l0 == c) ? P->lev[c].x : P->lev[l0].y;
        lup = l0;
    } else {
        k_mg_coarse<false><<<1, mg_coarse_threads(P->lev[c]), 0, s>>>(P->desc(c), P->dS, P->lev[c].f, P->lev[c].x,
                                                                      nullptr);
        FOTO_HIP_CHECK(hipGetLastError());
        e = P->lev[c].x;
    }
    for (size_t l = lup; l-- > 0;) {
        const auto& L = P->lev[l];
        const auto& C = P->lev[l + 1];
        if (l == 0) {
            mg_up0(P, C.w, C.h, e, r, L.x, z, rz_out);
        } else {
            k_mg_up2<false><<<mg_tiles(L.w, L.h), NT, 0, s>>>(P->desc(l), C.w, C.h, P->dS, e, L.f, L.x, L.y, nullptr);
            e = L.y;
        }
        FOTO_HIP_CHECK(hipGetLastError());
    }
    return 0;
}

// PCG iteration of parity `par` (k even: p0 -> p1, z_k's r.z in rz_part[0]; folded update: r in
// r, then r2 -> r by parity too)
static int gn_iteration(foto_gn_plan* P, int par) {
    const int w = P->w, h = P->h;
    double* po = par ? P->p1 : P->p0;
    double* pn = par ? P->p0 : P->p1;
    const double* rzc = P->rz_part[par];
    const double* rzp = P->rz_part[par ^ 1];
    k_gnp_dir<<<P->nb_pix, NT, 0, P->s>>>(w, h, P->fx, P->fy, P->d2, P->alpha, P->lam, P->z, po, pn, P->dS,
                                           P->rr_part, P->nb_pix, rzc, rzp, P->nb_rz, P->pq_part, P->rtol,
                                           P->fold ? P->q : nullptr, P->fold ? P->rr_part2 : nullptr, P->nb_rz);
    FOTO_HIP_CHECK(hipGetLastError());
    if (P->fold) {
        double* rold = par ? P->r2 : P->r;
        double* rnew = par ? P->r : P->r2;
        const MGUpd U{rold, rnew, P->q, pn, P->x, rzc, P->pq_part, P->rr_part2, P->dS, P->nb_rz, P->nb_pix,
                      MGCoef{P->fx, P->fy, P->d2}};
        return gn_vcycle(P, rnew, P->z, P->rz_part[par ^ 1], &U);
    }
    k_gnp_upd<<<P->nb_pix, NT, 0, P->s>>>(w, h, P->fx, P->fy, P->d2, P->alpha, P->lam, pn, P->x, P->r, P->dS, rzc,
                                           P->nb_rz, P->pq_part, P->nb_pix, P->rr_part);
    FOTO_HIP_CHECK(hipGetLastError());
    return gn_vcycle(P, P->r, P->z, P->rz_part[par ^ 1]);
}

// FOTO_GN_TRACE=1: wall time of each plan-creation phase on stderr (first-call cost studies)
struct GnTrace {
    bool on;
    std::chrono::steady_clock::time_point t0;
    GnTrace() : on(getenv("FOTO_GN_TRACE") != nullptr), t0(std::chrono::steady_clock::now()) {}
    void mark(const char* what) {
        if (!on) return;
        const auto t = std::chrono::steady_clock::now();
        fprintf(stderr, "[gn plan] %-22s %8.3f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
        t0 = t;
    }
};

static int gn_plan_init(foto_gn_plan* P) {
    const int w = P->w, h = P->h;
    const size_t n = (size_t)w * h;
    GnTrace tr;
    FOTO_HIP_CHECK(hipGetDevice(&P->device));
    FOTO_TRY(stream_acquire(&P->s));   // (pooled: a new stream cost ~10 ms)
    tr.mark("stream");
    for (auto& e : P->ev) FOTO_HIP_CHECK(hipEventCreate(&e));
    for (auto& e : P->dl_ev) FOTO_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    tr.mark("events");
    FOTO_HIP_CHECK(hipHostMalloc((void**)&P->hS, sizeof(CGScal)));
    tr.mark("pinned scalars");   // (the pinned staging is made during the first solve: gn_staging)
    P->nb_pix = flat_blocks((int64_t)n);
    {
        const char* e = getenv("FOTO_MG_TAIL");
        P->tail = e && atoi(e) != 0 && MG_COARSE <= 1024;   // (k_mg_tail: one coarsest cell per thread)
    }
    // level geometry
    int lw = w, lh = h;
    double sc = 1.0;
    size_t lev_total = 0;
    for (;;) {
        foto_gn_plan::Lev L;
        L.w = lw; L.h = lh;
        L.s[0] = P->alpha * sc; L.s[1] = P->alpha * sc; L.s[2] = P->lam * sc;
        lev_total += 21 * (size_t)lw * lh;
        P->lev.push_back(L);
        if ((int64_t)lw * lh <= MG_COARSE) break;
        lw = (lw + 1) / 2;
        lh = (lh + 1) / 2;
        sc *= 0.25;
    }
    P->nb_rz = P->lev.size() == 1 ? 1 : mg_tiles(w, h);
    {
        const char* sf = getenv("FOTO_GN_SETUP_FUSE");
        P->setup_fuse = !(sf && atoi(sf) == 0);
        const char* rc = getenv("FOTO_GN_RECOMP");
        P->recomp = !(rc && atoi(rc) == 0);
        const char* ex = getenv("FOTO_GN_EXACT");
        P->exact_tail = !(ex && atoi(ex) == 0);
        const char* e = getenv("FOTO_GN_FOLD");
        P->fold = P->lev.size() > 1 && !(e && atoi(e) == 0);   // (one level: no down leg to fold into)
    }
    const size_t nscal = sizeof(CGScal) / sizeof(double) + 1;
    const size_t nfold = P->fold ? 6 * n + (size_t)P->nb_rz : 0;
    const size_t total = 23 * n + lev_total + 2 * (size_t)P->nb_pix + 2 * (size_t)P->nb_rz + nfold + nscal + 64;
    FOTO_HIP_CHECK(hipMalloc((void**)&P->base, total * sizeof(double)));
    tr.mark("device buffers");
    double* q = P->base;
    P->d1 = q; q += n; P->d2 = q; q += n; P->fx = q; q += n; P->fy = q; q += n; P->ft = q; q += n;
    P->b = q; q += 3 * n; P->x = q; q += 3 * n; P->r = q; q += 3 * n; P->z = q; q += 3 * n;
    P->p0 = q; q += 3 * n; P->p1 = q; q += 3 * n;
    for (auto& L : P->lev) {
        const size_t m = (size_t)L.w * L.h;
        L.B = q; q += 6 * m; L.Dinv = q; q += 6 * m; L.f = q; q += 3 * m; L.x = q; q += 3 * m; L.y = q; q += 3 * m;
    }
    P->rr_part = q; q += P->nb_pix;
    P->pq_part = q; q += P->nb_pix;
    P->rz_part[0] = q; q += P->nb_rz;
    P->rz_part[1] = q; q += P->nb_rz;
    if (P->fold) {
        P->r2 = q; q += 3 * n;
        P->q = q; q += 3 * n;
        P->rr_part2 = q; q += P->nb_rz;
    }
    P->dS = (CGScal*)q;
    q += nscal;
    P->pt_counter = (unsigned*)q;   // (within total's slack)
    {   // the persistent small-level launch: from the first level of at most MG_PT_TILES tiles
        const char* e = getenv("FOTO_MG_PTAIL");
        const size_t nl = P->lev.size();
        if (e && atoi(e) != 0 && !P->tail)   // (opt-in: measured slower, see k_mg_ptail)
            for (size_t l = 1; l + 1 < nl; ++l)
                if (mg_tiles(P->lev[l].w, P->lev[l].h) <= MG_PT_TILES) {
                    if (nl - l <= (size_t)MG_PT_MAX) P->pt_l0 = l;
                    break;
                }
    }
    {   // the last level above the coarsest and the coarsest in LDS (FOTO_MG_LTAIL=0: level kernels)
        const char* e = getenv("FOTO_MG_LTAIL");
        const size_t nl = P->lev.size();
        if (!(e && atoi(e) == 0) && !P->tail && P->pt_l0 == 0 && nl >= 3 &&
            (int64_t)P->lev[nl - 2].w * P->lev[nl - 2].h <= MG_LT_CELLS &&
            (int64_t)P->lev[nl - 1].w * P->lev[nl - 1].h <= MG_LT_NTH) {
            P->lt = true;
            const size_t bytes = mg_lt_lds(P->lev[nl - 2].w * P->lev[nl - 2].h, P->lev[nl - 1].w * P->lev[nl - 1].h) *
                                 sizeof(double);
            FOTO_HIP_CHECK(hipFuncSetAttribute((const void*)k_mg_ltail, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)bytes));
        }
    }
    // P->graph_its iterations (p0 -> p1 -> p0 ...) captured once; the kernels read the iteration
    // index from the device, so the graph is replayed unchanged.  Round 5: 4 instead of 2 -- a
    // replay boundary cost ~17 us of idle GPU (profiles/r05_gn_trace.txt: 8.4 us per iteration
    // before k_gnp_dir), and a reused plan launches its predicted count in one go either way
    {
        const char* e = getenv("FOTO_GN_GRAPH");
        const int g = e ? atoi(e) : 4;
        P->graph_its = (g >= 2 && g <= 16 && g % 2 == 0) ? g : 4;
    }
    FOTO_HIP_CHECK(hipStreamBeginCapture(P->s, hipStreamCaptureModeThreadLocal));
    int c2 = 0;
    for (int it = 0; it < P->graph_its && c2 >= 0; ++it) c2 = gn_iteration(P, it & 1);
    const hipError_t ec = hipStreamEndCapture(P->s, &P->graph);
    FOTO_TRY(c2);
    FOTO_HIP_CHECK(ec);
    tr.mark("graph capture");
    FOTO_HIP_CHECK(hipGraphInstantiate(&P->gexec, P->graph, nullptr, nullptr, 0));
    tr.mark("graph instantiate");
    return 0;
}

// The pinned staging (f1, f2 up; u, v, m down), made while the first solve's iterations run:
// pinning 12 MB took ~3 ms at 640x480, a third of a first call (FOTO_GN_TRACE); that solve
// uploads from the caller's pageable arrays instead.
static int gn_staging(foto_gn_plan* P) {
    if (P->hbuf) return 0;
    const size_t n = (size_t)P->w * P->h;
    FOTO_HIP_CHECK(hipHostMalloc((void**)&P->hbuf, 5 * n * sizeof(double)));
    memset(P->hbuf, 0, 5 * n * sizeof(double));   // first touch on the host, not by the device
    FOTO_HIP_CHECK(hipHostGetDevicePointer((void**)&P->hbuf_dev, P->hbuf, 0));
    const char* e = getenv("FOTO_GN_HOST_THREADS");
    const int workers = e ? std::max(0, std::min(16, atoi(e))) : 4;
    if (workers > 0) P->pool = std::make_unique<HostPool>(workers);
    return 0;
}

static int gn_plan_solve(foto_gn_plan* P, const double* f1, const double* f2, double* u, double* v, double* m,
                         int* iterations) {
    const int w = P->w, h = P->h;
    const int64_t n = (int64_t)w * h;
    hipStream_t s = P->s;
    GnTrace tr;
    FOTO_HIP_CHECK(hipEventRecord(P->ev[0], s));
    if (P->hbuf) {
        double* hb = P->hbuf;
        pool_memcpy(P->pool.get(), hb, f1, n * sizeof(double));
        FOTO_HIP_CHECK(hipMemcpyAsync(P->d1, hb, n * sizeof(double), hipMemcpyHostToDevice, s));
        pool_memcpy(P->pool.get(), hb + n, f2, n * sizeof(double));
        FOTO_HIP_CHECK(hipMemcpyAsync(P->d2, hb + n, n * sizeof(double), hipMemcpyHostToDevice, s));
    } else {   // first solve of the plan (gn_staging)
        FOTO_HIP_CHECK(hipMemcpyAsync(P->d1, f1, n * sizeof(double), hipMemcpyHostToDevice, s));
        FOTO_HIP_CHECK(hipMemcpyAsync(P->d2, f2, n * sizeof(double), hipMemcpyHostToDevice, s));
    }
    tr.mark("solve: upload staged");
    FOTO_HIP_CHECK(hipMemsetAsync(P->dS, 0, sizeof(CGScal), s));
    if (P->pt_l0 > 0) FOTO_HIP_CHECK(hipMemsetAsync(P->pt_counter, 0, sizeof(unsigned), s));
    FOTO_HIP_CHECK(hipMemsetAsync(P->x, 0, 3 * n * sizeof(double), s));
    FOTO_HIP_CHECK(launch_gn_coeffs(w, h, P->d1, P->d2, P->fx, P->fy, P->ft, s));
    FOTO_HIP_CHECK(launch_gn_rhs(w, h, P->fx, P->fy, P->d2, P->ft, P->b, s));
    // image-dependent multigrid coefficients
    if (P->setup_fuse) {
        k_mg_b0_d<<<flat_blocks(n), NT, 0, s>>>(P->desc(0), P->fx, P->fy, P->d2, P->lev[0].B, P->lev[0].Dinv);
        FOTO_HIP_CHECK(hipGetLastError());
        for (size_t l = 1; l < P->lev.size(); ++l) {
            const auto& L = P->lev[l - 1];
            const auto& C = P->lev[l];
            k_mg_coarsen_d<<<flat_blocks((int64_t)C.w * C.h), NT, 0, s>>>(L.w, L.h, L.B, P->desc(l), C.B, C.Dinv);
            FOTO_HIP_CHECK(hipGetLastError());
        }
    } else {
        k_mg_b0<<<flat_blocks(n), NT, 0, s>>>(n, P->fx, P->fy, P->d2, P->lev[0].B);
        FOTO_HIP_CHECK(hipGetLastError());
        for (size_t l = 1; l < P->lev.size(); ++l) {
            const auto& L = P->lev[l - 1];
            const auto& C = P->lev[l];
            k_mg_coarsen<<<flat_blocks((int64_t)C.w * C.h), NT, 0, s>>>(L.w, L.h, L.B, C.w, C.h, C.B);
            FOTO_HIP_CHECK(hipGetLastError());
        }
        for (size_t l = 0; l < P->lev.size(); ++l) {
            k_mg_dinv<<<flat_blocks((int64_t)P->lev[l].w * P->lev[l].h), NT, 0, s>>>(P->desc(l), P->lev[l].Dinv);
            FOTO_HIP_CHECK(hipGetLastError());
        }
    }
    // r = b, r.r; z_0 = V(r), r.z -> rz_part[0]
    k_gnp_init<<<P->nb_pix, NT, 0, s>>>(n, P->b, P->r, P->rr_part);
    FOTO_HIP_CHECK(hipGetLastError());
    FOTO_TRY(gn_vcycle(P, P->r, P->z, P->rz_part[0]));
    FOTO_HIP_CHECK(hipEventRecord(P->ev[1], s));
    tr.mark("solve: setup enqueued");
    // replay the graph (G = graph_its iterations); the first wait comes after the previous solve's
    // count: the top-of-iteration test that ends a solve of `its` iterations runs in iteration
    // its, so its + 1 iterations are launched (rounded up to whole graphs)
    int k = 0;
    bool done = false;
    const int maxiter = P->maxiter;
    const int G = P->graph_its;
    const int first = P->last_its > 0 ? ((P->last_its + 1 + G - 1) / G) * G : 16;
    // (round 6: a reused plan launches exactly its predicted its + 1, the remainder past whole
    // graphs as single iterations -- a graph's surplus iterations each cost ~25 us of early exits)
    const int first_exact = P->last_its > 0 ? P->last_its + 1 : 16;
    while (k < maxiter) {
        const int chunk = std::min(k == 0 ? (P->exact_tail ? first_exact : first) : G, maxiter - k);
        int j = 0;
        if ((k & 1) && chunk > 0) {   // (after an under-predicted exact count: the graph starts on parity 0)
            FOTO_TRY(gn_iteration(P, 1));
            ++j;
            ++k;
        }
        for (; j + G <= chunk; j += G, k += G) FOTO_HIP_CHECK(hipGraphLaunch(P->gexec, s));
        for (; j < chunk; ++j, ++k) FOTO_TRY(gn_iteration(P, k & 1));   // (the remainder, outside the graph)
        FOTO_HIP_CHECK(hipMemcpyAsync(P->hS, P->dS, sizeof(CGScal), hipMemcpyDeviceToHost, s));
        if (k == chunk) FOTO_TRY(gn_staging(P));   // while the first iterations run
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        if (P->hS->done) { done = true; break; }
    }
    FOTO_HIP_CHECK(hipEventRecord(P->ev[2], s));
    tr.mark("solve: PCG done");
    if (P->hS->pad[1]) {   // (k_mg_ptail: a grid barrier gave up -- blocks not co-resident)
        set_error("GN: the persistent small-level launch could not synchronise its blocks (FOTO_MG_PTAIL=0 avoids it)");
        return FOTO_ERR_HIP;
    }
    // the solution straight into the mapped pinned staging by a kernel: the first large
    // device-to-host hipMemcpy of a process took 8.5-14.8 ms at 640x480 (0.15-0.4 ms later)
    FOTO_TRY(gn_staging(P));   // (maxiter 0: no iteration ran)
    // u, v, m one after the other, each copied out while the next crosses PCIe
    double* const outs[3] = {u, v, m};
    for (int c = 0; c < 3; ++c) {
        k_gn_download<<<flat_blocks(n), NT, 0, s>>>(n, P->x + c * n, P->hbuf_dev + (2 + c) * n);
        FOTO_HIP_CHECK(hipGetLastError());
        FOTO_HIP_CHECK(hipEventRecord(P->dl_ev[c], s));
    }
    for (int c = 0; c < 3; ++c) {
        FOTO_HIP_CHECK(hipEventSynchronize(P->dl_ev[c]));
        if (c == 0) tr.mark("solve: download u");
        pool_memcpy(P->pool.get(), outs[c], P->hbuf + (2 + c) * n, n * sizeof(double));
    }
    tr.mark("solve: copy out");
    const int its = done ? P->hS->iters : maxiter;
    float t0 = 0.f, t1 = 0.f;
    FOTO_HIP_CHECK(hipEventElapsedTime(&t0, P->ev[0], P->ev[1]));
    FOTO_HIP_CHECK(hipEventElapsedTime(&t1, P->ev[1], P->ev[2]));
    P->last[0] = t0; P->last[1] = t1; P->last[2] = its; P->last[3] = k;
    P->last_its = done ? its : 0;
    if (iterations) *iterations = its;
    return done ? 0 : maxiter;
}

}  // namespace foto

extern "C" {

int foto_gn_plan_create(int w, int h, double alpha, double lambda_, double rtol, int maxiter, foto_gn_plan** out) {
    if (!out) { set_error("null argument"); return FOTO_ERR_ARG; }
    if (w < 2 || h < 2) { set_error("w = %d, h = %d: GN needs >= 2 pixels per axis", w, h); return FOTO_ERR_ARG; }
    if (!(alpha > 0) || !(lambda_ > 0)) {
        set_error("GN needs alpha > 0 and lambda > 0 (the block-Jacobi smoother divides by them)");
        return FOTO_ERR_ARG;
    }
    if (maxiter < 0) { set_error("maxiter < 0"); return FOTO_ERR_ARG; }
    auto P = std::make_unique<foto_gn_plan>();
    P->w = w; P->h = h; P->alpha = alpha; P->lam = lambda_; P->rtol = rtol; P->maxiter = maxiter;
    FOTO_TRY(gn_plan_init(P.get()));
    *out = P.release();
    return 0;
}

int foto_gn_plan_solve(foto_gn_plan* p, const double* f1, const double* f2, double* u, double* v, double* m,
                       int* iterations) {
    if (!p || !f1 || !f2 || !u || !v || !m) { set_error("null argument"); return FOTO_ERR_ARG; }
    return gn_plan_solve(p, f1, f2, u, v, m, iterations);
}

int foto_gn_plan_timing(const foto_gn_plan* p, double* out4) {
    if (!p || !out4) { set_error("null argument"); return FOTO_ERR_ARG; }
    for (int k = 0; k < 4; ++k) out4[k] = p->last[k];
    return 0;
}

int foto_gn_plan_device(const foto_gn_plan* p) { return p ? p->device : -1; }

void foto_gn_plan_destroy(foto_gn_plan* p) { delete p; }

}  // extern "C"
