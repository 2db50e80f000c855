// libfoto: Gennert-Negahdaripour variational baseline (classical.GLLOpticalFlow,
// classical.py:25-130) on gfx950.
//
// The reference assembles a 3wh x 3wh sparse SPD system
//   [[-a L + fx^2, fx fy, -fx f2], [fy fx, -a L + fy^2, -fy f2], [-f2 fx, -f2 fy, -l L + f2^2]]
// (L = 5-point Neumann Laplacian = -G^T G with G = grad_forward) and solves it with SuperLU.
// Here the operator is applied matrix-free (one thread per pixel, all three fields) and
// solved with block-Jacobi preconditioned CG (the per-pixel 3x3 block D + v v^T,
// v = (fx, fy, -f2), inverted in registers by Sherman-Morrison), driven on the device
// with the same last-block reductions as the BB CG.
#include "foto_internal.h"

#include <algorithm>

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
__global__ __launch_bounds__(NT) void k_gn_pcg_dir(int w, int h, int k, const double* __restrict__ fx,
                                                   const double* __restrict__ fy, const double* __restrict__ f2,
                                                   double a, double l, const double* __restrict__ z,
                                                   const double* __restrict__ po, double* __restrict__ pn, CGScal* S,
                                                   RedBuf rb, const double* __restrict__ gath_rz,
                                                   double* __restrict__ gath_pq, double rtol) {
    if (S->done) return;
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

}  // namespace foto
