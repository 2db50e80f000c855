// Spectral CG for the stepA Poisson solve (benamou_brenier.py:85) -- gfx950.
//
// A = -r L_st + r eps I with the Neumann lap1d stencils of operators.py:95-110 is
// diagonalised exactly by the orthonormal DCT-II along each axis:
//     A = C^T diag(lam) C,  C = Ct (x) Cy (x) Cx,
//     lam(kt,ky,kx) = r eps + r (mu_t[kt] + mu_y[ky] + mu_x[kx]),  mu_n[k] = 2 - 2 cos(pi k / n).
// CG is basis-invariant: running scipy's CG recurrence on (diag(lam), C b) produces C x_k
// for the same x_k, the same residual norms, hence the same stopping iteration (up to
// rounding).  In that basis every CG iteration is pointwise, so one pass per iteration
// (Chronopoulos-Gear form: p.Ap from r.Ar, one fused reduction) reads and writes only r
// and p; x is recovered at the end as x = C^T ((b^ - r^) / lam).  The two vectors
// (2 x 78.6 MB at 640x480x32) stay resident in the 256 MiB Infinity Cache.
//
// The per-axis DCTs are GEMMs (n x n matrix applied along an axis) on f64 MFMA
// (v_mfma_f64_16x16x4_f64), 64x64x16 block tiles staged through LDS.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <vector>

#include "foto_spectral.h"
#include "foto_twiddles.h"

namespace foto {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Write-through 16-B stores (buffer_store_dwordx4 ... sc1): the line leaves the XCD's L2 at
// once instead of staying dirty there.  A streaming kernel that ends with its L2s full of
// dirty lines pays their write-back at the kernel boundary (MI355X_MICROARCH.md price list,
// row "boundary": + B / 6 TB/s for B dirty bytes, up to 32 MiB here).  The resource covers
// [base, base + 2^31 B); offsets are in bytes.
#ifndef FOTO_PASS_WT
#define FOTO_PASS_WT 1
#endif
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(double* base) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t rs, int off_bytes, dbl2 v) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, off_bytes, 0, 16 /* sc1 */);
}

// ============================================================================ reductions (local copies)

__device__ __forceinline__ double sp_wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    return v;
}

template <int K>
__device__ __forceinline__ void sp_block_sum(double (&v)[K], double* sh) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        v[k] = sp_wave_sum(v[k]);
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
__device__ bool sp_reduce_last(double (&v)[K], RedBuf rb, double (&tot)[K]) {
    __shared__ double sh[K * (NT / 64)];
    __shared__ int is_last;
    sp_block_sum<K>(v, sh);
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
    sp_block_sum<K>(acc, sh);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) tot[k] = acc[k];
        __hip_atomic_store(rb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// Variant for NTH-thread blocks and many quantities (the s-step pass, K = 48).  Measured on
// gfx950 (tools/s2_ablation.hip, 1024 blocks): the block sum is an LDS transpose (each
// thread writes CH of its values, CH x 16 threads sum 16-element segments, CH threads the
// 16 segment sums), CH = 16 quantities at a time, instead of K shuffle butterflies;
// partials are k-major ([k][block], so a wave's load covers 4 cache lines); the last block
// issues a chunk's loads before the first use (clamped block index, unconditional) -- one
// round trip per chunk instead of one per load.  Fixed summation order: deterministic.
// Compensated (TwoSum) accumulation: s + c carries the running sum to ~2^-100 relative,
// so the block sums are correctly rounded to within ~1 ulp.  The s-step plan's Gram-form
// inner products cancel by up to S_CLIM and need moments that accurate: with plain fp64
// trees the textured golden solve drifts to 1e-7 relative in crit, with compensated block
// sums to 1e-8 (prototype measurement; tests/test_sstep_plan.py).
__device__ __forceinline__ void two_sum_acc(double& s, double& c, double x) {
    const double t = s + x;
    const double bp = t - s;
    c += (s - (t - bp)) + (x - bp);
    s = t;
}

template <int CH, int NTH>
__device__ __forceinline__ void sp_blk_sum_lds(const double* v /* CH values of this thread */, double* red /* CH*NTH */,
                                               double* red2 /* 2*CH*16: sums | compensations */) {
    static_assert(NTH % 16 == 0 && CH * 16 <= NTH, "segment layout");
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < CH; ++k) red[k * NTH + tid] = v[k];
    __syncthreads();
    constexpr int SEG = NTH / 16;
    if (tid < CH * 16) {
        const double* a = red + (tid >> 4) * NTH + (tid & 15) * SEG;
        double s = a[0], c = 0.0;
#pragma unroll
        for (int j = 1; j < SEG; ++j) two_sum_acc(s, c, a[j]);
        red2[tid] = s;
        red2[CH * 16 + tid] = c;
    }
    __syncthreads();
}

// total of quantity k's 16 compensated segment sums, rounded once
template <int CH>
__device__ __forceinline__ double sp_seg_total(const double* red2, int k) {
    double s = red2[k * 16], c = red2[CH * 16 + k * 16];
#pragma unroll
    for (int j = 1; j < 16; ++j) {
        two_sum_acc(s, c, red2[k * 16 + j]);
        c += red2[CH * 16 + k * 16 + j];
    }
    return s + c;
}

// ---------------------------------------------------------------------------- reduce-scatter
// Wave-level sum of K per-lane values without LDS: at each xor level a lane keeps one half
// of its remaining values and adds the partner's copy of that half (the partner sends it),
// so the K values halve per level (48 -> 24 -> 12 -> 6 -> 3 over xor 32, 16, 8, 4) and the
// last levels butterfly the remainder.  Lane l ends with the wave totals of quantities
// rs_base(l) + j, j < rs_count<K>(); lanes differing only in the butterflied low bits hold
// identical values.  Every total is a pairwise tree over the 64 lanes: deterministic, and
// (measured in the s-step prototype) as accurate as compensated summation for the moments.
template <int K>
constexpr int rs_levels() {   // halving levels
    int c = K, l = 0;
    while (c % 2 == 0 && l < 6) { c /= 2; ++l; }
    return l;
}
template <int K>
constexpr int rs_count() { return K >> rs_levels<K>(); }

template <int C, int MASK>
__device__ __forceinline__ void rs_halve(double* v, int lane) {
    if constexpr (C % 2 == 0 && MASK >= 1) {
        const bool hi = (lane & MASK) != 0;
#pragma unroll
        for (int j = 0; j < C / 2; ++j) {
            if (j % 8 == 0) asm volatile("" ::: "memory");   // bound batched shuffles (registers)
            const double send = hi ? v[j] : v[C / 2 + j];
            const double keep = hi ? v[C / 2 + j] : v[j];
            v[j] = keep + __shfl_xor(send, MASK, 64);
        }
        rs_halve<C / 2, MASK / 2>(v, lane);
    } else if constexpr (MASK >= 1) {
#pragma unroll
        for (int j = 0; j < C; ++j) v[j] += __shfl_xor(v[j], MASK, 64);
        rs_halve<C, MASK / 2>(v, lane);
    }
}

template <int K>
__device__ __forceinline__ int rs_base(int lane) {
    int base = 0, c = K;
#pragma unroll
    for (int l = 0, mask = 32; l < rs_levels<K>(); ++l, mask >>= 1) {
        c /= 2;
        if (lane & mask) base += c;
    }
    return base;
}

// Block (NTH threads) sum of K values per thread into red[k] (shared, K): reduce-scatter per
// wave, then the waves' partials are added pairwise by K threads.  wred: shared, (NTH/64) * K.
template <int K, int NTH>
__device__ __forceinline__ void blk_sum_rs(double (&v)[K], double* wred, double* out /* shared K */) {
    constexpr int NW = NTH / 64, LEV = rs_levels<K>(), CNT = rs_count<K>();
    constexpr int LOWMASK = (LEV >= 6) ? 0 : ((32 >> (LEV > 0 ? LEV - 1 : 0)) - 1) & (LEV > 0 ? 63 : 63);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    rs_halve<K, 32>(v, lane);
    const int base = rs_base<K>(lane);
    const int low = (LEV == 0) ? 63 : ((32 >> (LEV - 1)) - 1);
    (void)LOWMASK;
    if ((lane & low) == 0) {
#pragma unroll
        for (int j = 0; j < CNT; ++j) wred[w * K + base + j] = v[j];
    }
    __syncthreads();
    if (threadIdx.x < K) {
        double a[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) a[i] = wred[i * K + threadIdx.x];
#pragma unroll
        for (int st = 1; st < NW; st *= 2)
#pragma unroll
            for (int i = 0; i + st < NW; i += 2 * st) a[i] += a[i + st];
        out[threadIdx.x] = a[0];
    }
    __syncthreads();
}

// Cross-block sum of K values per thread: block sums by reduce-scatter, k-major partials,
// agent-scope ticket; the last block gathers the partials with 16 threads per quantity
// (16 loads in flight each: one round trip for up to 256 blocks), pairwise throughout.
// With 256-thread blocks and 1024 blocks the gather was 14 us of each pass; with 1024-thread
// blocks (one per CU) and this layout of the loads it is ~3 us (tools/s2_ablation.hip).
template <int K, int NTH>
__device__ bool sp_reduce_last_rs(double (&v)[K], RedBuf rb, double* tot /* shared, K */) {
    constexpr int NW = NTH / 64;
    __shared__ double wred[NW * K];
    __shared__ double bsum[K];
    __shared__ int is_last;
    const int tid = threadIdx.x, nb = gridDim.x;
    blk_sum_rs<K, NTH>(v, wred, bsum);
    if (tid < K)
        __hip_atomic_store(&rb.partials[(int64_t)tid * nb + blockIdx.x], bsum[tid], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#if defined(FOTO_S2_ABLATE) && FOTO_S2_ABLATE == 5   // timing studies only: no ticket, no tail
    return false;
#endif
    if (tid < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // wave 0's stores drained before its ticket add
        if (tid == 0) {
            const unsigned t = __hip_atomic_fetch_add(rb.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            is_last = (t == (unsigned)(nb - 1));
        }
    }
    __syncthreads();
#if defined(FOTO_S2_ABLATE) && FOTO_S2_ABLATE == 6   // timing studies only: ticket, no tail
    if (is_last && tid == 0) __hip_atomic_store(rb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
#endif
    if (!is_last) return false;
    // Gather: thread t sums quantity t / 16 over the blocks b = t % 16 + 16 j (16 loads in
    // flight per round, pairwise), then the 16 lanes of a quantity combine by xor butterfly.
    // K * 16 threads per round of quantities (all 48 at once with 1024-thread blocks).
    constexpr int QPR = NTH / 16;   // quantities per round
#pragma unroll
    for (int c = 0; c < K; c += QPR) {
        const int k = c + (tid >> 4), sub = tid & 15;
        double x = 0.0;
        if (k < K) {
            for (int base = 0; base < nb; base += 256) {
                double y[16];
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const int b = min(base + sub + 16 * j, nb - 1);
                    y[j] = __hip_atomic_load(&rb.partials[(int64_t)k * nb + b], __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) y[j] = (base + sub + 16 * j < nb) ? y[j] : 0.0;
#pragma unroll
                for (int st = 1; st < 16; st *= 2)
#pragma unroll
                    for (int j = 0; j + st < 16; j += 2 * st) y[j] += y[j + st];
                x += y[0];
            }
        }
#pragma unroll
        for (int m = 8; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
        if (k < K && sub == 0) tot[k] = x;
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_store(rb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

constexpr int sp_chunk(int K) {   // largest divisor of K that is <= 16
    int c = K < 16 ? K : 16;
    while (K % c) --c;
    return c;
}

template <int K, int NTH>
__device__ bool sp_reduce_last_wide(double (&v)[K], RedBuf rb, double* tot /* shared, K */) {
    constexpr int CH = sp_chunk(K);
    static_assert(K % CH == 0, "whole chunks");
    __shared__ double red[CH * NTH];
    __shared__ double red2[2 * CH * 16];
    __shared__ int is_last;
    const int tid = threadIdx.x, nb = gridDim.x;
#pragma unroll
    for (int c = 0; c < K; c += CH) {
        sp_blk_sum_lds<CH, NTH>(v + c, red, red2);
        if (tid < CH)
            __hip_atomic_store(&rb.partials[(int64_t)(c + tid) * nb + blockIdx.x], sp_seg_total<CH>(red2, tid),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // wave 0's stores drained before its ticket add
        if (tid == 0) {
            const unsigned t = __hip_atomic_fetch_add(rb.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            is_last = (t == (unsigned)(nb - 1));
        }
    }
    __syncthreads();
    if (!is_last) return false;
    constexpr int RPT = 2;   // blocks per thread per round trip (register peak of the pass)
#pragma unroll
    for (int c = 0; c < K; c += CH) {
        double x[CH];
#pragma unroll
        for (int k = 0; k < CH; ++k) x[k] = 0.0;
        for (int base = 0; base < nb; base += RPT * NTH) {
            double y[RPT][CH];
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const int b = min(base + tid + j * NTH, nb - 1);
#pragma unroll
                for (int k = 0; k < CH; ++k)
                    y[j][k] = __hip_atomic_load(&rb.partials[(int64_t)(c + k) * nb + b], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const bool ok = base + tid + j * NTH < nb;
#pragma unroll
                for (int k = 0; k < CH; ++k) x[k] += ok ? y[j][k] : 0.0;
            }
        }
        __syncthreads();   // red / red2 reuse
        sp_blk_sum_lds<CH, NTH>(x, red, red2);
        if (tid < CH) tot[c + tid] = sp_seg_total<CH>(red2, tid);
    }
    __syncthreads();
    if (tid == 0) __hip_atomic_store(rb.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// ============================================================================ DCT along one axis (f64 MFMA GEMM)

constexpr int BM = 64, BN = 64, BK = 16;
constexpr int AS_LD = BK + 1;   // 17 doubles: column reads across 16 rows hit 16 distinct bank pairs
constexpr int BS_LD = BN + 16;  // 80 doubles = 160 dwords = 32 mod 64: the 4 k-rows of a read split the banks

// out[o][k][i] = sum_j M[k][j] in[o][j][i] over an array viewed as [outer][n][inner].
// CONTIG (inner == 1): GEMM rows = o, cols = k   (A = in rows, B = M^T)
// otherwise          : GEMM rows = k, cols = i, batch o = blockIdx.z (A = M, B = in[o])
template <bool CONTIG>
__global__ __launch_bounds__(256) void k_dct_axis(int outer, int n, int inner, const double* __restrict__ M,
                                                  const double* __restrict__ in, double* __restrict__ out) {
    __shared__ double As[BM * AS_LD];
    __shared__ double Bs[BK * BS_LD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    int row0, col0;
    const double* inb;
    double* outb;
    int nrows, ncols;
    if (CONTIG) {
        row0 = blockIdx.y * BM;   // o
        col0 = blockIdx.x * BN;   // k
        nrows = outer;
        ncols = n;
        inb = in;
        outb = out;
    } else {
        row0 = blockIdx.y * BM;   // k
        col0 = blockIdx.x * BN;   // i
        nrows = n;
        ncols = inner;
        inb = in + (int64_t)blockIdx.z * n * inner;
        outb = out + (int64_t)blockIdx.z * n * inner;
    }
    dbl4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};

    for (int j0 = 0; j0 < n; j0 += BK) {
        // ---- stage A (BM x BK) and B (BK x BN)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q;
            {   // A[m][kk]
                const int m = e >> 4, kk = e & 15;
                const int gr = row0 + m, gj = j0 + kk;
                double v = 0.0;
                if (gr < nrows && gj < n) v = CONTIG ? inb[(int64_t)gr * n + gj] : M[(int64_t)gr * n + gj];
                As[m * AS_LD + kk] = v;
            }
            if (CONTIG) {   // B[kk][c] = M[col0 + c][j0 + kk]
                const int c = e >> 4, kk = e & 15;
                const int gk = col0 + c, gj = j0 + kk;
                Bs[kk * BS_LD + c] = (gk < ncols && gj < n) ? M[(int64_t)gk * n + gj] : 0.0;
            } else {        // B[kk][c] = in[j0 + kk][col0 + c]
                const int kk = e >> 6, c = e & 63;
                const int gj = j0 + kk, gi = col0 + c;
                Bs[kk * BS_LD + c] = (gj < n && gi < ncols) ? inb[(int64_t)gj * inner + gi] : 0.0;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k4 = 0; k4 < BK / 4; ++k4) {
            const int kk = k4 * 4 + (lane >> 4);
            double a[2], b[2];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) a[mi] = As[(wm * 32 + mi * 16 + (lane & 15)) * AS_LD + kk];
#pragma unroll
            for (int ni = 0; ni < 2; ++ni) b[ni] = Bs[kk * BS_LD + wn * 32 + ni * 16 + (lane & 15)];
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
        __syncthreads();
    }
    // ---- store: D[row = (lane>>4) + 4 r][col = lane & 15]
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gr = row0 + wm * 32 + mi * 16 + (lane >> 4) + 4 * r;
                const int gc = col0 + wn * 32 + ni * 16 + (lane & 15);
                if (gr < nrows && gc < ncols) {
                    if (CONTIG) outb[(int64_t)gr * n + gc] = acc[mi][ni][r];
                    else outb[(int64_t)gr * inner + gc] = acc[mi][ni][r];
                }
            }
}

// Large-tile variant: BM x BN = 128 x 128 per 256-thread block, each wave a 64 x 64
// sub-tile (4 x 4 MFMA 16x16x4 accumulators), BK = 16.  The next K-step's A/B elements are
// loaded into registers before the current step's MFMAs and written to the other LDS
// buffer after them (one barrier per K-step): global latency overlaps the matrix work and
// the loaded bytes per MFMA are half those of the 64 x 64 kernel.
constexpr int LBM = 128, LBN = 128, LBK = 16;
constexpr int LAS = LBK + 1;      // A row stride (doubles)
constexpr int LBS = LBN + 16;     // B row stride: 144 doubles = 288 dwords = 32 mod 64

template <bool CONTIG>
__global__ __launch_bounds__(256) void k_dct_axis_l(int outer, int n, int inner, const double* __restrict__ M,
                                                    const double* __restrict__ in, double* __restrict__ out) {
    __shared__ double As[2][LBM * LAS];
    __shared__ double Bs[2][LBK * LBS];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wm = w >> 1, wn = w & 1;
    const int row0 = blockIdx.y * LBM, col0 = blockIdx.x * LBN;
    const int nrows = CONTIG ? outer : n;
    const int ncols = CONTIG ? n : inner;
    const double* inb = CONTIG ? in : in + (int64_t)blockIdx.z * n * inner;
    double* outb = CONTIG ? out : out + (int64_t)blockIdx.z * n * inner;

    // staging map: 2048 A and 2048 B elements per K-step, 8 + 8 per thread
    double ra[8], rb[8];
    auto gload = [&](int j0) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            {   // A[m][kk], m = e / 16
                const int m = e >> 4, kk = e & 15;
                const int gr = row0 + m, gj = j0 + kk;
                ra[q] = (gr < nrows && gj < n) ? (CONTIG ? inb[(int64_t)gr * n + gj] : M[(int64_t)gr * n + gj]) : 0.0;
            }
            if (CONTIG) {   // B[kk][c] = M[col0 + c][j0 + kk]
                const int c = e >> 4, kk = e & 15;
                const int gk = col0 + c, gj = j0 + kk;
                rb[q] = (gk < ncols && gj < n) ? M[(int64_t)gk * n + gj] : 0.0;
            } else {        // B[kk][c] = in[j0 + kk][col0 + c]
                const int kk = e >> 7, c = e & 127;
                const int gj = j0 + kk, gi = col0 + c;
                rb[q] = (gj < n && gi < ncols) ? inb[(int64_t)gj * inner + gi] : 0.0;
            }
        }
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int e = tid + 256 * q;
            As[buf][(e >> 4) * LAS + (e & 15)] = ra[q];
            if (CONTIG) Bs[buf][(e & 15) * LBS + (e >> 4)] = rb[q];
            else Bs[buf][(e >> 7) * LBS + (e & 127)] = rb[q];
        }
    };

    dbl4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};

    gload(0);
    lstore(0);
    __syncthreads();
    int buf = 0;
    for (int j0 = 0; j0 < n; j0 += LBK) {
        const bool more = j0 + LBK < n;
        if (more) gload(j0 + LBK);
#pragma unroll
        for (int k4 = 0; k4 < LBK / 4; ++k4) {
            const int kk = k4 * 4 + (lane >> 4);
            double a[4], b[4];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) a[mi] = As[buf][(wm * 64 + mi * 16 + (lane & 15)) * LAS + kk];
#pragma unroll
            for (int ni = 0; ni < 4; ++ni) b[ni] = Bs[buf][kk * LBS + wn * 64 + ni * 16 + (lane & 15)];
#pragma unroll
            for (int mi = 0; mi < 4; ++mi)
#pragma unroll
                for (int ni = 0; ni < 4; ++ni)
                    acc[mi][ni] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[mi], b[ni], acc[mi][ni], 0, 0, 0);
        }
        if (more) lstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gr = row0 + wm * 64 + mi * 16 + (lane >> 4) + 4 * r;
                const int gc = col0 + wn * 64 + ni * 16 + (lane & 15);
                if (gr < nrows && gc < ncols) {
                    if (CONTIG) outb[(int64_t)gr * n + gc] = acc[mi][ni][r];
                    else outb[(int64_t)gr * inner + gc] = acc[mi][ni][r];
                }
            }
}

static int g_dct_large = -1;   // FOTO_DCT_LARGE=0 selects the 64 x 64 kernel (A/B runs)

static hipError_t dct_axis(int outer, int n, int inner, const double* M, const double* in, double* out,
                           hipStream_t s) {
    if (g_dct_large < 0) {
        const char* e = getenv("FOTO_DCT_LARGE");
        g_dct_large = e ? atoi(e) : 1;
    }
    // the t-axis (n = Nt, small) keeps the 64 x 64 tile; x and y use 128 x 128
    const bool large = g_dct_large && n >= 96;
    if (inner == 1) {
        if (large) {
            dim3 grid((n + LBN - 1) / LBN, (outer + LBM - 1) / LBM, 1);
            k_dct_axis_l<true><<<grid, 256, 0, s>>>(outer, n, inner, M, in, out);
        } else {
            dim3 grid((n + BN - 1) / BN, (outer + BM - 1) / BM, 1);
            k_dct_axis<true><<<grid, 256, 0, s>>>(outer, n, inner, M, in, out);
        }
    } else {
        if (large) {
            dim3 grid((inner + LBN - 1) / LBN, (n + LBM - 1) / LBM, outer);
            k_dct_axis_l<false><<<grid, 256, 0, s>>>(outer, n, inner, M, in, out);
        } else {
            dim3 grid((inner + BN - 1) / BN, (n + BM - 1) / BM, outer);
            k_dct_axis<false><<<grid, 256, 0, s>>>(outer, n, inner, M, in, out);
        }
    }
    return hipGetLastError();
}

// ============================================================================ DCT along one axis (FFT)
//
// Orthonormal DCT-II (forward) / DCT-III (inverse) of real lines of even length N = 2M
// through a length-M complex DFT (Makhoul's reordering): v = (x0, x2, x4, ..., x5, x3, x1),
// z_j = v_2j + i v_2j+1, Z = DFT_M(z), then with C_k = conj Z_{(M-k) mod M}
//     V_k = (Z_k + C_k) / 2 + e^{-2 pi i k/N} (Z_k - C_k) / (2i)      (= DFT_N(v)_k)
//     Y_k = e^{-i pi k/(2N)} V_k,   X_k = s_k Re Y_k,   X_{N-k} = -s_{N-k} Im Y_k,
// s_0 = sqrt(1/N), s_k = sqrt(2/N).  The inverse runs the same steps backwards (V from X by
// Hermitian symmetry, Z_k = Ve_k + i Vo_k, z = IDFT_M(Z), x from v).  DFT_M is two-stage
// Cooley-Tukey, M = M1 M2: M2 DFTs of length M1 over the stride-M2 subsequences, twiddle
// e^{-2 pi i j2 k1 / M}, M1 DFTs of length M2; the small DFTs are direct with compile-time
// roots (foto_twiddles.h), so multiplications by 0 / +-1 fold away.  About 2 (M1 + M2) + 8
// fp64 FMA per element (75 at N = 640) instead of the GEMM's N; each axis pass reads and
// writes the volume once.  LPB lines per block are staged in LDS; transforms are in place
// within a line.  Lines are contiguous rows (CONTIG, the x axis) or strided columns (y, t)
// taken LPB consecutive columns at a time so global loads and stores stay coalesced.
//
// Per-axis table (fp64): WM[2M] = e^{-2 pi i p/M}, PA[2(M+1)] = e^{-2 pi i k/N},
// PB[2(M+1)] = e^{-i pi k/(2N)}, then s_0, s.

// LDS image of a line: complex element j (natural order, index M2 j1 + j2) at position
// j1 (M2 + 1) + j2 -- each M2-row padded by one complex, so stage 2 (one thread per row,
// lane stride M2 + 1 complex) is free of bank conflicts (unpadded, the stride is 2 M2
// doubles: 32-way conflicts at M2 = 16), while stage 1 still touches only its own
// positions (. (M2 + 1) + j2) and runs in place.
#ifndef FOTO_FFT_TW_LDS
#define FOTO_FFT_TW_LDS 0      // 1: stage-1 twiddles staged in LDS (costs lines per block; measured slower)
#endif
#ifndef FOTO_FFT_LPB_MAX
#define FOTO_FFT_LPB_MAX 64
#endif
#ifndef FOTO_FFT_LPB_CONTIG_MAX
#define FOTO_FFT_LPB_CONTIG_MAX 64   // contiguous (x-axis) lines per block cap (A/B builds)
#endif
#ifndef FOTO_FFT_SYM
#define FOTO_FFT_SYM 1         // odd prime-length codelets by symmetric pairs (0: direct codelets)
#endif
#ifndef FOTO_FFT_LPB_POW2
#define FOTO_FFT_LPB_POW2 1    // power-of-two line counts only (whole 128-B segments on strided axes)
#endif
// Loads of a pass's input that is dead after the pass (the DCT chain's intermediates, x^, b^
// in the x^ kernel) are non-temporal: the lines leave the caches first, so the pass's output
// and the next kernel's inputs keep them -- 1652-1660 -> 1667-1671 it/s, k_prox_rhs (after
// the inverse x-DCT) 170-172 -> 167 us (A/B, profiles/r04n_ab_nt_loads.txt).  0: plain loads.
#ifndef FOTO_NT_LD
#define FOTO_NT_LD 1
#endif
template <class V>
__device__ __forceinline__ V ld_dead(const V* p) {
#if FOTO_NT_LD
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// Strided (y-axis) lines get a slightly larger LDS budget: at N = 1024 a line image is 8448 B,
// so 64 KB held 4 lines (32-B row segments) and 68 KB holds 8 (64 B; still two blocks per CU)
#ifndef FOTO_FFT_LINE_THREADS
#define FOTO_FFT_LINE_THREADS 1   // contiguous lines: output rounds per thread group of one line (0: flat idx rounds)
#endif
#ifndef FOTO_FFT_TW_PT
#define FOTO_FFT_TW_PT 0       // 1: stage-1 twiddles from the LDS post-twiddle table (PT_LDS kernels; measured no faster)
#endif
#ifndef FOTO_FFT_PT_LDS
#define FOTO_FFT_PT_LDS 1      // 0: the pre / post twiddles read from the global table per element
#endif
#ifndef FOTO_FFT_STRIDED_LDS
#define FOTO_FFT_STRIDED_LDS 69632
#endif
template <int M1, int M2, bool CONTIG = true>
struct FftGeom {
    static constexpr int M = M1 * M2, N = 2 * M;
    static constexpr int LS = 2 * M1 * (M2 + 1);   // doubles per line in LDS
    // lines per block: LDS (lines + twiddles) <= 64 KB (contiguous lines) / FOTO_FFT_STRIDED_LDS
    static constexpr int lpb() {
        const int c[8] = {64, 32, 16, 12, 8, 4, 2, 1};
        const int budget = CONTIG ? 65536 : FOTO_FFT_STRIDED_LDS;
        for (int i = 0; i < 8; ++i)
            if (c[i] <= FOTO_FFT_LPB_MAX && (!CONTIG || M2 > 32 || c[i] <= FOTO_FFT_LPB_CONTIG_MAX) &&
                !(FOTO_FFT_LPB_POW2 && c[i] == 12) &&
                c[i] * LS * 8 + (FOTO_FFT_TW_LDS ? 16 * M : 0) <= budget)
                return c[i];
        return 1;
    }
    static constexpr int LPB = lpb();
    static constexpr int TAB = 6 * M + 6;
    // the output / input phase twiddles (PA, PB of the table: 4 doubles per k = 0 .. M) staged in
    // LDS when that keeps the blocks per CU the LDS allows (x at 640: 3 of 43 + 10 KB; y at 480: 2
    // of 65 + 8 KB; not y at 1024, whose 8 lines already take 66 KB)
    static constexpr int PTN = 4 * (M + 1);
    static constexpr int LDS_B = LPB * LS * 8 + 16;
    static constexpr bool PT_LDS = FOTO_FFT_PT_LDS && (163840 / (LDS_B + 8 * PTN)) == (163840 / LDS_B);
};

// PT[4k .. 4k + 3] = (PA_k, PB_k): e^{-2 pi i k / N}, e^{-i pi k / (2N)}
template <class G>
__device__ __forceinline__ void fft_pt_fill(double* PT, const double* __restrict__ tab) {
    if constexpr (G::PT_LDS) {
        const double* PA = tab + 2 * G::M;
        const double* PB = PA + 2 * (G::M + 1);
        for (int p = threadIdx.x; p < G::M + 1; p += blockDim.x) {
            const double a0 = PA[2 * p], a1 = PA[2 * p + 1], b0 = PB[2 * p], b1 = PB[2 * p + 1];
            PT[4 * p] = a0;
            PT[4 * p + 1] = a1;
            PT[4 * p + 2] = b0;
            PT[4 * p + 3] = b1;
        }
    }
}

template <int M2>
__device__ __forceinline__ int fft_zpos(int j) { return j + j / M2; }   // natural index -> LDS complex position

template <int R, bool INV>
__device__ __forceinline__ constexpr double root_re(int p) { return Roots<R>::re[p]; }
template <int R, bool INV>
__device__ __forceinline__ constexpr double root_im(int p) { return INV ? -Roots<R>::im[p] : Roots<R>::im[p]; }

// acc += x * w (complex) with w a compile-time root: zero / unit parts fold away
template <int R, bool INV>
__device__ __forceinline__ void cmac_root(double& ar, double& ai, double xr, double xi, int p) {
    const double wr = root_re<R, INV>(p), wi = root_im<R, INV>(p);
    if (wr == 1.0) { ar += xr; ai += xi; }
    else if (wr == -1.0) { ar -= xr; ai -= xi; }
    else if (wr != 0.0) { ar = fma(xr, wr, ar); ai = fma(xi, wr, ai); }
    if (wi == 1.0) { ar -= xi; ai += xr; }
    else if (wi == -1.0) { ar += xi; ai -= xr; }
    else if (wi != 0.0) { ar = fma(-xi, wi, ar); ai = fma(xr, wi, ai); }
}

// In-register DFT of length R (natural order in and out), mixed radix: R = R1 R2 with R1
// the smallest of {4, 2, 3, 5} dividing R; R2 DFTs of length R1 over the stride-R2
// subsequences, twiddles e^{-+2 pi i n2 k1 / R}, R1 DFTs of length R2 -- all indices
// compile-time, roots folded (16 points: ~300 flops instead of 1024 FMA direct).
template <int R>
constexpr int dft_radix() {
    return (R % 4 == 0 && R > 4) ? 4 : (R % 2 == 0 && R > 2) ? 2 : (R % 3 == 0 && R > 3) ? 3 : (R % 5 == 0 && R > 5) ? 5 : R;
}

// Odd prime R (3, 5, 7, 19: the 640-, 480-, 420- and 380-point plans) by the symmetric pairs
// t_j = x_j + x_{R-j}, d_j = x_j - x_{R-j} (j = 1 .. H = (R - 1) / 2):
//   A_k = x_0 + sum_j cos(2 pi jk / R) t_j,  B_k = sum_j sin(2 pi jk / R) d_j,
//   forward X_k = A_k - i B_k, X_{R-k} = A_k + i B_k (inverse: swapped),
// about R real FMA per output instead of the direct codelet's 4R (roots compile-time).
template <int R, bool INV>
__device__ __forceinline__ void dft_sym(double (&xr)[R], double (&xi)[R]) {
    constexpr int H = (R - 1) / 2;
    double tr[H + 1], ti[H + 1], dr[H + 1], di[H + 1];
    double s0r = 0.0, s0i = 0.0;
#pragma unroll
    for (int j = 1; j <= H; ++j) {
        tr[j] = xr[j] + xr[R - j];
        ti[j] = xi[j] + xi[R - j];
        dr[j] = xr[j] - xr[R - j];
        di[j] = xi[j] - xi[R - j];
        s0r += tr[j];
        s0i += ti[j];
    }
    double ar[H + 1], ai[H + 1], br[H + 1], bi[H + 1];
#pragma unroll
    for (int k = 1; k <= H; ++k) {
        ar[k] = xr[0];
        ai[k] = xi[0];
        br[k] = 0.0;
        bi[k] = 0.0;
#pragma unroll
        for (int j = 1; j <= H; ++j) {
            const int p = (j * k) % R;
            const double c = Roots<R>::re[p], sn = -Roots<R>::im[p];   // cos, sin of 2 pi p / R
            ar[k] = fma(c, tr[j], ar[k]);
            ai[k] = fma(c, ti[j], ai[k]);
            br[k] = fma(sn, dr[j], br[k]);
            bi[k] = fma(sn, di[j], bi[k]);
        }
    }
    xr[0] += s0r;
    xi[0] += s0i;
#pragma unroll
    for (int k = 1; k <= H; ++k) {
        // A - i B = (ar + bi, ai - br);  A + i B = (ar - bi, ai + br)
        const int kf = INV ? R - k : k, kb = INV ? k : R - k;
        xr[kf] = ar[k] + bi[k];
        xi[kf] = ai[k] - br[k];
        xr[kb] = ar[k] - bi[k];
        xi[kb] = ai[k] + br[k];
    }
}

template <int R, bool INV>
__device__ __forceinline__ void dft_reg(double (&xr)[R], double (&xi)[R]) {
    constexpr int R1 = dft_radix<R>();
    if constexpr (R1 == R && R % 2 == 1 && R > 1 && FOTO_FFT_SYM) {
        dft_sym<R, INV>(xr, xi);
    } else if constexpr (R1 == R) {   // codelet: direct with compile-time roots
        double yr[R], yi[R];
#pragma unroll
        for (int k = 0; k < R; ++k) {
            double ar = 0.0, ai = 0.0;
#pragma unroll
            for (int n = 0; n < R; ++n) cmac_root<R, INV>(ar, ai, xr[n], xi[n], (n * k) % R);
            yr[k] = ar;
            yi[k] = ai;
        }
#pragma unroll
        for (int k = 0; k < R; ++k) { xr[k] = yr[k]; xi[k] = yi[k]; }
    } else {
        constexpr int R2 = R / R1;
        double ar[R1][R2], ai[R1][R2];   // A[k1][n2]
#pragma unroll
        for (int n2 = 0; n2 < R2; ++n2) {
            double tr[R1], ti[R1];
#pragma unroll
            for (int n1 = 0; n1 < R1; ++n1) { tr[n1] = xr[R2 * n1 + n2]; ti[n1] = xi[R2 * n1 + n2]; }
            dft_reg<R1, INV>(tr, ti);
#pragma unroll
            for (int k1 = 0; k1 < R1; ++k1) {
                const int p = (n2 * k1) % R;
                const double wr = root_re<R, INV>(p), wi = root_im<R, INV>(p);
                if (p == 0) { ar[k1][n2] = tr[k1]; ai[k1][n2] = ti[k1]; }
                else { ar[k1][n2] = fma(tr[k1], wr, -ti[k1] * wi); ai[k1][n2] = fma(tr[k1], wi, ti[k1] * wr); }
            }
        }
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) {
            dft_reg<R2, INV>(ar[k1], ai[k1]);
#pragma unroll
            for (int k2 = 0; k2 < R2; ++k2) { xr[k1 + R1 * k2] = ar[k1][k2]; xi[k1 + R1 * k2] = ai[k1][k2]; }
        }
    }
}

// stage 1 (in place on the LDS lines): for each (line, j2): the length-M1 DFT of
// z[M2 j1 + j2] (dft_reg), times e^{-+2 pi i j2 k1 / M}, stored at row k1, column j2
// PT (TWPT, round 6): the twiddles from the LDS copy of the post-twiddle table instead of the
// global table: e^{-2 pi i q / M} = PA_{2q} for 2q <= M (the same bits: the table's long-double
// angle 2 pi (2q) / (2M) is 2 pi q / M exactly), conj PA_{2(M-q)} above (within an ulp)
template <int M1, int M2, bool INV, int LPB, int NTH = 256, bool TWPT = false>
__device__ __forceinline__ void fft_stage1(double* L, const double* TW, const double* PT = nullptr) {
    constexpr int LS = FftGeom<M1, M2>::LS;
    constexpr int M = M1 * M2;
    for (int task = threadIdx.x; task < LPB * M2; task += NTH) {
        const int l = task / M2, j2 = task - (task / M2) * M2;
        double* Ll = L + l * LS;
        double xr[M1], xi[M1];
#pragma unroll
        for (int j1 = 0; j1 < M1; ++j1) {
            xr[j1] = Ll[2 * ((M2 + 1) * j1 + j2)];
            xi[j1] = Ll[2 * ((M2 + 1) * j1 + j2) + 1];
        }
        dft_reg<M1, INV>(xr, xi);
#pragma unroll
        for (int k1 = 0; k1 < M1; ++k1) {
            const int q = j2 * k1;   // < M
            double tr, ti;
            if constexpr (TWPT) {
                const bool lo = 2 * q <= M;
                const dbl2 w = *reinterpret_cast<const dbl2*>(&PT[8 * (lo ? q : M - q)]);
                tr = w.x;
                ti = (lo != INV) ? w.y : -w.y;
            } else {
                tr = TW[2 * q];
                ti = INV ? -TW[2 * q + 1] : TW[2 * q + 1];
            }
            Ll[2 * ((M2 + 1) * k1 + j2)] = fma(xr[k1], tr, -xi[k1] * ti);
            Ll[2 * ((M2 + 1) * k1 + j2) + 1] = fma(xr[k1], ti, xi[k1] * tr);
        }
    }
}

// stage 2 (in place): for each (line, k1): the length-M2 DFT of row k1; element
// k = k1 + M1 k2 of the result lands at row k1, column k2
template <int M1, int M2, bool INV, int LPB, int NTH = 256>
__device__ __forceinline__ void fft_stage2(double* L) {
    constexpr int LS = FftGeom<M1, M2>::LS;
    for (int task = threadIdx.x; task < LPB * M1; task += NTH) {
        const int l = task / M1, k1 = task - (task / M1) * M1;
        double* Lr = L + l * LS + 2 * (M2 + 1) * k1;
        double xr[M2], xi[M2];
#pragma unroll
        for (int j2 = 0; j2 < M2; ++j2) {
            xr[j2] = Lr[2 * j2];
            xi[j2] = Lr[2 * j2 + 1];
        }
        dft_reg<M2, INV>(xr, xi);
#pragma unroll
        for (int k2 = 0; k2 < M2; ++k2) {
            Lr[2 * k2] = xr[k2];
            Lr[2 * k2 + 1] = xi[k2];
        }
    }
}

// Stage 2 for a prime row length P too long for an in-register codelet (~2P live fp64
// registers: Middlebury's half-lengths 292 = 4 * 73 and 194 = 2 * 97).  Symmetric direct DFT:
// with u_j = z_j + z_{P-j}, v_j = z_j - z_{P-j} (j = 1 .. H, H = (P - 1) / 2),
//     A_k = z_0 + sum_j u_j cos(2 pi jk/P),   B_k = sum_j v_j sin(2 pi jk/P),   k = 0 .. H,
//     forward Z_k = A_k - i B_k, Z_{P-k} = A_k + i B_k       (inverse: the conjugate pairing).
// For all ROWS rows of the block the two sums are real GEMMs, (2 ROWS x H) (H x (H + 1)),
// run on the f64 MFMA (v_mfma_f64_16x16x4_f64): an M tile is 8 complex rows (tile rows 0-7
// their real parts, 8-15 their imaginary parts, so a lane's four results are the real and
// imaginary parts of two rows in one output column), K = H (a multiple of 4), N = H + 1
// padded to 16.  The B operands (cos, sin of 2 pi q / P) come from the P-entry root table CS in
// LDS, one 16-B read per k-step and N tile for both GEMMs.  (A direct per-output loop read
// ~48 B of LDS per multiply-add and was LDS-bound: 70-95 us per axis pass at 584x388x32.)
template <int P>
struct LdsPrime { static constexpr bool value = P > 32; };

template <int M1, int P, bool INV, int LPB, int NTH = 256>
__device__ __forceinline__ void fft_stage2_prime(double* L, const double* CS) {
    constexpr int LS = FftGeom<M1, P>::LS;
    constexpr int H = (P - 1) / 2;
    constexpr int ROWS = LPB * M1;
    constexpr int KS = H / 4, NTL = (H + 1 + 15) / 16, MT = ROWS / 8;
    constexpr int NW = NTH / 64;   // waves of the block (the M tiles are dealt to them)
    static_assert(H % 4 == 0 && ROWS % 8 == 0, "prime stage: K steps of 4, M tiles of 8 rows");
    static_assert(NTH % 64 == 0, "whole waves");
    for (int task = threadIdx.x; task < ROWS * H; task += NTH) {   // u, v in place
        const int row = task / H, j = 1 + task - row * H;
        const int l = row / M1, k1 = row - l * M1;
        double* Lr = L + l * LS + 2 * (P + 1) * k1;
        const double ar = Lr[2 * j], ai = Lr[2 * j + 1], br = Lr[2 * (P - j)], bi = Lr[2 * (P - j) + 1];
        Lr[2 * j] = ar + br;
        Lr[2 * j + 1] = ai + bi;
        Lr[2 * (P - j)] = ar - br;
        Lr[2 * (P - j) + 1] = ai - bi;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int am = lane & 15, ak = lane >> 4;   // A operand: row am, k ak of the step
    constexpr int MTW = (MT + NW - 1) / NW;     // M tiles per wave
    dbl4 dc[MTW][NTL], ds[MTW][NTL];
    double z0r[MTW][2], z0i[MTW][2];
#pragma unroll
    for (int w = 0; w < MTW; ++w) {
        const int mt = wave + NW * w;
        if (MT % NW != 0 && mt >= MT) continue;
        // this lane's A row: complex row 8 mt + (am & 7), real (am < 8) or imaginary part
        const int rowa = 8 * mt + (am & 7);
        const int offa = (rowa / M1) * LS + 2 * (P + 1) * (rowa % M1) + (am >> 3);
#pragma unroll
        for (int t = 0; t < NTL; ++t) { dc[w][t] = dbl4{0.0, 0.0, 0.0, 0.0}; ds[w][t] = dbl4{0.0, 0.0, 0.0, 0.0}; }
#pragma unroll 3
        for (int ks = 0; ks < KS; ++ks) {
            const int j = 4 * ks + ak + 1;
            const double au = L[offa + 2 * j], av = L[offa + 2 * (P - j)];
#pragma unroll
            for (int t = 0; t < NTL; ++t) {
                const int n = 16 * t + am;   // B operand: k ak, column n
                double bc = 0.0, bs = 0.0;
                if (n <= H) {
                    const int q = (j * n) % P;
                    bc = CS[2 * q];
                    bs = CS[2 * q + 1];
                }
                dc[w][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(au, bc, dc[w][t], 0, 0, 0);
                ds[w][t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bs, ds[w][t], 0, 0, 0);
            }
        }
        // D rows of this lane: (lane >> 4) + 4 reg -> complex rows g, g + 4 of the tile (reg 0, 1
        // real, reg 2, 3 imaginary); their z_0
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = 8 * mt + (lane >> 4) + 4 * h;
            const double* Lr = L + (row / M1) * LS + 2 * (P + 1) * (row % M1);
            z0r[w][h] = Lr[0];
            z0i[w][h] = Lr[1];
        }
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < MTW; ++w) {
        const int mt = wave + NW * w;
        if (MT % NW != 0 && mt >= MT) continue;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = 8 * mt + (lane >> 4) + 4 * h;
            double* Lr = L + (row / M1) * LS + 2 * (P + 1) * (row % M1);
#pragma unroll
            for (int t = 0; t < NTL; ++t) {
                const int k = 16 * t + (lane & 15);
                if (k > H) continue;
                const double Ar = z0r[w][h] + dc[w][t][h], Ai = z0i[w][h] + dc[w][t][2 + h];
                const double Br = ds[w][t][h], Bi = ds[w][t][2 + h];
                if (k == 0) {
                    Lr[0] = Ar;
                    Lr[1] = Ai;
                } else {
                    // A - i B = (Ar + Bi, Ai - Br);  A + i B = (Ar - Bi, Ai + Br)
                    const int kf = INV ? P - k : k, kb = INV ? k : P - k;
                    Lr[2 * kf] = Ar + Bi;
                    Lr[2 * kf + 1] = Ai - Br;
                    Lr[2 * kb] = Ar - Bi;
                    Lr[2 * kb + 1] = Ai + Br;
                }
            }
        }
    }
}

// the stage-2 variant for row length M2, and the LDS root table it needs (doubles)
template <int M1, int M2, bool INV, int LPB, int NTH = 256>
__device__ __forceinline__ void fft_stage2_any(double* L, const double* CS) {
    if constexpr (LdsPrime<M2>::value) fft_stage2_prime<M1, M2, INV, LPB, NTH>(L, CS);
    else fft_stage2<M1, M2, INV, LPB, NTH>(L);
}
template <int M2>
constexpr int fft_cs_len() { return LdsPrime<M2>::value ? 2 * M2 : 2; }

template <int M1, int M2>
__device__ __forceinline__ int fft_pos(int k) { return (M2 + 1) * (k % M1) + k / M1; }   // where Z_k lands

struct FftLines {   // this block's lines: CONTIG rows o0 + l, or columns (o0, i0 + l) of stride `inner`
    int o0, i0, nl;
};

// Strided lines (CONTIG = false: the y axis, element stride Nx) read LPB adjacent columns per
// block, LPB * 8 B of every row: 32 B at N = 1024 (LPB 4), a quarter of a 128-B line.  Blocks are
// dealt to the 8 XCDs round robin, so the neighbours that read the rest of each line sat on
// other XCDs and every XCD's L2 fetched the whole line (C4's y transforms ran at 1.6-1.8 TB/s).
// The swizzle gives each XCD a contiguous range of column groups: the blocks that share a
// line run on one XCD at about the same time (FOTO_FFT_XCD=0: the plain order, A/B builds).
#ifndef FOTO_FFT_XCD
#define FOTO_FFT_XCD 1
#endif
template <bool CONTIG, int LPB>
__device__ __forceinline__ FftLines fft_lines(int outer, int inner) {
    FftLines f;
    if (CONTIG) {
        f.o0 = blockIdx.x * LPB;
        f.i0 = 0;
        f.nl = min(LPB, outer - f.o0);
    } else {
        int b = blockIdx.x;
#if FOTO_FFT_XCD
        constexpr int NXCD = 8;
        const int nb = gridDim.x, per = nb / NXCD, rem = nb % NXCD, xcd = b % NXCD;
        b = xcd * per + min(xcd, rem) + b / NXCD;
#endif
        const int nib = (inner + LPB - 1) / LPB;
        f.o0 = b / nib;
        f.i0 = (b - f.o0 * nib) * LPB;
        f.nl = min(LPB, inner - f.i0);
    }
    return f;
}

// Phase loops run a compile-time number of rounds over idx = tid + 256 j (predicated), so a
// thread's global loads are all issued before the first is consumed: a tid-strided runtime
// loop compiled to load -> wait -> LDS store per element, one load in flight per thread.
template <int COUNT, int NTH = 256>
struct FftRounds {
    static constexpr int R = (COUNT + NTH - 1) / NTH;
    static __device__ __forceinline__ bool ok(int idx) { return COUNT % NTH == 0 || idx < COUNT; }
};

template <int M1, int M2, bool CONTIG, int NTH = 256>
__global__ __launch_bounds__(NTH) void k_dct_fft_fwd(int outer, int inner, const double* __restrict__ tab,
                                                     const double* __restrict__ in, double* __restrict__ out) {
    using G = FftGeom<M1, M2, CONTIG>;
    constexpr int M = G::M, N = G::N, LPB = G::LPB, LS = G::LS;
    __shared__ double L[LPB * LS];
    __shared__ double CS[fft_cs_len<M2>()];   // prime stage-2 roots (LdsPrime rows only)
    __shared__ __attribute__((aligned(16))) double PT[G::PT_LDS ? G::PTN : 2];
#if FOTO_FFT_TW_LDS
    __shared__ double TW[2 * M];
#else
    const double* TW = tab;
#endif
    const int tid = threadIdx.x;
    const FftLines f = fft_lines<CONTIG, LPB>(outer, inner);
    if constexpr (LdsPrime<M2>::value)
        for (int p = tid; p < 2 * M2; p += NTH) CS[p] = tab[6 * M + 6 + p];
    fft_pt_fill<G>(PT, tab);
    const int64_t st = CONTIG ? 1 : inner;
    auto base = [&](int l) -> int64_t {
        return CONTIG ? (int64_t)(f.o0 + l) * N : (int64_t)f.o0 * N * inner + f.i0 + l;
    };
#if FOTO_FFT_TW_LDS
    for (int p = tid; p < 2 * M; p += NTH) TW[p] = tab[p];
#endif
    {   // load (all rounds' loads in flight), then store in Makhoul order
        using RD = FftRounds<LPB * N, NTH>;
        // element j0 of this thread: (line l, position j); contiguous lines by line thread groups
        // (round 6: no index division per element)
        constexpr bool LT = CONTIG && FOTO_FFT_LINE_THREADS && NTH % LPB == 0 && N % (NTH / LPB) == 0 &&
                            N / (NTH / LPB) == RD::R;
        auto lj = [&](int j0, int& l, int& j) -> bool {
            if constexpr (LT) {
                l = tid / (NTH / LPB);
                j = tid - l * (NTH / LPB) + (NTH / LPB) * j0;
                return true;
            } else {
                const int idx = tid + NTH * j0;
                if (CONTIG) { l = idx / N; j = idx - l * N; }
                else { j = idx / LPB; l = idx - j * LPB; }
                return RD::ok(idx);
            }
        };
        double xv[RD::R];
#pragma unroll
        for (int j0 = 0; j0 < RD::R; ++j0) {
            int l, j;
            const bool ok = lj(j0, l, j);
            xv[j0] = (ok && l < f.nl) ? ld_dead(&in[base(l) + j * st]) : 0.0;
        }
#pragma unroll
        for (int j0 = 0; j0 < RD::R; ++j0) {
            int l, j;
            if (!lj(j0, l, j)) continue;
            const int p = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
            L[l * LS + 2 * fft_zpos<M2>(p >> 1) + (p & 1)] = xv[j0];
        }
    }
    __syncthreads();
    fft_stage1<M1, M2, false, LPB, NTH, G::PT_LDS && FOTO_FFT_TW_PT>(L, TW, PT);
    __syncthreads();
    fft_stage2_any<M1, M2, false, LPB, NTH>(L, CS);
    __syncthreads();
    const double* PA = tab + 2 * M;
    const double* PB = PA + 2 * (M + 1);
    const double s0 = PB[2 * (M + 1)], s = PB[2 * (M + 1) + 1];
    auto emit = [&](int l, int k) {   // X_k and X_{N-k} of line l
        const double* Ll = L + l * LS;
        const int pa = 2 * fft_pos<M1, M2>(k == M ? 0 : k), pb = 2 * fft_pos<M1, M2>(k == 0 ? 0 : M - k);
        const double zr = Ll[pa], zi = Ll[pa + 1], cr = Ll[pb], ci = -Ll[pb + 1];
        const double er = 0.5 * (zr + cr), ei = 0.5 * (zi + ci);     // DFT of the even samples
        const double orr = 0.5 * (zi - ci), oi = 0.5 * (cr - zr);     // DFT of the odd samples
        double war, wai, wbr, wbi;
        if constexpr (G::PT_LDS) {
            const dbl2 a = *reinterpret_cast<const dbl2*>(&PT[4 * k]), b = *reinterpret_cast<const dbl2*>(&PT[4 * k + 2]);
            war = a.x; wai = a.y; wbr = b.x; wbi = b.y;
        } else {
            war = PA[2 * k]; wai = PA[2 * k + 1]; wbr = PB[2 * k]; wbi = PB[2 * k + 1];
        }
        const double vr = er + fma(war, orr, -wai * oi), vi = ei + fma(war, oi, wai * orr);
        const double yr = fma(wbr, vr, -wbi * vi), yi = fma(wbr, vi, wbi * vr);
        const int64_t b = base(l);
        out[b + k * st] = (k == 0 ? s0 : s) * yr;
        if (k > 0 && k < M) out[b + (N - k) * st] = -s * yi;
    };
    if constexpr (CONTIG && FOTO_FFT_LINE_THREADS && NTH % LPB == 0) {
        // (round 6) a fixed line per thread group of NTH / LPB threads, k = t, t + TPL, ...: no
        // index division per element, and the line test hoisted out of the rounds
        constexpr int TPL = NTH / LPB, RK = (M + 1 + TPL - 1) / TPL;
        const int l = tid / TPL, t = tid - l * TPL;
        if (l < f.nl) {
#pragma unroll
            for (int r = 0; r < RK; ++r) {
                const int k = t + TPL * r;
                if ((M + 1) % TPL != 0 && r == RK - 1 && k > M) break;
                emit(l, k);
            }
        }
    } else {
        using RO = FftRounds<LPB * (M + 1), NTH>;
#pragma unroll
        for (int j0 = 0; j0 < RO::R; ++j0) {
            const int idx = tid + NTH * j0;
            if (!RO::ok(idx)) continue;
            int l, k;
            if (CONTIG) { l = idx / (M + 1); k = idx - l * (M + 1); }
            else { k = idx / LPB; l = idx - k * LPB; }
            if (l >= f.nl) continue;
            emit(l, k);
        }
    }
}

template <int M1, int M2, bool CONTIG, int NTH = 256>
__global__ __launch_bounds__(NTH) void k_dct_fft_inv(int outer, int inner, const double* __restrict__ tab,
                                                     const double* __restrict__ in, double* __restrict__ out) {
    using G = FftGeom<M1, M2, CONTIG>;
    constexpr int M = G::M, N = G::N, LPB = G::LPB, LS = G::LS;
    __shared__ double L[LPB * LS];
    __shared__ double CS[fft_cs_len<M2>()];   // prime stage-2 roots (LdsPrime rows only)
    __shared__ __attribute__((aligned(16))) double PT[G::PT_LDS ? G::PTN : 2];
#if FOTO_FFT_TW_LDS
    __shared__ double TW[2 * M];
#else
    const double* TW = tab;
#endif
    const int tid = threadIdx.x;
    const FftLines f = fft_lines<CONTIG, LPB>(outer, inner);
    if constexpr (LdsPrime<M2>::value)
        for (int p = tid; p < 2 * M2; p += NTH) CS[p] = tab[6 * M + 6 + p];
    fft_pt_fill<G>(PT, tab);
    const int64_t st = CONTIG ? 1 : inner;
    auto base = [&](int l) -> int64_t {
        return CONTIG ? (int64_t)(f.o0 + l) * N : (int64_t)f.o0 * N * inner + f.i0 + l;
    };
#if FOTO_FFT_TW_LDS
    for (int p = tid; p < 2 * M; p += NTH) TW[p] = tab[p];
#endif
    const double* PA = tab + 2 * M;
    const double* PB = PA + 2 * (M + 1);
    const double is0 = 1.0 / PB[2 * (M + 1)], is = 1.0 / PB[2 * (M + 1) + 1];
    // Z_k and Z_{M-k} need the same four inputs X_k, X_{N-k}, X_{M-k}, X_{M+k} (V_k and V_{M-k},
    // conjugated in the other's formula), so one thread makes both: k in [0, M/2], half the
    // global reads of one Z per thread (L2-resident lines, read straight from global; no LDS
    // image of X, so Z is written once and nothing is held in registers across a barrier)
    constexpr int MH = M / 2 + 1;
    using RP = FftRounds<LPB * MH, NTH>;
    // element j0 of this thread: (line l, k); contiguous lines by line thread groups (round 6)
    constexpr bool LT = CONTIG && FOTO_FFT_LINE_THREADS && NTH % LPB == 0 &&
                        (MH + NTH / LPB - 1) / (NTH / LPB) == RP::R;
    auto lk = [&](int j0, int& l, int& k) -> bool {
        if constexpr (LT) {
            l = tid / (NTH / LPB);
            k = tid - l * (NTH / LPB) + (NTH / LPB) * j0;
            return k < MH;
        } else {
            const int idx = tid + NTH * j0;
            if (CONTIG) { l = idx / MH; k = idx - l * MH; }
            else { k = idx / LPB; l = idx - k * LPB; }
            return RP::ok(idx);
        }
    };
    double xk[RP::R], xnk[RP::R], xmk[RP::R], xpk[RP::R];   // X_k, X_{N-k}, X_{M-k}, X_{N-M+k}
#pragma unroll
    for (int j0 = 0; j0 < RP::R; ++j0) {   // all rounds' loads first
        int l, k;
        const bool ok = lk(j0, l, k);
        xk[j0] = xnk[j0] = xmk[j0] = xpk[j0] = 0.0;
        if (ok && l < f.nl) {
            const double* X = in + base(l);
            xk[j0] = ld_dead(&X[k * st]);
            if (k != 0) xnk[j0] = ld_dead(&X[(N - k) * st]);
            xmk[j0] = ld_dead(&X[(M - k) * st]);
            if (M - k != 0) xpk[j0] = ld_dead(&X[(N - (M - k)) * st]);
        }
    }
    if constexpr (G::PT_LDS) __syncthreads();   // (PT; the X loads stay in flight across it)
#pragma unroll
    for (int j0 = 0; j0 < RP::R; ++j0) {
        int l, k;
        if (!lk(j0, l, k)) continue;
        // V_j = e^{+i pi j/(2N)} Y_j, Y_j = (X_j / s_j, -X_{N-j} / s_{N-j}), j in {k, M - k}
        auto V = [&](int j, double xj, double xnj, double& vr, double& vi) {
            const double yr = xj * (j == 0 ? is0 : is), yi = (j == 0) ? 0.0 : -xnj * is;
            double wbr, wbi;
            if constexpr (G::PT_LDS) {
                const dbl2 b = *reinterpret_cast<const dbl2*>(&PT[4 * j + 2]);
                wbr = b.x;
                wbi = -b.y;
            } else {
                wbr = PB[2 * j];
                wbi = -PB[2 * j + 1];
            }
            vr = fma(wbr, yr, -wbi * yi);
            vi = fma(wbr, yi, wbi * yr);
        };
        // Z_q from V_q = (ar, ai) and V_{M-q} = (br, bi)
        auto Zq = [&](int q, double ar, double ai, double br, double bi, double& zr, double& zi) {
            bi = -bi;                                                  // conj V_{M-q} = V_{q+M}
            const double er = 0.5 * (ar + br), ei = 0.5 * (ai + bi);   // Ve_q
            const double dr = 0.5 * (ar - br), di = 0.5 * (ai - bi);
            double war, wai;                                           // e^{+2 pi i q/N}
            if constexpr (G::PT_LDS) {
                const dbl2 a = *reinterpret_cast<const dbl2*>(&PT[4 * q]);
                war = a.x;
                wai = -a.y;
            } else {
                war = PA[2 * q];
                wai = -PA[2 * q + 1];
            }
            const double orr = fma(war, dr, -wai * di), oi = fma(war, di, wai * dr);   // Vo_q
            zr = er - oi;                                              // Z = Ve + i Vo
            zi = ei + orr;
        };
        double z1r = 0.0, z1i = 0.0, z2r = 0.0, z2i = 0.0;
        if (l < f.nl) {
            double ar, ai, br, bi;
            V(k, xk[j0], xnk[j0], ar, ai);
            V(M - k, xmk[j0], xpk[j0], br, bi);
            Zq(k, ar, ai, br, bi, z1r, z1i);
            Zq(M - k, br, bi, ar, ai, z2r, z2i);
        }
        L[l * LS + 2 * fft_zpos<M2>(k)] = z1r;
        L[l * LS + 2 * fft_zpos<M2>(k) + 1] = z1i;
        if (k != 0 && 2 * k != M) {   // Z_{M-k} (k = 0: M - k = M is no Z index; 2k = M: the same Z)
            L[l * LS + 2 * fft_zpos<M2>(M - k)] = z2r;
            L[l * LS + 2 * fft_zpos<M2>(M - k) + 1] = z2i;
        }
    }
    __syncthreads();
    fft_stage1<M1, M2, true, LPB, NTH, G::PT_LDS && FOTO_FFT_TW_PT>(L, TW, PT);
    __syncthreads();
    fft_stage2_any<M1, M2, true, LPB, NTH>(L, CS);
    __syncthreads();
    constexpr double iM = 1.0 / M;
    if constexpr (CONTIG && FOTO_FFT_LINE_THREADS && NTH % LPB == 0 && N % (NTH / LPB) == 0) {
        constexpr int TPL = NTH / LPB, RI = N / TPL;   // (round 6) a fixed line per thread group
        const int l = tid / TPL, t = tid - l * TPL;
        if (l < f.nl) {
            const double* Ll = L + l * LS;
            double* o = out + base(l);
#pragma unroll
            for (int r = 0; r < RI; ++r) {   // x_i = v_p, p = Makhoul position of i
                const int i = t + TPL * r;
                const int p = (i & 1) ? N - 1 - (i >> 1) : (i >> 1);
                o[i] = Ll[2 * fft_pos<M1, M2>(p >> 1) + (p & 1)] * iM;
            }
        }
    } else {
        using RS = FftRounds<LPB * N, NTH>;
#pragma unroll
        for (int j0 = 0; j0 < RS::R; ++j0) {   // x_i = v_p, p = Makhoul position of i
            const int idx = tid + NTH * j0;
            if (!RS::ok(idx)) continue;
            int l, i;
            if (CONTIG) { l = idx / N; i = idx - l * N; }
            else { i = idx / LPB; l = idx - i * LPB; }
            if (l >= f.nl) continue;
            const int p = (i & 1) ? N - 1 - (i >> 1) : (i >> 1);
            out[base(l) + i * st] = L[l * LS + 2 * fft_pos<M1, M2>(p >> 1) + (p & 1)] * iM;
        }
    }
}

// supported line lengths N = 2 M1 M2 (others use the GEMM kernels)
#define FOTO_FFT_SIZES(X) X(8, 2, 2) X(16, 2, 4) X(32, 4, 4) X(64, 4, 8) X(128, 8, 8) X(256, 8, 16) \
    X(146, 1, 73) X(194, 1, 97) X(380, 10, 19) X(388, 2, 97) X(420, 14, 15) X(480, 15, 16) X(512, 16, 16) X(584, 4, 73) X(640, 16, 20)    \
    X(1024, 16, 32)

static bool fft_factors(int n, int* m1, int* m2) {
#define FOTO_FFT_CASE(NN, A, B) if (n == NN) { *m1 = A; *m2 = B; return true; }
    FOTO_FFT_SIZES(FOTO_FFT_CASE)
#undef FOTO_FFT_CASE
    return false;
}

// per-axis table (host, long double): see the layout above
static std::vector<double> fft_table(int n) {
    const int M = n / 2;
    std::vector<double> t;
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int p = 0; p < M; ++p) {
        t.push_back((double)cosl(2.0L * pi * p / M));
        t.push_back((double)-sinl(2.0L * pi * p / M));
    }
    for (int k = 0; k <= M; ++k) {
        t.push_back((double)cosl(2.0L * pi * k / n));
        t.push_back((double)-sinl(2.0L * pi * k / n));
    }
    for (int k = 0; k <= M; ++k) {
        t.push_back((double)cosl(pi * k / (2.0L * n)));
        t.push_back((double)-sinl(pi * k / (2.0L * n)));
    }
    t.push_back((double)sqrtl(1.0L / n));
    t.push_back((double)sqrtl(2.0L / n));
    int m1 = 0, m2 = 0;
    if (fft_factors(n, &m1, &m2) && m2 > 32)   // LdsPrime rows: cos, sin of 2 pi q / m2 (at 6 M + 6)
        for (int q = 0; q < m2; ++q) {
            t.push_back((double)cosl(2.0L * pi * q / m2));
            t.push_back((double)sinl(2.0L * pi * q / m2));
        }
    return t;
}

static int g_dct_fft = -1;   // FOTO_DCT_FFT=0 selects the GEMM kernels (A/B runs)
// threads per block of the contiguous (x) and strided (y, t) axis passes (A/B builds)
#ifndef FOTO_FFT_NTH_C
#define FOTO_FFT_NTH_C 256
#endif
#ifndef FOTO_FFT_NTH_S
#define FOTO_FFT_NTH_S 256
#endif
constexpr int FFT_NTH_C = FOTO_FFT_NTH_C, FFT_NTH_S = FOTO_FFT_NTH_S;

// FFT path along one axis of [outer][n][inner]; hipErrorNotSupported if n has no instantiation
static hipError_t dct_fft_axis(int outer, int n, int inner, bool inv, const double* tab, const double* in,
                               double* out, hipStream_t s) {
    if (g_dct_fft < 0) {
        const char* e = getenv("FOTO_DCT_FFT");
        g_dct_fft = e ? atoi(e) : 1;
    }
    int m1, m2;
    // n < 64: the GEMM kernel is as fast (t axis at 32: 49 vs 54 us)
    if (!g_dct_fft || !tab || n < 64 || !fft_factors(n, &m1, &m2)) return hipErrorNotSupported;
#define FOTO_FFT_LAUNCH(NN, A, B)                                                                  \
    if (n == NN) {                                                                                 \
        const bool contig = (inner == 1);                                                          \
        const int LPB = contig ? FftGeom<A, B, true>::LPB : FftGeom<A, B, false>::LPB;             \
        const int nb = contig ? (outer + LPB - 1) / LPB : outer * ((inner + LPB - 1) / LPB);       \
        if (contig) {                                                                              \
            if (inv) k_dct_fft_inv<A, B, true, FFT_NTH_C><<<nb, FFT_NTH_C, 0, s>>>(outer, inner, tab, in, out); \
            else k_dct_fft_fwd<A, B, true, FFT_NTH_C><<<nb, FFT_NTH_C, 0, s>>>(outer, inner, tab, in, out);     \
        } else {                                                                                   \
            if (inv) k_dct_fft_inv<A, B, false, FFT_NTH_S><<<nb, FFT_NTH_S, 0, s>>>(outer, inner, tab, in, out); \
            else k_dct_fft_fwd<A, B, false, FFT_NTH_S><<<nb, FFT_NTH_S, 0, s>>>(outer, inner, tab, in, out);     \
        }                                                                                          \
        return hipGetLastError();                                                                  \
    }
    FOTO_FFT_SIZES(FOTO_FFT_LAUNCH)
#undef FOTO_FFT_LAUNCH
    return hipErrorNotSupported;
}

// ============================================================================ x and t axes in one pass
//
// A single shard's 3-D DCT is separable, and DCTs along different axes commute, so the solve's
// forward transform can run as (x, t) then y instead of x, y, t: one block per row y takes the
// Nt lines (t, y, :) through the x-axis FFT DCT above (XT_LPB line images in LDS at a time) and
// folds each finished pair of lines (j, Nt - 1 - j) into the t-axis DCT of its columns the way
// the column kernels do (thread kx: e_m += E[m][j] (x_j + x_{Nt-1-j}), o_m += O[m][j] (x_j -
// x_{Nt-1-j}), j ascending -- TCol's even / odd halves in Cth, the same sums in the same order).
// The x-transformed volume never goes to HBM: the chain is two full-volume passes instead of
// three, and the output is in the layout the plain y pass expects ([kt][y][kx]), which then
// leaves b^ exactly where the histogram and x^ read it.  The inverse mirrors it: the y pass,
// then one block per row y loads its columns x^[kt][y][kx], forms the inverse t-DCT of a chunk
// of line pairs in registers, stages those lines in LDS and runs the x-axis inverse on them.
// MEASURED SLOWER, so opt-in (FOTO_DCT_XT=1, SpectralPlan::init): 151 / 165 us per launch at the
// bench grid against 69 / 72 us for the pairs of passes it replaces -- the slab's state pins
// one block per CU and its phases serialise; the passes are latency-bound, not HBM-bound (their
// intermediates stay in the Infinity Cache), so removing one saves less than it costs here.
// Single shard, Nt even and <= 32 (the column kernels' sizes), 64 <= Nx <= 640 with an FFT plan.
// A block carries the whole x-transformed row slab's t-sums (Nt x Nx values, 164 KB at the bench
// grid) through the line loop: 512 threads (two waves per SIMD, 256 VGPRs each -- 640 threads
// would leave 168 and spill), thread kx owning column kx's sums, the even half in registers and
// the odd half in LDS (read, advanced by the chunk's pairs and written back once per chunk, so
// neither is live in registers beside the FFT stages' codelets: both in registers spilled ~68
// VGPRs).  The columns beyond 512 (Nx = 584, 640) are split four ways, part p of column
// 512 + tid / 4 taking the sums m = p, p + 4, ... of both halves in registers.  The sums run over
// j in ascending order as in the column kernels.
constexpr int XT_MAXH = 16;   // Nt <= 2 XT_MAXH
constexpr int XT_NTH = 512;
constexpr int XT_SPLIT = 4;   // parts of a column beyond XT_NTH
constexpr int XT_MAXN = XT_NTH + XT_NTH / XT_SPLIT;   // 640
constexpr int XT_HB = XT_MAXH / XT_SPLIT;             // sums of a part
template <int M1, int M2>
struct XtGeom {
    static constexpr int M = M1 * M2, N = 2 * M;
    static constexpr int LS = FftGeom<M1, M2>::LS;
    static constexpr int LPBF = 16;                    // forward: lines per chunk (8 pairs)
    static constexpr int LPBI = 8;                     // inverse: lines per chunk (+ their X rows)
    static constexpr int NB = N > XT_NTH ? N - XT_NTH : 1;   // split columns (>= 1: array sizes)
};

// line slot l of chunk q (pairs q PP .. q PP + PP - 1): slot 2 i is t = j, slot 2 i + 1 is
// t = Nt - 1 - j, j = q PP + i
__device__ __forceinline__ int xt_line_t(int q, int pp, int nt, int l) {
    const int j = q * pp + (l >> 1);
    return (l & 1) ? nt - 1 - j : j;
}

// X_kx of a line from its DFT image (k_dct_fft_fwd's output phase for one column)
struct XtCol {
    int pa, pb;
    double war, wai, wbr, wbi, sk;
    bool hi;
    template <int M1, int M2>
    __device__ __forceinline__ void init(const double* PA, const double* PB, int kx) {
        constexpr int M = M1 * M2, N = 2 * M;
        hi = kx > M;
        const int k = hi ? N - kx : kx;
        pa = 2 * fft_pos<M1, M2>(k == M ? 0 : k);
        pb = 2 * fft_pos<M1, M2>(k == 0 ? 0 : M - k);
        war = PA[2 * k];
        wai = PA[2 * k + 1];
        wbr = PB[2 * k];
        wbi = PB[2 * k + 1];
        const double s0 = PB[2 * (M + 1)], s = PB[2 * (M + 1) + 1];
        sk = hi ? -s : (k == 0 ? s0 : s);
    }
    __device__ __forceinline__ double x(const double* Ll) const {
        const double zr = Ll[pa], zi = Ll[pa + 1], cr = Ll[pb], ci = -Ll[pb + 1];
        const double er = 0.5 * (zr + cr), ei = 0.5 * (zi + ci);
        const double orr = 0.5 * (zi - ci), oi = 0.5 * (cr - zr);
        const double vr = er + fma(war, orr, -wai * oi), vi = ei + fma(war, oi, wai * orr);
        const double yr = fma(wbr, vr, -wbi * vi), yi = fma(wbr, vi, wbi * vr);
        return sk * (hi ? yi : yr);
    }
};

template <int M1, int M2>
__global__ __launch_bounds__(XT_NTH) void k_dct_xt_fwd(int Nt, int Ny, const double* __restrict__ tab,
                                                       const double* __restrict__ Ch, const double* __restrict__ in,
                                                       double* __restrict__ out) {
    using G = XtGeom<M1, M2>;
    constexpr int M = G::M, N = G::N, NTH = XT_NTH, LS = G::LS, LPB = G::LPBF, PP = LPB / 2;
    static_assert(N <= XT_MAXN, "columns beyond 512 split four ways: Nx <= 640");
    __shared__ double L[LPB * LS];
    __shared__ double OS[XT_MAXH][XT_NTH];   // part A's odd sums, [m][column]
    __shared__ double CS[fft_cs_len<M2>()];
    const int tid = threadIdx.x, y = blockIdx.x;
    const int H = Nt / 2;
    if constexpr (LdsPrime<M2>::value)
        for (int p = tid; p < 2 * M2; p += NTH) CS[p] = tab[6 * M + 6 + p];
    const double* TW = tab;
    const double* PA = tab + 2 * M;
    const double* PB = PA + 2 * (M + 1);
    // part A: column tid, all sums; part B (Nx > 512): column 512 + tid / 4, sums m = p + 4 i
    const bool ha = tid < N;
    const int cb = XT_NTH + tid / XT_SPLIT, pb = tid % XT_SPLIT;
    const bool hb = (N > XT_NTH) && cb < N;
    double e[XT_MAXH], eb[XT_HB], ob[XT_HB];
#pragma unroll
    for (int m = 0; m < XT_MAXH; ++m) {
        e[m] = 0.0;
        OS[m][tid] = 0.0;   // (a thread only ever touches its own column's slots)
    }
#pragma unroll
    for (int i = 0; i < XT_HB; ++i) { eb[i] = 0.0; ob[i] = 0.0; }
    const int nq = (H + PP - 1) / PP;
    for (int q = 0; q < nq; ++q) {
        const int npair = min(PP, H - q * PP), nl = 2 * npair;
        {   // the chunk's lines into LDS in Makhoul order (all loads issued first); a thread takes
            // columns tid + NTH c of every line, so its LDS positions are the same in every line
            // and chunk (an index decomposition per element was hoisted out of the chunk loop and
            // spilled)
            constexpr int CPL = (N + NTH - 1) / NTH;
            double xv[LPB][CPL];
#pragma unroll
            for (int l = 0; l < LPB; ++l) {
                const double* row = in + ((int64_t)xt_line_t(q, PP, Nt, l) * Ny + y) * N;
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const int j = tid + NTH * c;
                    xv[l][c] = (l < nl && (N % NTH == 0 || j < N)) ? ld_dead(&row[j]) : 0.0;
                }
            }
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const int j = tid + NTH * c;
                if (N % NTH != 0 && j >= N) continue;
                const int p = (j & 1) ? N - 1 - (j >> 1) : (j >> 1);
                const int pos = 2 * fft_zpos<M2>(p >> 1) + (p & 1);
#pragma unroll
                for (int l = 0; l < LPB; ++l) L[l * LS + pos] = xv[l][c];
            }
        }
        __syncthreads();
        fft_stage1<M1, M2, false, LPB, NTH>(L, TW);
        __syncthreads();
        fft_stage2_any<M1, M2, false, LPB, NTH>(L, CS);
        __syncthreads();
        double od[XT_MAXH];   // part A's odd sums while this chunk's pairs are added
#pragma unroll
        for (int m = 0; m < XT_MAXH; ++m) od[m] = OS[m][tid];
        // (the columns' twiddles are re-read per chunk, L1 hits: held across the FFT stages they
        // cost ~26 VGPRs)
        XtCol A, B;
        if (ha) A.init<M1, M2>(PA, PB, tid);
        if (hb) B.init<M1, M2>(PA, PB, cb);
        for (int i = 0; i < npair; ++i) {   // pair j = q PP + i: lines t = j (slot 2 i), Nt - 1 - j
            const int j = q * PP + i;
            const double* L0 = L + (2 * i) * LS;
            const double* L1 = L0 + LS;
            if (ha) {
                const double x0 = A.x(L0), x1 = A.x(L1);
                const double sv = x0 + x1, dv = x0 - x1;
#pragma unroll
                for (int m = 0; m < XT_MAXH; ++m) {
                    if (m < H) {
                        e[m] = fma(Ch[m * H + j], sv, e[m]);
                        od[m] = fma(Ch[H * H + m * H + j], dv, od[m]);
                    }
                }
            }
            if (hb) {
                const double x0 = B.x(L0), x1 = B.x(L1);
                const double sv = x0 + x1, dv = x0 - x1;
#pragma unroll
                for (int i4 = 0; i4 < XT_HB; ++i4) {
                    const int m = pb + XT_SPLIT * i4;
                    if (m < H) {
                        eb[i4] = fma(Ch[m * H + j], sv, eb[i4]);
                        ob[i4] = fma(Ch[H * H + m * H + j], dv, ob[i4]);
                    }
                }
            }
        }
#pragma unroll
        for (int m = 0; m < XT_MAXH; ++m) OS[m][tid] = od[m];
        __syncthreads();   // (the next chunk's lines overwrite L)
    }
    if (ha) {
#pragma unroll
        for (int m = 0; m < XT_MAXH; ++m) {
            if (m < H) {
                out[((int64_t)(2 * m) * Ny + y) * N + tid] = e[m];
                out[((int64_t)(2 * m + 1) * Ny + y) * N + tid] = OS[m][tid];
            }
        }
    }
    if (hb) {
#pragma unroll
        for (int i4 = 0; i4 < XT_HB; ++i4) {
            const int m = pb + XT_SPLIT * i4;
            if (m < H) {
                out[((int64_t)(2 * m) * Ny + y) * N + cb] = eb[i4];
                out[((int64_t)(2 * m + 1) * Ny + y) * N + cb] = ob[i4];
            }
        }
    }
}

template <int M1, int M2>
__global__ __launch_bounds__(XT_NTH) void k_dct_tx_inv(int Nt, int Ny, const double* __restrict__ tab,
                                                       const double* __restrict__ Ch, const double* __restrict__ in,
                                                       double* __restrict__ out) {
    using G = XtGeom<M1, M2>;
    constexpr int M = G::M, N = G::N, NTH = XT_NTH, LS = G::LS, LPB = G::LPBI, PP = LPB / 2, NB = G::NB;
    static_assert(N <= XT_MAXN, "columns beyond 512 split four ways: Nx <= 640");
    // L: the chunk's line images; before the input phase writes them, the split columns'
    // partial sums PE / PO live in the same space
    static_assert(2 * XT_SPLIT * PP * NB <= LPB * LS, "partial sums fit the line images");
    __shared__ double L[LPB * LS];
    __shared__ double XL[LPB * N];            // the chunk's lines after the inverse t-DCT, natural order
    __shared__ double XO[XT_MAXH][XT_NTH];    // part A's odd inputs x^_{2m+1}, [m][column]
    __shared__ double CS[fft_cs_len<M2>()];
    double(*PE)[PP][NB] = reinterpret_cast<double(*)[PP][NB]>(L);
    double(*PO)[PP][NB] = reinterpret_cast<double(*)[PP][NB]>(L + XT_SPLIT * PP * NB);
    const int tid = threadIdx.x, y = blockIdx.x;
    const int H = Nt / 2;
    if constexpr (LdsPrime<M2>::value)
        for (int p = tid; p < 2 * M2; p += NTH) CS[p] = tab[6 * M + 6 + p];
    const double* TW = tab;
    const double* PA = tab + 2 * M;
    const double* PB = PA + 2 * (M + 1);
    const double is0 = 1.0 / PB[2 * (M + 1)], is = 1.0 / PB[2 * (M + 1) + 1];
    const bool ha = tid < N;
    const int cb = XT_NTH + tid / XT_SPLIT, pb = tid % XT_SPLIT;
    const bool hb = (N > XT_NTH) && cb < N;
    double xe[XT_MAXH], xeb[XT_HB], xob[XT_HB];   // x^_{2m}, x^_{2m+1} (all loads first)
    {
        double xo[XT_MAXH];
#pragma unroll
        for (int m = 0; m < XT_MAXH; ++m) {
            xe[m] = (m < H && ha) ? ld_dead(&in[((int64_t)(2 * m) * Ny + y) * N + tid]) : 0.0;
            xo[m] = (m < H && ha) ? ld_dead(&in[((int64_t)(2 * m + 1) * Ny + y) * N + tid]) : 0.0;
        }
#pragma unroll
        for (int m = 0; m < XT_MAXH; ++m) XO[m][tid] = xo[m];   // (own column's slots only)
    }
#pragma unroll
    for (int i4 = 0; i4 < XT_HB; ++i4) {
        const int m = pb + XT_SPLIT * i4;
        xeb[i4] = (m < H && hb) ? ld_dead(&in[((int64_t)(2 * m) * Ny + y) * N + cb]) : 0.0;
        xob[i4] = (m < H && hb) ? ld_dead(&in[((int64_t)(2 * m + 1) * Ny + y) * N + cb]) : 0.0;
    }
    const int nq = (H + PP - 1) / PP;
    for (int q = 0; q < nq; ++q) {
        const int npair = min(PP, H - q * PP), nl = 2 * npair;
        double xo[XT_MAXH];   // part A's odd inputs for this chunk's sums
#pragma unroll
        for (int m = 0; m < XT_MAXH; ++m) xo[m] = XO[m][tid];
        for (int i = 0; i < npair; ++i) {   // k_dct_t_inv_xhat's sums for t = j, Nt - 1 - j
            const int j = q * PP + i;
            if (ha) {
                double ev = 0.0, ov = 0.0;
#pragma unroll
                for (int m = 0; m < XT_MAXH; ++m) {
                    if (m < H) {
                        ev = fma(Ch[m * H + j], xe[m], ev);
                        ov = fma(Ch[H * H + m * H + j], xo[m], ov);
                    }
                }
                XL[(2 * i) * N + tid] = ev + ov;
                XL[(2 * i + 1) * N + tid] = ev - ov;
            }
            if (hb) {
                double ev = 0.0, ov = 0.0;
#pragma unroll
                for (int i4 = 0; i4 < XT_HB; ++i4) {
                    const int m = pb + XT_SPLIT * i4;
                    if (m < H) {
                        ev = fma(Ch[m * H + j], xeb[i4], ev);
                        ov = fma(Ch[H * H + m * H + j], xob[i4], ov);
                    }
                }
                PE[pb][i][cb - XT_NTH] = ev;
                PO[pb][i][cb - XT_NTH] = ov;
            }
        }
        if (N > XT_NTH) {   // the split columns' lines: the four parts in order
            __syncthreads();
            for (int w = tid; w < npair * NB; w += NTH) {
                const int i = w / NB, c = w - i * NB;
                const double ev = ((PE[0][i][c] + PE[1][i][c]) + PE[2][i][c]) + PE[3][i][c];
                const double ov = ((PO[0][i][c] + PO[1][i][c]) + PO[2][i][c]) + PO[3][i][c];
                XL[(2 * i) * N + XT_NTH + c] = ev + ov;
                XL[(2 * i + 1) * N + XT_NTH + c] = ev - ov;
            }
        }
        __syncthreads();
        // k_dct_fft_inv's input phase on the LDS rows: Z_k and Z_{M-k} from X_k, X_{N-k}, X_{M-k},
        // X_{N-M+k}; thread: k = tid + NTH c of every line (the per-k twiddles once per chunk)
        constexpr int MH = M / 2 + 1;
        constexpr int CPK = (MH + NTH - 1) / NTH;
#pragma unroll
        for (int c = 0; c < CPK; ++c) {
            const int kk = tid + NTH * c;
            if (MH % NTH != 0 && kk >= MH) continue;
            // V_j = e^{+i pi j/(2N)} Y_j (j = kk, M - kk), then Z_q = Ve_q + i Vo_q (q = kk, M - kk)
            const int j1 = kk, j2 = M - kk;
            const double s1 = (j1 == 0) ? is0 : is, s2 = (j2 == 0) ? is0 : is;
            const double b1r = PB[2 * j1], b1i = -PB[2 * j1 + 1], b2r = PB[2 * j2], b2i = -PB[2 * j2 + 1];
            const double a1r = PA[2 * j1], a1i = -PA[2 * j1 + 1], a2r = PA[2 * j2], a2i = -PA[2 * j2 + 1];
            const int q1 = 2 * fft_zpos<M2>(kk), q2 = 2 * fft_zpos<M2>(M - kk);
            const bool two = kk != 0 && 2 * kk != M;
#pragma unroll
            for (int l = 0; l < LPB; ++l) {
                double z1r = 0.0, z1i = 0.0, z2r = 0.0, z2i = 0.0;
                if (l < nl) {
                    const double* X = XL + l * N;
                    const double xk = X[kk], xnk = (kk != 0) ? X[N - kk] : 0.0;
                    const double xmk = X[M - kk], xpk = (M - kk != 0) ? X[N - (M - kk)] : 0.0;
                    const double y1r = xk * s1, y1i = (j1 == 0) ? 0.0 : -xnk * is;
                    const double y2r = xmk * s2, y2i = (j2 == 0) ? 0.0 : -xpk * is;
                    const double ar = fma(b1r, y1r, -b1i * y1i), ai = fma(b1r, y1i, b1i * y1r);
                    const double br = fma(b2r, y2r, -b2i * y2i), bi = fma(b2r, y2i, b2i * y2r);
                    {   // Z_kk from V_kk = (ar, ai), V_{M-kk} = (br, bi)
                        const double cbi = -bi;
                        const double er = 0.5 * (ar + br), ei = 0.5 * (ai + cbi);
                        const double dr = 0.5 * (ar - br), di = 0.5 * (ai - cbi);
                        const double orr = fma(a1r, dr, -a1i * di), oi = fma(a1r, di, a1i * dr);
                        z1r = er - oi;
                        z1i = ei + orr;
                    }
                    {   // Z_{M-kk} from V_{M-kk}, V_kk
                        const double cai = -ai;
                        const double er = 0.5 * (br + ar), ei = 0.5 * (bi + cai);
                        const double dr = 0.5 * (br - ar), di = 0.5 * (bi - cai);
                        const double orr = fma(a2r, dr, -a2i * di), oi = fma(a2r, di, a2i * dr);
                        z2r = er - oi;
                        z2i = ei + orr;
                    }
                }
                L[l * LS + q1] = z1r;
                L[l * LS + q1 + 1] = z1i;
                if (two) {
                    L[l * LS + q2] = z2r;
                    L[l * LS + q2 + 1] = z2i;
                }
            }
        }
        __syncthreads();
        fft_stage1<M1, M2, true, LPB, NTH>(L, TW);
        __syncthreads();
        fft_stage2_any<M1, M2, true, LPB, NTH>(L, CS);
        __syncthreads();
        constexpr double iM = 1.0 / M;
        constexpr int CPL = (N + NTH - 1) / NTH;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {   // x_i = v_p, p = Makhoul position of i (i = tid + NTH c)
            const int i = tid + NTH * c;
            if (N % NTH != 0 && i >= N) continue;
            const int p = (i & 1) ? N - 1 - (i >> 1) : (i >> 1);
            const int pos = 2 * fft_pos<M1, M2>(p >> 1) + (p & 1);
#pragma unroll
            for (int l = 0; l < LPB; ++l)
                if (l < nl) out[((int64_t)xt_line_t(q, PP, Nt, l) * Ny + y) * N + i] = L[l * LS + pos] * iM;
        }
        __syncthreads();   // (the next chunk rewrites XL and L)
    }
}

static bool xt_supported(int Nx, int Nt) {
    int m1, m2;
    return Nt % 2 == 0 && Nt >= 2 && Nt <= 2 * XT_MAXH && Nx >= 64 && Nx <= XT_MAXN && fft_factors(Nx, &m1, &m2);
}

// the fused (x, t) forward / (t, x) inverse of a single shard's [t][y][x] volume <-> [kt][y][kx]
static hipError_t dct_xt(int Nt, int Ny, int Nx, bool inv, const double* tab, const double* Ch, const double* in,
                         double* out, hipStream_t s) {
#define FOTO_XT_LAUNCH(NN, A, B)                                                                              \
    if constexpr (NN >= 64 && NN <= XT_MAXN) {                                                                \
        if (Nx == NN) {                                                                                       \
            if (inv) k_dct_tx_inv<A, B><<<Ny, XT_NTH, 0, s>>>(Nt, Ny, tab, Ch, in, out);                      \
            else k_dct_xt_fwd<A, B><<<Ny, XT_NTH, 0, s>>>(Nt, Ny, tab, Ch, in, out);                          \
            return hipGetLastError();                                                                         \
        }                                                                                                     \
    }
    FOTO_FFT_SIZES(FOTO_XT_LAUNCH)
#undef FOTO_XT_LAUNCH
    return hipErrorNotSupported;
}


// ============================================================================ CG in the eigenbasis

// The spectral box a shard owns: all kt, rows ky in [y0, y0 + nyl), all kx; laid out
// [kt][ky - y0][kx] (single shard: the whole grid, y0 = 0, nyl = Ny).
struct SpecTab {
    const double* mt;   // mu_t[kt]
    const double* my;   // mu_y[ky]
    const double* mx;   // mu_x[kx]
    double r, reps;     // r, r * eps
    int Nt, Ny, Nx;
    int y0, nyl;
};

__device__ __forceinline__ double spec_lam(const SpecTab& T, double rowmu, int kx) {
    return T.reps + T.r * (rowmu + T.mx[kx]);
}

// tile = 4 rows x 128 columns; thread (tx, ty) owns columns 2tx, 2tx+1 of row ty.
// f(i, lam0, lam1, n2): elements i and i+1 (n2 = number valid: 1 or 2).  With Nx even,
// i is even and both elements are 16-B aligned (one dwordx4 per lane).
template <class F>
__device__ __forceinline__ void spec_for_each(const SpecTab& T, F f) {
    const int rows = T.Nt * T.nyl;
    const int ntx = (T.Nx + 127) / 128;
    const int ntiles = ntx * ((rows + 3) / 4);
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int row = (t / ntx) * 4 + ty;
        const int kx = (t % ntx) * 128 + 2 * tx;
        if (row >= rows || kx >= T.Nx) continue;
        const int kt = row / T.nyl, ky = T.y0 + (row - kt * T.nyl);
        const double rowmu = T.mt[kt] + T.my[ky];
        const int64_t i = (int64_t)row * T.Nx + kx;
        const int n2 = (kx + 1 < T.Nx) ? 2 : 1;
        f(i, spec_lam(T, rowmu, kx), n2 == 2 ? spec_lam(T, rowmu, kx + 1) : 1.0, n2);
    }
}

template <bool VEC>
__device__ __forceinline__ void ld2(const double* p, int64_t i, int n2, double& a, double& b) {
    if (VEC && n2 == 2) {
        const dbl2 v = *reinterpret_cast<const dbl2*>(p + i);
        a = v[0];
        b = v[1];
    } else {
        a = p[i];
        b = (n2 == 2) ? p[i + 1] : 0.0;
    }
}

template <bool VEC>
__device__ __forceinline__ void st2(double* p, int64_t i, int n2, double a, double b) {
    if (VEC && n2 == 2) {
        *reinterpret_cast<dbl2*>(p + i) = dbl2{a, b};
    } else {
        p[i] = a;
        if (n2 == 2) p[i + 1] = b;
    }
}

// r^ = b^; partials (r.r, r.lam.r) -> gath[0..1]
template <bool VEC>
__global__ __launch_bounds__(NT) void k_spec_init(SpecTab T, const double* __restrict__ bh, double* __restrict__ rh,
                                                  RedBuf rb, double* gath) {
    double a0 = 0.0, a1 = 0.0;
    spec_for_each(T, [&](int64_t i, double l0, double l1, int n2) {
        double b0, b1;
        ld2<VEC>(bh, i, n2, b0, b1);
        st2<VEC>(rh, i, n2, b0, b1);
        a0 += b0 * b0;
        a1 += l0 * (b0 * b0);
        if (n2 == 2) {
            a0 += b1 * b1;
            a1 += l1 * (b1 * b1);
        }
    });
    double v[2] = {a0, a1}, tot[2];
    if (sp_reduce_last<2>(v, rb, tot) && threadIdx.x == 0) { gath[0] = tot[0]; gath[1] = tot[1]; }
}

// One CG iteration k (Chronopoulos-Gear): given rho_k = r.r and m_k = r.lam.r (gathered),
//   stop if ||r_k|| < atol (scipy's top-of-loop test); beta = rho_k / rho_{k-1};
//   p.Ap = m_k - beta rho_k / alpha_{k-1} (k > 0), = m_0 (k = 0); alpha = rho_k / p.Ap;
//   p = beta p + r;  r = r - alpha (lam p);  partials (r.r, r.lam.r) of r_{k+1}.
template <bool VEC>
__global__ __launch_bounds__(NT) void k_spec_cg(SpecTab T, int k, double* __restrict__ rh, double* __restrict__ ph,
                                                CGScal* S, RedBuf rb, double* gath, double rtol) {
    if (S->done) return;
    const double rho = gath[0], mk = gath[1];
    double atol, beta = 0.0, pap;
    if (k == 0) {
        atol = fmax(0.0, rtol * sqrt(rho));
        if (rho == 0.0) {
            if (blockIdx.x == 0 && threadIdx.x == 0) { S->done = 1; S->iters = 0; }
            return;
        }
        pap = mk;
    } else {
        atol = S->atol;
        beta = rho / S->rho;
        pap = mk - beta * rho / S->pap;   // S->pap holds alpha_{k-1}
    }
    if (sqrt(rho) < atol) {
        if (blockIdx.x == 0 && threadIdx.x == 0) { S->done = 1; S->iters = k; }
        return;
    }
    const double alpha = rho / pap;
    double a0 = 0.0, a1 = 0.0;
    spec_for_each(T, [&](int64_t i, double l0, double l1, int n2) {
        double r0, r1, p0 = 0.0, p1 = 0.0;
        ld2<VEC>(rh, i, n2, r0, r1);
        if (k > 0) ld2<VEC>(ph, i, n2, p0, p1);
        p0 = (k == 0) ? r0 : beta * p0 + r0;
        p1 = (k == 0) ? r1 : beta * p1 + r1;
        const double n0 = r0 - alpha * (l0 * p0);
        const double n1 = r1 - alpha * (l1 * p1);
        st2<VEC>(ph, i, n2, p0, p1);
        st2<VEC>(rh, i, n2, n0, n1);
        a0 += n0 * n0;
        a1 += l0 * (n0 * n0);
        if (n2 == 2) {
            a0 += n1 * n1;
            a1 += l1 * (n1 * n1);
        }
    });
    double v[2] = {a0, a1}, tot[2];
    if (sp_reduce_last<2>(v, rb, tot) && threadIdx.x == 0) {
        S->rho = rho;
        S->pap = alpha;
        if (k == 0) { S->atol = atol; S->bb = rho; }
        gath[0] = tot[0];
        gath[1] = tot[1];
    }
}

// x^ = (b^ - r^) / lam
template <bool VEC>
__global__ __launch_bounds__(NT) void k_spec_xhat(SpecTab T, const double* __restrict__ bh,
                                                  const double* __restrict__ rh, double* __restrict__ xh) {
    spec_for_each(T, [&](int64_t i, double l0, double l1, int n2) {
        double b0, b1, r0, r1;
        ld2<VEC>(bh, i, n2, b0, b1);
        ld2<VEC>(rh, i, n2, r0, r1);
        st2<VEC>(xh, i, n2, (b0 - r0) / l0, (b1 - r1) / l1);
    });
}

// ============================================================================ s-step CG in the eigenbasis
//
// One pass = up to SMAX CG iterations.  State between passes: r = r_k, q = p_{k-1}.  The
// pass applies the planned steps pointwise (p = beta q + r; r -= alpha lam p; q = p --
// scipy's per-element recurrence) with scalars prepared by the previous pass, then
// accumulates the Chebyshev moments of the NEW state,
//     M^rr_m = sum T_m(x) r^2,  M^rq_m = sum T_m(x) r q,  M^qq_m = sum T_m(x) q^2,
//     x = (lam - c0) / c1 in [-1, 1],  m = 0 .. 2 SMAX - 1,
// from which one wavefront of the last block plans the next pass: r_{k+i} = A_i(lam) r +
// B_i(lam) q with Chebyshev-coefficient polynomials, inner products through the Gram matrix
// (M_{a+c} + M_{|a-c|}) / 2.  Step i > 0 is taken only while its two Gram-form inner
// products (rho_{k+i} and p.Ap) are well conditioned: sum |terms| / |result| <= S_CLIM
// (3e4, i.e. ~3e-12 relative rounding; DESIGN.md 3.1.1 has the sweep).  Early in a solve
// the residual measure is a few dominant low-frequency components, the Chebyshev-Krylov basis is nearly degenerate and
// passes take 1-2 steps; later ones take SMAX.  A fixed s >= 3 loses digits in the first
// passes (measured: alpha off by 1e-4 at s = 3, k = 0).  tests/test_sstep_plan.py checks
// the planning rule (numpy restatement) against the golden solves: the same CG counts as
// scipy; at 640x480x32, 24 passes for 147 iterations (s = 2: 74).

#ifndef FOTO_SMAX
#define FOTO_SMAX 8
#endif
constexpr int SMAX = FOTO_SMAX;      // max CG steps per pass
constexpr int NMOM = 2 * SMAX;       // moments per family: degrees 0 .. 2 SMAX - 1
constexpr int NACC = 3 * NMOM;       // rr, rq, qq
constexpr int NCO = SMAX + 1;        // Chebyshev coefficients per part (degree <= SMAX)
constexpr int NG = 2 * NCO;          // combined (r part, q part) coefficient index
#ifndef FOTO_S_CLIM
#define FOTO_S_CLIM 3e4
#endif
constexpr double S_CLIM = FOTO_S_CLIM;   // cancellation limit of a Gram-form inner product
static_assert(NG <= 64, "coefficients live one per lane");

struct SStep {
    int k;        // iterations applied so far
    int nsteps;   // steps the next pass applies (0 .. SMAX)
    int fin;      // after applying nsteps the solve is finished
    int conv;     // ... because the stop test passed (else: maxiter reached)
    int done;     // 1 converged, 2 maxiter reached (host polls this)
    int iters;    // iterations at finish
    int passes;   // plans made in this solve
    int flags;    // bit 0: no interval adaptation (A/B runs, FOTO_SADAPT=0)
    int pend;     // the moments in gath await their plan (made at the start of the next pass)
    int pad_;
    double a[SMAX], b[SMAX];
    double rho_prev;   // rho_{k-1}
    double atol;
    double c0, c1;     // Chebyshev interval of the next pass's moments: lam in [c0 - c1, c0 + c1]
    double gc0, gc1;   // the whole spectrum's interval (fixed)
    double ic0, ic1;   // interval of the next solve's INIT moments (set by each INIT plan)
};

// Interval adaptation: the Chebyshev-Krylov basis is well conditioned when [c0 - c1, c0 + c1]
// spans where the residual measure sum r^2 delta(lam) has its weight.  Early in a solve that
// weight sits at low frequencies and the full-spectrum basis is nearly degenerate (passes of
// 1-2 steps); so the plan sets the next pass's interval to [lmin, min(lmax, mean + S_KAPPA sd)]
// of the measure of the state it just received (from M_0..M_2 of the rr family).  Elements
// above the interval get |x| > 1 (large T_m); the cancellation rule keeps every planned step
// accurate regardless.  Measured (numpy restatement, tests/test_sstep_plan.py): at the bench
// grid 24 -> 22 passes on the first outer iteration, 33 -> 28 at 160x120x32; no change in
// CG counts or iterates.
#ifndef FOTO_S_KAPPA
#define FOTO_S_KAPPA 2.0
#endif
constexpr double S_KAPPA = FOTO_S_KAPPA;
constexpr int S_PROJ = (NMOM - 3) / 2;   // projected interval after n <= S_PROJ steps (2n + 2 < NMOM)

// Plan helpers.  Coefficient vectors are distributed one entry per lane: lane j < NG holds
// index j of (r part | q part), lanes >= NG hold 0; lane j also holds row j of the Gram
// matrix H.  Cross-lane traffic goes through the planning wave's LDS buffer xb (one
// ds_write per lane, broadcast reads); one wave, so ordering only needs the
// write-completion wait.
#define FOTO_LDS_WAIT() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// <U, V> = sum_j U_j (H V)_j and whether its cancellation ratio sum |terms| / |<U, V>| is
// within S_CLIM (*cratio = 1, else infinity; tested as sum|terms| <= S_CLIM |<U, V>|); lanes 0 and
// 1 sum the NG lane values (value, |terms|) in lane order, every lane reads the result.
__device__ __forceinline__ double plan_ip(double U, double V, const double (&hrow)[NG], double* xb, double* cratio) {
    const int lane = threadIdx.x & 63;
    if (lane < NG) xb[lane] = V;
    FOTO_LDS_WAIT();
    double w0 = 0.0, w1 = 0.0, a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int c = 0; c < NG; c += 2) {
        const double t0 = hrow[c] * xb[c];
        const double t1 = (c + 1 < NG) ? hrow[c + 1] * xb[c + 1] : 0.0;
        w0 += t0;
        w1 += t1;
        a0 += fabs(t0);
        a1 += fabs(t1);
    }
    FOTO_LDS_WAIT();
    if (lane < NG) {
        xb[NG + lane] = U * (w0 + w1);
        xb[2 * NG + lane] = fabs(U) * (a0 + a1);
    }
    FOTO_LDS_WAIT();
    if (lane < 2) {
        const double* src = xb + NG + lane * NG;
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int j = 0; j < NG; j += 2) {
            s0 += src[j];
            if (j + 1 < NG) s1 += src[j + 1];
        }
        FOTO_LDS_WAIT();
        xb[3 * NG + lane] = s0 + s1;
    }
    FOTO_LDS_WAIT();
    const double s = xb[3 * NG], sa = xb[3 * NG + 1];
    FOTO_LDS_WAIT();
    *cratio = (s != 0.0 && sa <= S_CLIM * fabs(s)) ? 1.0 : INFINITY;   // (no division)
    return s;
}

// lam U = c0 U + c1 x U, x T_0 = T_1, x T_m = (T_{m+1} + T_{m-1}) / 2 within each part; the
// top coefficient is never multiplied (its degree would exceed SMAX; it is zero whenever
// this is called).
__device__ __forceinline__ double plan_mul_lam(double U, double c0, double c1, double* xb) {
    const int lane = threadIdx.x & 63;
    if (lane < NG) xb[lane] = U;
    FOTO_LDS_WAIT();
    const int pb = (lane < NCO) ? 0 : NCO, m = lane - pb;
    double X = 0.0;
    if (lane < NG) {
        if (m == 1) X += xb[pb];
        if (m >= 2) X += 0.5 * xb[lane - 1];
        if (m <= NCO - 3) X += 0.5 * xb[lane + 1];
    }
    FOTO_LDS_WAIT();
    return (lane < NG) ? c0 * U + c1 * X : 0.0;
}

// Register-only variants (FOTO_PLAN_DPP): V broadcast by v_readlane into SGPRs, the |terms|
// sums by FMA with |.| operand modifiers, lane sums by a DPP row_shr tree (lanes 15 and 31
// hold the row totals), neighbours for lam U by DPP wave shifts -- no LDS round trip.
#ifndef FOTO_PLAN_DPP
#define FOTO_PLAN_DPP 1
#endif

__device__ __forceinline__ double dbl_readlane(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int CTRL>
__device__ __forceinline__ double dbl_dpp(double v) {   // lanes without a source read 0
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// sum over lanes 0 .. 31 (lanes >= NG hold 0), uniform result: row_shr 1, 2, 4, 8 tree
__device__ __forceinline__ double dpp_sum32(double v) {
    v += dbl_dpp<0x111>(v);
    v += dbl_dpp<0x112>(v);
    v += dbl_dpp<0x114>(v);
    v += dbl_dpp<0x118>(v);
    return dbl_readlane(v, 15) + dbl_readlane(v, 31);
}

// nc: V's coefficients of degree >= nc are zero in both parts (step i of a plan: R has degree
// i, lam Pn degree i + 1); with the step loop unrolled nc is a constant and the zero columns
// cost nothing (about half the broadcasts and FMAs of a plan).
__device__ __forceinline__ double plan_ip_dpp(double U, double V, const double (&hrow)[NG], double* cratio,
                                              int nc = NCO) {
    double w0 = 0.0, w1 = 0.0, a0 = 0.0, a1 = 0.0;
    int j = 0;
#pragma unroll
    for (int c = 0; c < NG; ++c) {
        if (c % NCO >= nc) continue;
        const double v = dbl_readlane(V, c);
        if (j++ % 2 == 0) {
            w0 = fma(hrow[c], v, w0);
            a0 = fma(fabs(hrow[c]), fabs(v), a0);
        } else {
            w1 = fma(hrow[c], v, w1);
            a1 = fma(fabs(hrow[c]), fabs(v), a1);
        }
    }
    const double s = dpp_sum32(U * (w0 + w1));
    const double sa = dpp_sum32(fabs(U) * (a0 + a1));
    *cratio = (s != 0.0 && sa <= S_CLIM * fabs(s)) ? 1.0 : INFINITY;   // (no division)
    return s;
}

// FOTO_PLAN_DPP == 2: V broadcast through LDS instead (one ds_write, NG/2 broadcast
// ds_read_b128; the LDS pipe instead of 2 NG v_readlane VALU ops and their hazards).
__device__ __forceinline__ double plan_ip_lds(double U, double V, const double (&hrow)[NG], double* xb,
                                              double* cratio) {
    const int lane = threadIdx.x & 63;
    if (lane < NG) xb[lane] = V;   // one wave: its LDS operations complete in order
    double w0 = 0.0, w1 = 0.0, a0 = 0.0, a1 = 0.0;
#pragma unroll
    for (int c = 0; c < NG; c += 2) {
        const dbl2 v = *reinterpret_cast<const dbl2*>(xb + c);
        w0 = fma(hrow[c], v[0], w0);
        a0 = fma(fabs(hrow[c]), fabs(v[0]), a0);
        w1 = fma(hrow[c + 1], v[1], w1);
        a1 = fma(fabs(hrow[c + 1]), fabs(v[1]), a1);
    }
    const double s = dpp_sum32(U * (w0 + w1));
    const double sa = dpp_sum32(fabs(U) * (a0 + a1));
    *cratio = (s != 0.0 && sa <= S_CLIM * fabs(s)) ? 1.0 : INFINITY;   // (no division)
    return s;
}
static_assert(NG % 2 == 0, "pairs of coefficients per broadcast read");

__device__ __forceinline__ double plan_mul_lam_dpp(double U, double c0, double c1) {
    const int lane = threadIdx.x & 63;
    const double um = dbl_dpp<0x138>(U);   // wave_shr:1 -> U[lane - 1]
    const double up = dbl_dpp<0x130>(U);   // wave_shl:1 -> U[lane + 1]
    const int pb = (lane < NCO) ? 0 : NCO, m = lane - pb;
    double X = 0.0;
    if (lane < NG) {
        if (m == 1) X += um;
        if (m >= 2) X += 0.5 * um;
        if (m <= NCO - 3) X += 0.5 * up;
    }
    return (lane < NG) ? c0 * U + c1 * X : 0.0;
}

// Finish the pass's bookkeeping and plan the next pass (scipy's loop: top-of-iteration test
// ||r|| < atol, then p = beta p + r, alpha = rho / p.Ap, r -= alpha A p).  Called by all 64
// lanes of one wave with the same S (state at the start of the pass) and the summed
// moments tot[NACC] (shared); lane 0 stores the new state.
#ifdef FOTO_PLAN_CLOCK   // timing studies only (tools/pass_lab.hip): 100 MHz stamps of block 0
__device__ long long foto_plan_clock[8];
#define FOTO_PLAN_STAMP(k) \
    if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) foto_plan_clock[k] = wall_clock64()
#else
#define FOTO_PLAN_STAMP(k)
#endif

// n / d on the plan's critical chain: v_rcp_f64, one Newton step and one residual correction (5
// dependent FMAs instead of the ~10-instruction IEEE division sequence; within an ulp of n / d)
#ifndef FOTO_PLAN_RCP
#define FOTO_PLAN_RCP 0
#endif
__device__ __forceinline__ double plan_div(double n, double d) {
#if FOTO_PLAN_RCP
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    const double q = n * r;
    return fma(fma(-d, q, n), r, q);
#else
    return n / d;
#endif
}

__device__ void sstep_plan_wave(SStep* Sg, SStep S, const double* tot, double* xb /* shared, 3 NG + 2 */, int init,
                                double rtol, int maxiter) {
    const int lane = threadIdx.x & 63;
    if (init) {
        S.c0 = S.ic0;   // the interval the INIT moments were taken over
        S.c1 = S.ic1;
        S.k = 0;
        S.rho_prev = 0.0;
        S.atol = fmax(0.0, rtol * sqrt(tot[0]));   // scipy: max(atol, rtol * ||b||)
        S.done = 0;
        S.passes = 0;
    } else {
        S.k += S.nsteps;
        if (S.fin) {
            S.done = S.conv ? 1 : 2;
            S.nsteps = 0;
            S.pend = 0;
            if (lane == 0) *Sg = S;
            return;
        }
    }
    // row `lane` of H[a][c] = <T_a u, T_c v>, u, v in {r, q} by part: (M_{a+c} + M_{|a-c|}) / 2
    // of family rr / rq / qq (degrees >= NMOM are never needed)
    double hrow[NG];
    {
        const int a = lane < NG ? lane : 0, ia = a % NCO, pa = a / NCO;
#pragma unroll
        for (int c = 0; c < NG; ++c) {
            const int ic = c % NCO, fam = pa + c / NCO;
            const double* M = tot + fam * NMOM;
            hrow[c] = (lane < NG && ia + ic < NMOM) ? 0.5 * (M[ia + ic] + M[ia > ic ? ia - ic : ic - ia]) : 0.0;
        }
    }
    FOTO_PLAN_STAMP(3);
    double R = (lane == 0) ? 1.0 : 0.0;     // r_k     = 1 * r
    double P = (lane == NCO) ? 1.0 : 0.0;   // p_{k-1} = 1 * q
    double rho_prev = S.rho_prev;
    int n = 0;
    bool conv = false;
    double av = 0.0, bv = 0.0;   // lane i: step i's alpha, beta (stored after the loop)
    // wave-uniform tests as scalar branches (the values are uniform; the compiler cannot see it)
    auto uni = [](bool b) { return __builtin_amdgcn_readfirstlane(b ? 1 : 0) != 0; };
#pragma clang loop unroll(full)
    for (int i = 0; i < SMAX; ++i) {
        if (S.k + i >= maxiter) break;
        double rho, cr = 0.0;
        if (i == 0) rho = tot[0];
        else {
#if FOTO_PLAN_DPP == 2
            rho = plan_ip_lds(R, R, hrow, xb, &cr);
#elif FOTO_PLAN_DPP
            rho = plan_ip_dpp(R, R, hrow, &cr, i + 1);
#else
            rho = plan_ip(R, R, hrow, xb, &cr);
#endif
            if (uni(!(cr <= 1.0))) break;   // badly conditioned (or NaN): leave it to the next pass
        }
        if (uni(rho == 0.0 || sqrt(rho) < S.atol)) { conv = true; break; }
        const bool first = (S.k + i == 0);
        const double beta = first ? 0.0 : plan_div(rho, rho_prev);
        const double Pn = first ? R : beta * P + R;
#if FOTO_PLAN_DPP == 2
        const double Q = plan_mul_lam_dpp(Pn, S.c0, S.c1);
        const double den = plan_ip_lds(Pn, Q, hrow, xb, &cr);
#elif FOTO_PLAN_DPP
        const double Q = plan_mul_lam_dpp(Pn, S.c0, S.c1);
        const double den = plan_ip_dpp(Pn, Q, hrow, &cr, i + 2);
#else
        const double Q = plan_mul_lam(Pn, S.c0, S.c1, xb);
        const double den = plan_ip(Pn, Q, hrow, xb, &cr);
#endif
        if (i > 0 && uni(!(cr <= 1.0))) break;
        const double alpha = plan_div(rho, den);
        R = R - alpha * Q;
        P = Pn;
        rho_prev = rho;
        av = (lane == i) ? alpha : av;
        bv = (lane == i) ? beta : bv;
        ++n;
    }
    if (lane < n) {
        Sg->a[lane] = av;
        Sg->b[lane] = bv;
    }
    FOTO_PLAN_STAMP(4);
    S.nsteps = n;
    S.rho_prev = rho_prev;
    S.passes += 1;
    S.fin = 0;
    S.conv = conv ? 1 : 0;
    if (conv || S.k + n >= maxiter) {
        S.fin = 1;
        S.iters = conv ? S.k + n : maxiter;
        if (n == 0) S.done = conv ? 1 : 2;   // nothing left to apply
    }
    // Next pass's interval.  After n <= S_PROJ steps the plan knows the new residual's
    // coefficients R, so the mean and variance of its measure are Gram forms
    // (<R, lam R>, <lam R, lam R> over <R, R>; degrees <= 2n + 2 < NMOM); after more steps
    // it falls back to the measure these moments describe (one pass behind).  An INIT plan
    // also sets the next solve's INIT interval from the measure of b^ (consecutive outer
    // iterations' right-hand sides are close).
    const double lmin = S.gc0 - S.gc1, lmax = S.gc0 + S.gc1;
    auto to_interval = [&](double mean, double var, double& c0o, double& c1o) {
        double hi = fmin(lmax, mean + S_KAPPA * sqrt(fmax(var, 0.0)));
        hi = fmax(hi, lmin + 1e-3 * (lmax - lmin));
        if (hi == hi) {   // not NaN
            c0o = 0.5 * (hi + lmin);
            c1o = 0.5 * (hi - lmin);
        }
    };
    double nc0 = S.c0, nc1 = S.c1, ic0 = S.ic0, ic1 = S.ic1;
    double mom_mean = 0.0, mom_var = -1.0;   // the moments' own measure
    if (tot[0] > 0.0) {
        const double ex = tot[1] / tot[0], ex2 = 0.5 * (tot[2] + tot[0]) / tot[0];
        mom_mean = S.c0 + S.c1 * ex;
        mom_var = S.c1 * S.c1 * (ex2 - ex * ex);
    }
    const bool adapt = !(S.flags & 1);
    if (adapt && init && mom_var >= 0.0) to_interval(mom_mean, mom_var, ic0, ic1);
    bool projected = false;
    if (adapt && n > 0 && n <= S_PROJ && !S.fin) {
        double c1r, c2r, c3r;
#if FOTO_PLAN_DPP
        const double LR = plan_mul_lam_dpp(R, S.c0, S.c1);
        const double rr = plan_ip_dpp(R, R, hrow, &c1r, n + 1);
        const double rl = plan_ip_dpp(R, LR, hrow, &c2r, n + 2);
        const double ll = plan_ip_dpp(LR, LR, hrow, &c3r, n + 2);
#else
        const double LR = plan_mul_lam(R, S.c0, S.c1, xb);
        const double rr = plan_ip(R, R, hrow, xb, &c1r);
        const double rl = plan_ip(R, LR, hrow, xb, &c2r);
        const double ll = plan_ip(LR, LR, hrow, xb, &c3r);
#endif
        if (rr > 0.0) {
            const double mean = rl / rr;
            to_interval(mean, ll / rr - mean * mean, nc0, nc1);
            projected = true;
        }
    }
    if (adapt && !projected && mom_var >= 0.0) to_interval(mom_mean, mom_var, nc0, nc1);
    FOTO_PLAN_STAMP(5);
    if (lane == 0) {   // scalars only: a[], b[] were stored above
        Sg->k = S.k; Sg->nsteps = S.nsteps; Sg->fin = S.fin; Sg->conv = S.conv; Sg->done = S.done;
        Sg->iters = S.iters; Sg->passes = S.passes; Sg->rho_prev = S.rho_prev; Sg->atol = S.atol;
        Sg->c0 = nc0; Sg->c1 = nc1; Sg->ic0 = ic0; Sg->ic1 = ic1; Sg->pend = 0;
    }
}

// element pair of tile t owned by this thread (see spec_for_each); n2 = 0: none
struct SpElem {
    int64_t i;
    double l0, l1;
    int n2;
};

template <int TR>
__device__ __forceinline__ SpElem spec_elem(const SpecTab& T, int t, int ntx, int rows) {
    SpElem e;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const int row = (t / ntx) * TR + ty;
    const int kx = (t % ntx) * 128 + 2 * tx;
    e.n2 = 0;
    e.i = 0;
    e.l0 = e.l1 = 1.0;
    if (row < rows && kx < T.Nx) {
        const int kt = row / T.nyl, ky = T.y0 + (row - kt * T.nyl);
        const double rowmu = T.mt[kt] + T.my[ky];
        e.i = (int64_t)row * T.Nx + kx;
        e.n2 = (kx + 1 < T.Nx) ? 2 : 1;
        e.l0 = spec_lam(T, rowmu, kx);
        e.l1 = (e.n2 == 2) ? spec_lam(T, rowmu, kx + 1) : 1.0;
    }
    return e;
}

// gath == nullptr (FUSE): single shard, the last block plans the next pass itself.
// Otherwise the last block stores this shard's moments at gath[rank * NACC]; after the
// all-gather, k_spec_s2_plan sums them in rank order and plans (identically on every rank).
// 1024 threads: one block per CU at the pass's occupancy (4 waves / SIMD), so the
// cross-block tail gathers 48 x 256 partials in one round trip (with 256-thread blocks it
// was 48 x 1024 in six: 14 us of each pass, tools/s2_ablation.hip).
// Occupancy of the pass kernels follows the accumulator count: 2 SMAX x 3 fp64 moments per
// thread = 12 SMAX VGPRs (96 at SMAX 8: 4 waves/SIMD in <= 128; 120 at 10: 3 waves in <= 168;
// 144 at 12: 2 waves), and a block is one CU's worth of waves (one block per CU).
#ifndef FOTO_S2_WPE
#define FOTO_S2_WPE (SMAX <= 8 ? 4 : (SMAX <= 10 ? 3 : 2))
#endif
constexpr int S2_WPE = FOTO_S2_WPE;                              // waves per SIMD
constexpr int S2_NTH = 256 * S2_WPE;                            // threads per block of the s-step pass

// 4 waves / SIMD: the streaming body needs the occupancy; the fused plan must fit beside it.
template <bool VEC, bool INIT, bool FUSE>
__global__ __launch_bounds__(S2_NTH) __attribute__((amdgpu_waves_per_eu(S2_WPE))) void k_spec_s2(SpecTab T, double* __restrict__ rh, double* __restrict__ ph,
                                                    const double* __restrict__ bh, SStep* Sg, RedBuf rb,
                                                    double rtol, int maxiter, double* gath, int rank) {
    constexpr int TR = S2_NTH / 64;   // tile = TR rows x 128 columns
    const SStep S0 = *Sg;             // uniform: scalar loads
    if (!INIT && (S0.done || S0.nsteps == 0)) return;
    const int k = S0.k, ns = INIT ? 0 : S0.nsteps;
    const double c0 = INIT ? S0.ic0 : S0.c0, ic1 = 1.0 / (INIT ? S0.ic1 : S0.c1);
    const bool loadq = !INIT && k > 0;
    // r_0 = b^: the INIT pass (or the fused t-axis kernel, which writes no r^) leaves it in b^
    const double* src = (INIT || k == 0) ? bh : rh;
    double acc[NACC];
#pragma unroll
    for (int m = 0; m < NACC; ++m) acc[m] = 0.0;
    auto moments = [&](double lam, double r, double q) {
        const double x = (lam - c0) * ic1, x2 = x + x;
        const double rr = r * r, rq = r * q, qq = q * q;
        acc[0] += rr;
        acc[NMOM] += rq;
        acc[2 * NMOM] += qq;
        acc[1] = fma(x, rr, acc[1]);
        acc[NMOM + 1] = fma(x, rq, acc[NMOM + 1]);
        acc[2 * NMOM + 1] = fma(x, qq, acc[2 * NMOM + 1]);
        double tm2 = 1.0, tm1 = x;
#pragma unroll
        for (int m = 2; m < NMOM; ++m) {
            const double t = fma(x2, tm1, -tm2);
            acc[m] = fma(t, rr, acc[m]);
            acc[NMOM + m] = fma(t, rq, acc[NMOM + m]);
            acc[2 * NMOM + m] = fma(t, qq, acc[2 * NMOM + m]);
            tm2 = tm1;
            tm1 = t;
        }
    };
    const int rows = T.Nt * T.nyl;
    const int ntx = (T.Nx + 127) / 128;
    const int ntiles = ntx * ((rows + TR - 1) / TR);
    // A plain grid-stride tile loop: software-pipelining it (next tile's loads issued first)
    // measured no faster at SMAX = 6 and spills at SMAX = 8 (tools/s2_ablation.hip).
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const SpElem e = spec_elem<TR>(T, t, ntx, rows);
        if (!e.n2) continue;
        double r0, r1, q0 = 0.0, q1 = 0.0;
        ld2<VEC>(src, e.i, e.n2, r0, r1);
        if (loadq) ld2<VEC>(ph, e.i, e.n2, q0, q1);
        if (INIT) {
            st2<VEC>(rh, e.i, e.n2, r0, r1);
        } else {
#pragma clang loop unroll(full)
            for (int i = 0; i < SMAX; ++i) {
#if defined(FOTO_S2_ABLATE) && FOTO_S2_ABLATE == 2
                if (i >= 1) continue;
#endif
                if (i < ns) {   // guard, not break: keeps the loop fully unrolled (S0 out of scratch)
                    // iteration k + i: p = beta p + r (p = r at k = 0); r -= alpha (lam p)
                    const double a = S0.a[i], b = S0.b[i];
                    // (k + i = 0: b = 0 and q = 0, so p = r)
                    const double p0 = fma(b, q0, r0);
                    const double p1 = fma(b, q1, r1);
                    r0 = fma(-a, e.l0 * p0, r0);
                    r1 = fma(-a, e.l1 * p1, r1);
                    q0 = p0;
                    q1 = p1;
                }
            }
            st2<VEC>(rh, e.i, e.n2, r0, r1);
            st2<VEC>(ph, e.i, e.n2, q0, q1);
        }
#if defined(FOTO_S2_ABLATE) && (FOTO_S2_ABLATE == 1 || FOTO_S2_ABLATE == 4)   // timing studies only
        acc[0] += r0 * q0 + r1 * q1;
#else
        moments(e.l0, r0, q0);
        if (e.n2 == 2) moments(e.l1, r1, q1);
#endif
    }
    __shared__ double tot[NACC];
#if defined(FOTO_S2_ABLATE) && (FOTO_S2_ABLATE == 3 || FOTO_S2_ABLATE == 4)   // timing studies only: no reduction
    {
        double sacc = 0.0;
        for (int m = 0; m < NACC; ++m) sacc += acc[m];
        if (sacc == 1.2345) gath[0] = sacc;
        return;
    }
#endif
    if (!sp_reduce_last_rs<NACC, S2_NTH>(acc, rb, tot)) return;
    if (!FUSE) {
        for (int m = threadIdx.x; m < NACC; m += S2_NTH) gath[rank * NACC + m] = tot[m];
        return;
    }
    if (threadIdx.x >= 64) return;
    __shared__ __attribute__((aligned(16))) double xb[3 * NG + 2];
    sstep_plan_wave(Sg, S0, tot, xb, INIT ? 1 : 0, rtol, maxiter);
}

// ---------------------------------------------------------------------------- ring-fed pass
// The same pass with r, q streamed through a per-wave LDS ring by LDS-DMA
// (global_load_lds_dwordx4): each wave walks its own sequence of 128-column row segments
// ("wave tiles") and keeps D of them in flight, so a CU holds up to 16 x (D - 1) x 2 KiB of
// loads in flight without spending VGPRs on them (the register-fed pass, 121 VGPRs for the
// 48 moment accumulators, holds one tile per wave: ~32 KiB per CU, too little to cover the
// HBM latency under load -- it streamed at ~4.3 TB/s).  Counting: VMEM operations complete
// in issue order on gfx950 (stores included), so before reading tile j the wave waits until
// at most K operations are outstanding, K = those issued after tile j's loads.  The ring is
// read with inline-asm ds_read (invisible to hipcc's waitcnt pass, which would otherwise wait
// for the newest DMA), and the loop has no other vector-memory loads: the mu tables are
// staged in LDS before the pipeline starts (an ordinary load would complete behind every
// DMA in flight).  Per element the arithmetic is the register-fed pass's, in the same order:
// r, q are bit-identical; only the moment summation order differs (element-to-thread map).
// Ring depth: what the LDS left after the tables (18 KiB) and the reduction scratch allows
// (16 waves x 4 x 2 KiB at SMAX 8, 12 x 5 at 10, 8 x 8 at 12).
#ifndef FOTO_RING_D
#define FOTO_RING_D (S2_WPE == 4 ? 4 : (S2_WPE == 3 ? 5 : 8))
#endif
constexpr int RING_NW = S2_NTH / 64;    // waves per block
constexpr int RING_SLOT = 256;          // doubles per ring slot: r (128) then q (128)
constexpr int RING_TAB = 2304;          // mu_x, mu_t, mu_y (own rows) staged in LDS (doubles)
typedef __attribute__((address_space(3))) void lds_void_t;

__device__ __forceinline__ unsigned lds_u32(const void* p) { return (unsigned)(uintptr_t)(const lds_void_t*)p; }

__device__ __forceinline__ dbl2 lds_ld128(unsigned a) {   // caller waits lgkmcnt
    dbl2 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
    return v;
}
__device__ __forceinline__ double lds_ld64(unsigned a) {
    double v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a) : "memory");
    return v;
}

// wait until at most k vector-memory operations are outstanding (k wave-uniform; clamped)
template <int N>
__device__ __forceinline__ void vm_wait_imm() {
    static_assert(N >= 0 && N <= 63, "vmcnt range");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void vm_wait(int k) {
    switch (k) {
#define FOTO_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        FOTO_VMW(1) FOTO_VMW(2) FOTO_VMW(3) FOTO_VMW(4) FOTO_VMW(5) FOTO_VMW(6) FOTO_VMW(7) FOTO_VMW(8)
        FOTO_VMW(9) FOTO_VMW(10) FOTO_VMW(11) FOTO_VMW(12) FOTO_VMW(13) FOTO_VMW(14) FOTO_VMW(15)
        FOTO_VMW(16) FOTO_VMW(17) FOTO_VMW(18) FOTO_VMW(19) FOTO_VMW(20) FOTO_VMW(21) FOTO_VMW(22)
        FOTO_VMW(23) FOTO_VMW(24) FOTO_VMW(25) FOTO_VMW(26) FOTO_VMW(27) FOTO_VMW(28) FOTO_VMW(29)
        FOTO_VMW(30) FOTO_VMW(31)
#undef FOTO_VMW
        default:
            if (k > 31) asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

// Usable for a shard when Nx is even (16-B lanes) and the tables fit.  The flat tiling (Nx not
// a multiple of 128) also needs the box's element indices in 30 bits (32-bit element
// arithmetic; ring_divmod's quotients, at most Nt * nyl < 2^21 under the table bound, are
// exact); row-segment tiles index with 64-bit element offsets; the write-through stores take
// 32-bit byte offsets (a box under 4 GiB).
static inline bool ring_ok(const SpecTab& T) {
    const bool flat = (T.Nx % 128) != 0;
    return (T.Nx % 2) == 0 && T.Nx + T.Nt + T.nyl <= RING_TAB &&
           (!flat || (int64_t)T.Nt * T.nyl * T.Nx < (int64_t(1) << 30)) &&
           (!FOTO_PASS_WT || (int64_t)T.Nt * T.nyl * T.Nx * 8 < (int64_t(1) << 32));   // ring_store offsets
}

// Tables: mu_x [0, Nx), mu_t [Nx, Nx + Nt), mu_y of the own rows [Nx + Nt, + nyl).
// (first: the first thread taking part; a late-planning pass leaves wave 0 to its plan)
__device__ __forceinline__ void ring_stage_tables(const SpecTab& T, double* tab, int first = 0) {
    for (int i = (int)threadIdx.x - first; i >= 0 && i < T.Nx + T.Nt + T.nyl; i += S2_NTH - first)
        tab[i] = (i < T.Nx) ? T.mx[i] : (i < T.Nx + T.Nt) ? T.mt[i - T.Nx] : T.my[T.y0 + i - T.Nx - T.Nt];
}

// The wave's tile sequence: u = gw + j W (j < nj), u -> (row, 128-column segment cx) when the
// rows are whole tiles (Nx % 128 == 0); otherwise the box is tiled flat (tile u = elements
// [128 u, 128 u + 128) of the contiguous [t][y][x] box, rows found per lane), so row lengths
// like Middlebury's 584 (4.56 tiles) or 420 (3.28) leave no idle lanes in a last segment.
struct RingWave {
    int gw, W, nj, ntx;
    bool flat;
    int nel;         // elements of the box (flat tiling)
    double* wring;   // this wave's D slots
};

// floor(e / n) and the remainder, 0 <= e < 2^30, quotient < 2^21: the fp32 estimate is off by
// less than (e / n) 2^-21.7 + 1 < 2, and one correction each way makes it exact
__device__ __forceinline__ int ring_divmod(int e, int n, float inv, int* rem) {
    int q = (int)((float)e * inv);
    int r = e - q * n;
    if (r < 0) { --q; r += n; }
    else if (r >= n) { ++q; r -= n; }
    *rem = r;
    return q;
}

__device__ __forceinline__ RingWave ring_wave(const SpecTab& T, double* ring, int D) {
    RingWave w;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int rows = T.Nt * T.nyl;
    w.ntx = (T.Nx + 127) / 128;
    w.flat = (T.Nx % 128) != 0;
    w.nel = w.flat ? rows * T.Nx : 0;   // (< 2^30 when flat: ring_ok)
    const int nwt = w.flat ? (w.nel + 127) / 128 : rows * w.ntx;
    w.gw = blockIdx.x * RING_NW + wv;
    w.W = gridDim.x * RING_NW;
    w.nj = w.gw < nwt ? (nwt - 1 - w.gw) / w.W + 1 : 0;
    w.wring = ring + wv * D * RING_SLOT;
    return w;
}

// Wave-uniform position of a row-segment tile (Nx % 128 == 0): row = u / ntx, cx = u % ntx,
// kt = row / nyl, ky = row % nyl, advanced by W tiles with scalar adds instead of the three
// integer divisions per tile (~30 SALU instructions each) the loop used to spend.
struct RingCursor {
    int row, cx, kt, ky;
    int dr, dc;   // W = dr * ntx + dc
    __device__ __forceinline__ void init(int u, int W, int ntx, int nyl) {
        row = u / ntx; cx = u - row * ntx;
        kt = row / nyl; ky = row - kt * nyl;
        dr = W / ntx; dc = W - dr * ntx;
    }
    __device__ __forceinline__ void step(int ntx, int nyl) {
        cx += dc;
        int d = dr;
        if (cx >= ntx) { cx -= ntx; ++d; }
        row += d;
        ky += d;
        while (ky >= nyl) { ky -= nyl; ++kt; }
    }
};

// DMA of a tile (r from src, q from ph when loadq) into ring slot `slot`; i: the element of
// this lane's first value (16 B per lane)
__device__ __forceinline__ void ring_dma(double* slot, int64_t i, const double* src, const double* ph, bool loadq) {
    __builtin_amdgcn_global_load_lds((const void*)(src + i), (lds_void_t*)slot, 16, 0, 0);
    if (loadq) __builtin_amdgcn_global_load_lds((const void*)(ph + i), (lds_void_t*)(slot + 128), 16, 0, 0);
}

// element index of this lane's pair in tile u (flat: idle lanes fetch a valid address, never read)
template <bool FLAT>
__device__ __forceinline__ int64_t ring_elem(const SpecTab& T, const RingWave& w, int u, int row, int cx) {
    const int lane = threadIdx.x & 63;
    if (FLAT) {
        const int e = u * 128 + 2 * lane;
        return (e < w.nel) ? e : u * 128;
    }
    return (int64_t)row * T.Nx + cx * 128 + 2 * lane;
}

// DMA of the wave's tile j (prologue issue outside the pass loop: the late-planning prefetch)
template <int D>
__device__ __forceinline__ void ring_issue(const SpecTab& T, const RingWave& w, int j, const double* src,
                                           const double* ph, bool loadq) {
    const int u = w.gw + j * w.W;
    int64_t i;
    if (w.flat) {
        i = ring_elem<true>(T, w, u, 0, 0);
    } else {
        const int row = u / w.ntx;
        i = ring_elem<false>(T, w, u, row, u - row * w.ntx);
    }
    ring_dma(w.wring + (j % D) * RING_SLOT, i, src, ph, loadq);
}

// 16-B store of r or q: write-through (sc1) when FOTO_PASS_WT (see st_wt16); the s_nop covers
// the store-data hazard of a >8-B store before a later VALU write of its data registers
// (inline asm is outside the compiler's hazard tracking)
// (saddr form: the base in SGPRs and a 32-bit byte offset per lane, as the compiler's own stores;
// a 64-bit address per lane cost the tile loop 4 VGPRs and spilled it)
__device__ __forceinline__ void ring_store(double* base, int64_t i, dbl2 v) {
#if FOTO_PASS_WT
    const unsigned off = (unsigned)(i * 8);
    asm volatile("global_store_dwordx4 %0, %1, %2 sc1\n\ts_nop 1" ::"v"(off), "v"(v), "s"(base) : "memory");
#else
    *reinterpret_cast<dbl2*>(base + i) = v;
#endif
}

// One pass over the wave's tiles with S0's planned steps (none for INIT): apply them, write r
// (and q), accumulate the moments of the new state into acc.  issued: tiles [0, issued) already
// have their DMAs in flight or landed (a prefetch), the rest of the prologue is issued here.
// FLAT is compile-time, so the row-segment loop has no tiling branches and no lane masks.
template <int D, bool INIT, bool FLAT>
__device__ __forceinline__ void ring_pass_t(const SpecTab& T, const RingWave& w, unsigned tab_a, const SStep& S0,
                                            double* __restrict__ rh, double* __restrict__ ph,
                                            const double* __restrict__ bh, double (&acc)[NACC], int issued, bool mom) {
    const int lane = threadIdx.x & 63;
    const int k = S0.k, ns = INIT ? 0 : S0.nsteps;
    // (the division runs on the VALU: readlane puts c0, 1 / c1 back in SGPRs, not in two VGPR
    // pairs the register-bound loop would spill)
    const double c0 = dbl_readlane(INIT ? S0.ic0 : S0.c0, 0), ic1 = dbl_readlane(1.0 / (INIT ? S0.ic1 : S0.c1), 0);
    // wave-uniform flags as readfirstlane'd ints: a bool the compiler keeps as a lane mask turns
    // the count switch and the q DMA into exec-masked (divergent) code
    const bool loadq = __builtin_amdgcn_readfirstlane((!INIT && k > 0) ? 1 : 0) != 0;
    const bool momu = __builtin_amdgcn_readfirstlane(mom ? 1 : 0) != 0;
    const double* src = (INIT || k == 0) ? bh : rh;   // r_0 = b^ (the INIT pass leaves it there)
    auto moments = [&](double lam, double r, double q) {
        const double x = (lam - c0) * ic1, x2 = x + x;
        const double rr = r * r, rq = r * q, qq = q * q;
        acc[0] += rr;
        acc[NMOM] += rq;
        acc[2 * NMOM] += qq;
        acc[1] = fma(x, rr, acc[1]);
        acc[NMOM + 1] = fma(x, rq, acc[NMOM + 1]);
        acc[2 * NMOM + 1] = fma(x, qq, acc[2 * NMOM + 1]);
        double tm2 = 1.0, tm1 = x;
#pragma unroll
        for (int m = 2; m < NMOM; ++m) {
            const double t = fma(x2, tm1, -tm2);
            acc[m] = fma(t, rr, acc[m]);
            acc[NMOM + m] = fma(t, rq, acc[NMOM + m]);
            acc[2 * NMOM + m] = fma(t, qq, acc[2 * NMOM + m]);
            tm2 = tm1;
            tm1 = t;
        }
    };
    const int nj = w.nj;
    const float invx = 1.0f / (float)T.Nx, invy = 1.0f / (float)T.nyl;
    const int g = loadq ? 2 : 1;               // DMA instructions per tile
    constexpr int NST = INIT ? 1 : 2;          // store instructions per tile
    RingCursor cp{}, ci{};                     // the tile being processed / the next DMA's tile
    if (!FLAT) {
        cp.init(w.gw, w.W, w.ntx, T.nyl);
        ci.init(w.gw + issued * w.W, w.W, w.ntx, T.nyl);
    }
    for (int j = issued; j < D - 1 && j < nj; ++j) {
        ring_dma(w.wring + (j % D) * RING_SLOT, ring_elem<FLAT>(T, w, w.gw + j * w.W, ci.row, ci.cx), src, ph, loadq);
        if (!FLAT) ci.step(w.ntx, T.nyl);
    }
    if (!FLAT && issued > D - 1) {   // (a prefetch never issues more than the prologue)
        ci.init(w.gw + (D - 1) * w.W, w.W, w.ntx, T.nyl);
    }
    for (int j = 0; j < nj; ++j) {
        if (j + D - 1 < nj) {
            ring_dma(w.wring + ((j + D - 1) % D) * RING_SLOT,
                     ring_elem<FLAT>(T, w, w.gw + (j + D - 1) * w.W, ci.row, ci.cx), src, ph, loadq);
            if (!FLAT) ci.step(w.ntx, T.nyl);
        }
        const int nG = min(j + D - 1, nj - 1) - j, nS = min(j, D - 1);
        // steady state (D - 1 tiles ahead and behind) as one immediate wait; the switch over
        // counts (a branch tree) only in the prologue and drain
        if (nG == D - 1 && nS == D - 1) {
            if (INIT || !loadq) vm_wait_imm<(1 + NST) * (D - 1)>();
            else vm_wait_imm<(2 + NST) * (D - 1)>();
        } else {
            vm_wait(__builtin_amdgcn_readfirstlane(g * nG + NST * nS));
        }
        const int u = w.gw + j * w.W;
        int kx, kt, ky;
        bool ok = true;
        int64_t i;
        if (FLAT) {   // per lane: element e -> (row, kx) -> (kt, ky)
            const int e0 = u * 128 + 2 * lane;
            ok = e0 < w.nel;
            const int e = ok ? e0 : u * 128;
            const int row = ring_divmod(e, T.Nx, invx, &kx);
            kt = ring_divmod(row, T.nyl, invy, &ky);
            i = e;
        } else {      // whole row segments: every lane valid
            kx = cp.cx * 128 + 2 * lane;
            kt = cp.kt;
            ky = cp.ky;
            i = (int64_t)cp.row * T.Nx + kx;
            cp.step(w.ntx, T.nyl);
        }
        const unsigned sa = lds_u32(w.wring + (j % D) * RING_SLOT) + 16 * lane;
        dbl2 rv = lds_ld128(sa);
        dbl2 qv = loadq ? lds_ld128(sa + 1024) : dbl2{0.0, 0.0};
        double mtv = lds_ld64(tab_a + 8 * (T.Nx + kt));
        double myv = lds_ld64(tab_a + 8 * (T.Nx + T.Nt + ky));
        dbl2 mxv = lds_ld128(tab_a + 8 * (ok ? kx : 0));
        // the wait names every asm-loaded register, so no use is scheduled above it
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rv), "+v"(qv), "+v"(mtv), "+v"(myv), "+v"(mxv) :: "memory");
        const double rowmu = mtv + myv;
        const double l0 = T.reps + T.r * (rowmu + mxv[0]);
        const double l1 = T.reps + T.r * (rowmu + mxv[1]);
        double r0 = rv[0], r1 = rv[1], q0 = qv[0], q1 = qv[1];
        if (!INIT) {
            // fully unrolled with a guard, not a break (a break leaves a rolled loop that indexes
            // S0.a / S0.b from scratch with a divergent exit and a vmcnt(0) wait; measured 3x
            // slower at SMAX 10)
#pragma clang loop unroll(full)
            for (int st = 0; st < SMAX; ++st) {
                if (st < ns) {
                    // iteration k + st: p = beta p + r (k + st = 0: b = 0, q = 0, so p = r);
                    // r -= alpha (lam p)
                    const double a = S0.a[st], b = S0.b[st];
                    const double p0 = fma(b, q0, r0);
                    const double p1 = fma(b, q1, r1);
                    r0 = fma(-a, l0 * p0, r0);
                    r1 = fma(-a, l1 * p1, r1);
                    q0 = p0;
                    q1 = p1;
                }
            }
        }
        if (ok) {
            ring_store(rh, i, dbl2{r0, r1});
            if (!INIT) ring_store(ph, i, dbl2{q0, q1});
        }
        if (momu) {
            // idle lanes of a flat tail contribute exact zeros (r = q = 0: fma(t, 0, acc) = acc)
            if (!ok) r0 = r1 = q0 = q1 = 0.0;
#if defined(FOTO_RING_ABLATE)   // timing studies only (tools/pass_lab.hip): no moments
            acc[0] += r0 * q0 + r1 * q1 + l0 * l1;
#else
            moments(l0, r0, q0);
            moments(l1, r1, q1);
#endif
        }
    }
}

// The pass over the wave's tiles with S0's planned steps (dispatch on the tiling; per element the
// arithmetic is the register-fed pass's, in the same order).
template <int D, bool INIT>
__device__ __forceinline__ void ring_pass(const SpecTab& T, const RingWave& w, unsigned tab_a, const SStep& S0,
                                          double* __restrict__ rh, double* __restrict__ ph,
                                          const double* __restrict__ bh, double (&acc)[NACC], int issued,
                                          bool mom = true) {
    if (w.flat) ring_pass_t<D, INIT, true>(T, w, tab_a, S0, rh, ph, bh, acc, issued, mom);
    else ring_pass_t<D, INIT, false>(T, w, tab_a, S0, rh, ph, bh, acc, issued, mom);
}

// SStep from LDS into wave-uniform registers (the plan made in LDS feeds the step loop's
// scalar operands)
__device__ __forceinline__ SStep sstep_uniform(const SStep* p) {
    static_assert(sizeof(SStep) % 4 == 0, "SStep is whole dwords");
    constexpr int NW = sizeof(SStep) / 4;
    int wd[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) wd[i] = __builtin_amdgcn_readfirstlane(reinterpret_cast<const int*>(p)[i]);
    SStep s;
    __builtin_memcpy(&s, wd, sizeof s);
    return s;
}

// FUSE (working passes): a pass plans itself.  The pass that takes the moments leaves them in
// gath (this rank's slot; between passes of a sharded solve the all-gather fills the others)
// with S.pend = 1; the next pass's blocks each make that plan at their start, from the slots
// summed in rank order (as k_spec_s2_plan sums them, so every rank plans identically)
// (wave 0, identical inputs and code, so identical plans) while the other waves' first ring
// tiles are already loading, instead of one block planning in the tail of the previous pass
// with the whole chip idle behind it.  The last block (ticket) publishes the new moments and
// state once every block has read the old ones.  The pass whose plan finishes the solve (fin)
// skips the moments and its last block marks the solve done; a plan that finds the solve done
// at once (no step left) still passes the ticket, so that one block stores the final state.
// INIT passes plan in their tail (the fused t-DCT INIT and the ring INIT pass), leaving pend = 0.
template <int D, bool INIT, bool FUSE>
__global__ __launch_bounds__(S2_NTH) __attribute__((amdgpu_waves_per_eu(S2_WPE))) void k_spec_s2r(
        SpecTab T, double* __restrict__ rh, double* __restrict__ ph, const double* __restrict__ bh, SStep* Sg,
        RedBuf rb, double rtol, int maxiter, double* gath, int rank, int world) {
    constexpr bool LATE = FUSE && !INIT;
    __shared__ __attribute__((aligned(16))) double ring[RING_NW * D * RING_SLOT + RING_TAB];
    __shared__ __attribute__((aligned(16))) double xb[3 * NG + 2];
    // A late-planning pass needs the previous pass's moments: their loads are issued before the
    // state's, so the two round trips overlap instead of running back to back (the plan waits
    // for both).  The asm use pins the loads above the state checks.
    __shared__ double tot[NACC];
    // the state the tail publishes: the plan made at the start (late) or the one in Sg; kept in
    // LDS so the tile loop holds only the fields it uses in registers (the whole SStep live
    // across the loop cost SGPR spills -- v_readlane reloads in every tile)
    __shared__ SStep Sl;
    double gpre = 0.0;
    if (LATE && threadIdx.x < NACC) gpre = gath[threadIdx.x];   // rank 0's slot
    SStep S0 = *Sg;
    if (LATE && threadIdx.x < NACC) tot[threadIdx.x] = gpre;    // (waits for the moments only)
    if (!INIT && S0.done) return;
    const bool late = LATE && S0.pend;
    if (!INIT && !late && S0.nsteps == 0) return;
    double* tab = ring + RING_NW * D * RING_SLOT;
    const RingWave w = ring_wave(T, ring, D);
    int issued = 0;
    if constexpr (LATE) {
        if (late) {
            // Wave 0 plans at once: the previous pass's moments into LDS (its own lanes, so a
            // wave-local wait orders them), its first tiles issued behind them, the plan.  The
            // other waves stage the tables and issue their first tiles meanwhile.
            const int k = S0.k + S0.nsteps;
            const double* src = (k == 0) ? bh : rh;
            if (!S0.fin) issued = min(D - 1, w.nj);   // the plan will apply steps
#ifdef FOTO_PLAN_CLOCK   // timing studies only (tools/pass_lab.hip): 100 MHz stamps of block 0
            const long long c0 = wall_clock64();
#endif
            if (threadIdx.x < 64) {
                // the ranks' moments, summed in rank order (k_spec_s2_plan's: 0 + g0 = g0), rank
                // 0's loaded at entry
                if (threadIdx.x < NACC && world > 1) {
                    double t = gpre;
                    for (int g = 1; g < world; ++g) t += gath[g * NACC + threadIdx.x];
                    tot[threadIdx.x] = t;
                }
                if (threadIdx.x == 0) Sl = S0;
                FOTO_LDS_WAIT();
                for (int j = 0; j < issued; ++j) ring_issue<D>(T, w, j, src, ph, k > 0);
                sstep_plan_wave(&Sl, S0, tot, xb, 0, rtol, maxiter);
            } else {
                ring_stage_tables(T, tab, 64);
                for (int j = 0; j < issued; ++j) ring_issue<D>(T, w, j, src, ph, k > 0);
            }
#ifdef FOTO_PLAN_CLOCK
            const long long c1 = wall_clock64();
#endif
            __syncthreads();   // plan, tables
            S0 = sstep_uniform(&Sl);
#ifdef FOTO_PLAN_CLOCK
            if (blockIdx.x == 0 && threadIdx.x == 0) {
                foto_plan_clock[0] = c0;
                foto_plan_clock[1] = c1;
                foto_plan_clock[2] = wall_clock64();
            }
#endif
        } else {
            if (threadIdx.x == 0) Sl = S0;
            ring_stage_tables(T, tab);
            __syncthreads();
        }
    } else {
        ring_stage_tables(T, tab);
        __syncthreads();
    }
    double acc[NACC];
#pragma unroll
    for (int m = 0; m < NACC; ++m) acc[m] = 0.0;
    // the pass whose plan finished the solve (fin) needs no moments: its tail marks the solve
    // done (the bookkeeping sstep_plan_wave's fin branch would do at the next pass's start)
    const bool final_pass = LATE && S0.fin && !S0.done;
    if (!LATE || !S0.done) ring_pass<D, INIT>(T, w, lds_u32(tab), S0, rh, ph, bh, acc, issued, !final_pass);
    else if (issued) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // drain the prefetch
    if (!sp_reduce_last_rs<NACC, S2_NTH>(acc, rb, tot)) return;
    if constexpr (LATE) {
        if (!S0.done && !final_pass)   // this rank's slot (the all-gather between passes fills the others)
            for (int m = threadIdx.x; m < NACC; m += S2_NTH) gath[rank * NACC + m] = tot[m];
        if (threadIdx.x == 0) {
            SStep So = Sl;   // == S0 (thread 0 wrote it before the barrier)
            if (final_pass) {
                So.k += So.nsteps;
                So.done = So.conv ? 1 : 2;
                So.nsteps = 0;
                So.pend = 0;
            } else {
                So.pend = S0.done ? 0 : 1;
            }
            *Sg = So;
        }
        return;
    }
    if (!FUSE) {
        for (int m = threadIdx.x; m < NACC; m += S2_NTH) gath[rank * NACC + m] = tot[m];
        return;
    }
    if (threadIdx.x >= 64) return;
    sstep_plan_wave(Sg, S0, tot, xb, INIT ? 1 : 0, rtol, maxiter);
}

constexpr bool ring_fits(int D) { return (RING_NW * D * RING_SLOT + RING_TAB) * 8 <= 150 * 1024; }
static_assert(ring_fits(FOTO_RING_D), "ring + tables exceed the LDS");

// host launcher (D = 0: FOTO_RING_D)
static hipError_t launch_s2_ring(const SpecTab& T, double* rh, double* ph, const double* bh, SStep* Sg, RedBuf rb,
                                 double rtol, int maxiter, double* gath, int rank, bool init, bool fuse, int D,
                                 int nb = 256, hipStream_t s = 0, int world = 1) {
    if (D == 0) D = FOTO_RING_D;
#define FOTO_RL(DD, I, F) \
    k_spec_s2r<DD, I, F><<<nb, S2_NTH, 0, s>>>(T, rh, ph, bh, Sg, rb, rtol, maxiter, gath, rank, world)
#define FOTO_RL_D(DD)                                                                        \
    if (D == DD) {                                                                           \
        if constexpr (ring_fits(DD)) {                                                       \
            if (init) { if (fuse) FOTO_RL(DD, true, true); else FOTO_RL(DD, true, false); } \
            else { if (fuse) FOTO_RL(DD, false, true); else FOTO_RL(DD, false, false); }    \
        } else return hipErrorInvalidValue;                                                  \
    }
    FOTO_RL_D(2) else FOTO_RL_D(3) else FOTO_RL_D(4) else FOTO_RL_D(5) else FOTO_RL_D(8) else return hipErrorInvalidValue;
#undef FOTO_RL_D
#undef FOTO_RL
    return hipGetLastError();
}

// Multi-shard planning step (one wave): moments summed over ranks in rank order.
__global__ __launch_bounds__(64) void k_spec_s2_plan(SStep* Sg, const double* __restrict__ gath, int world, int init,
                                                     double rtol, int maxiter) {
    __shared__ double tot[NACC];
    const SStep S0 = *Sg;
    for (int m = threadIdx.x; m < NACC; m += 64) {
        double s = 0.0;
        for (int g = 0; g < world; ++g) s += gath[g * NACC + m];
        tot[m] = s;
    }
    __syncthreads();
    if (!init && S0.done) return;
    __shared__ __attribute__((aligned(16))) double xb[3 * NG + 2];
    sstep_plan_wave(Sg, S0, tot, xb, init, rtol, maxiter);
}

// ============================================================================ t axis, one thread per column
//
// The t-axis DCT of a single shard's spectral box [kt][ky][kx]: ncols = Ny Nx columns of NTT
// values at stride ncols.  A thread holds its column in registers, folds it into even / odd
// halves (C[k][NTT-1-j] = (-1)^k C[k][j]) and applies the two NTT/2 x NTT/2 halves of the
// DCT-II matrix, whose entries are wave-uniform (scalar loads): NTT^2 / 2 FMA per column and
// one read + one write of the volume, coalesced across the threads of a wave.  Ch holds
// E[m][j] = C[2m][j], then O[m][j] = C[2m+1][j] (m, j < NTT/2).  Two fusions remove whole
// passes from the s-step solve:
//   forward (+ INIT): b^ and, in the same sweep, the Chebyshev moments of r_0 = b^ (q = 0;
//     k_spec_s2<INIT>'s per-element formula), summed across blocks; the last block plans
//     the first pass.  The first pass reads r_0 from b^, so no r^ = b^ copy is made.
//   inverse (+ xhat): x^ = (b^ - r^) / lam formed in registers from b^ and r^.
template <int NTT>
struct TCol {
    static constexpr int H = NTT / 2;
    static_assert(NTT % 2 == 0 && NTT >= 2 && NTT <= 32, "even column lengths up to 32");
};

constexpr int TC_NTH = 256;
// Waves per SIMD of the t-column kernels (FOTO_TC_WPE, A/B builds).  At 4 (the VGPR count of the
// Nt = 32 kernels) 1024 of the bench grid's 1200 blocks are resident; forcing 5 so the grid fits
// in one round was measured much slower (INIT 70 -> 169 us, x^ 41 -> 98 us: the column loads
// and the 32-point butterflies no longer fit the registers).
#ifndef FOTO_TC_WPE
#define FOTO_TC_WPE 4
#endif

// MODE 2 (single shard): the last block plans the first pass; MODE 1 (a sharded box): it stores
// this rank's INIT moments at gath[rank * NACC] for the all-gather and k_spec_s2_plan; MODE 0:
// b^ only (the Gauss-compressed CG takes its own measure of b^)
constexpr int TC_PLAIN = 0, TC_GATH = 1, TC_PLAN = 2;
template <int NTT, int MODE>
__global__ __launch_bounds__(TC_NTH) __attribute__((amdgpu_waves_per_eu(FOTO_TC_WPE))) void k_dct_t_fwd_init(SpecTab T, const double* __restrict__ Ch,
                                                           const double* __restrict__ in, double* __restrict__ bh,
                                                           SStep* Sg, RedBuf rb, double rtol, int maxiter,
                                                           double* gath, int rank) {
    constexpr int H = TCol<NTT>::H;
    const int64_t ncols = (int64_t)T.nyl * T.Nx;
    const int64_t c = (int64_t)blockIdx.x * TC_NTH + threadIdx.x;
    if constexpr (MODE == TC_PLAIN) {
        // b^ only: the whole column's loads first (no mu_t staging, no barrier: with them the
        // column loads started a memory latency late and were waited for in pieces)
        if (c >= ncols) return;
        double x[NTT];
#pragma unroll
        for (int j = 0; j < NTT; ++j) x[j] = ld_dead(&in[j * ncols + c]);
#pragma unroll
        for (int m = 0; m < H; ++m) {
            double e = 0.0, o = 0.0;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                e = fma(Ch[m * H + j], x[j] + x[NTT - 1 - j], e);
                o = fma(Ch[H * H + m * H + j], x[j] - x[NTT - 1 - j], o);
            }
            bh[(2 * m) * ncols + c] = e;
            bh[(2 * m + 1) * ncols + c] = o;
        }
        return;
    }
    const SStep S0 = *Sg;
    const double c0 = S0.ic0, ic1 = 1.0 / S0.ic1;   // INIT interval (previous solve's b^ measure)
    double acc[NMOM];
#pragma unroll
    for (int m = 0; m < NMOM; ++m) acc[m] = 0.0;
    __shared__ double mts[NTT];   // mu_t in LDS (a global read per element after each b^ store)
    if (threadIdx.x < NTT) mts[threadIdx.x] = T.mt[threadIdx.x];
    __syncthreads();
    if (c < ncols) {
        const int kyl = (int)(c / T.Nx), kx = (int)(c - (int64_t)kyl * T.Nx), ky = T.y0 + kyl;
        // mu_y, mu_x of the column read once: inside emit they were re-read after every b^
        // store (the compiler cannot rule out aliasing), a dependent round trip per element
        const double myv = T.my[ky], mxv = T.mx[kx];
        double s[H], d[H];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const double a = in[j * ncols + c], b = in[(NTT - 1 - j) * ncols + c];
            s[j] = a + b;
            d[j] = a - b;
        }
        auto emit = [&](int k, double X) {
            bh[k * ncols + c] = X;
            if constexpr (MODE == TC_PLAIN) return;
            const double lam = T.reps + T.r * ((mts[k] + myv) + mxv);   // spec_lam's order
            const double x = (lam - c0) * ic1, x2 = x + x, rr = X * X;
            acc[0] += rr;
            acc[1] = fma(x, rr, acc[1]);
            double tm2 = 1.0, tm1 = x;
#pragma unroll
            for (int m = 2; m < NMOM; ++m) {
                const double t = fma(x2, tm1, -tm2);
                acc[m] = fma(t, rr, acc[m]);
                tm2 = tm1;
                tm1 = t;
            }
        };
#pragma unroll
        for (int m = 0; m < H; ++m) {
            double e = 0.0, o = 0.0;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                e = fma(Ch[m * H + j], s[j], e);
                o = fma(Ch[H * H + m * H + j], d[j], o);
            }
            emit(2 * m, e);
            emit(2 * m + 1, o);
        }
    }
    if constexpr (MODE == TC_PLAIN) return;
    __shared__ double tot[NACC];
    if (!sp_reduce_last_rs<NMOM, TC_NTH>(acc, rb, tot)) return;
    for (int m = NMOM + threadIdx.x; m < NACC; m += TC_NTH) tot[m] = 0.0;   // q = 0: rq, qq vanish
    __syncthreads();
    if (MODE == TC_GATH) {
        for (int m = threadIdx.x; m < NACC; m += TC_NTH) gath[rank * NACC + m] = tot[m];
        return;
    }
    if (threadIdx.x >= 64) return;
    __shared__ __attribute__((aligned(16))) double xb[3 * NG + 2];
    sstep_plan_wave(Sg, S0, tot, xb, 1, rtol, maxiter);
}

// Sg->k = iterations applied; 0: no pass ran, r^ was never written and r = b^ (x^ = 0).
// PLAIN: bh holds x^ itself (the Gauss-compressed CG's k_gq_xhat output); rh, Sg unused.
template <int NTT, bool PLAIN = false>
__global__ __launch_bounds__(TC_NTH) __attribute__((amdgpu_waves_per_eu(FOTO_TC_WPE))) void k_dct_t_inv_xhat(SpecTab T, const double* __restrict__ Ch,
                                                           const double* __restrict__ bh, const double* __restrict__ rh,
                                                           const SStep* Sg, double* __restrict__ out) {
    constexpr int H = TCol<NTT>::H;
    const int64_t ncols = (int64_t)T.nyl * T.Nx;
    const int64_t c = (int64_t)blockIdx.x * TC_NTH + threadIdx.x;
    if (c >= ncols) return;
    if (!PLAIN && Sg->k == 0) rh = bh;
    const int kyl = (int)(c / T.Nx), kx = (int)(c - (int64_t)kyl * T.Nx), ky = T.y0 + kyl;
    double xe[H], xo[H];   // x^_{2m}, x^_{2m+1}
#pragma unroll
    for (int m = 0; m < H; ++m) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int k = 2 * m + p;
            double v;
            if constexpr (PLAIN) {
                v = ld_dead(&bh[k * ncols + c]);
            } else {
                const double lam = spec_lam(T, T.mt[k] + T.my[ky], kx);
                v = (bh[k * ncols + c] - rh[k * ncols + c]) / lam;
            }
            if (p == 0) xe[m] = v;
            else xo[m] = v;
        }
    }
#pragma unroll
    for (int j = 0; j < H; ++j) {
        double e = 0.0, o = 0.0;
#pragma unroll
        for (int m = 0; m < H; ++m) {
            e = fma(Ch[m * H + j], xe[m], e);
            o = fma(Ch[H * H + m * H + j], xo[m], o);
        }
        out[j * ncols + c] = e + o;
        out[(NTT - 1 - j) * ncols + c] = e - o;
    }
}

// ---------------------------------------------------------------------------- t axis, two waves per column
// Columns too long for one thread's registers (Nt = 64 at BASELINE config 4, 1024 x 1024 x 64:
// 32 folded pairs + 32 outputs + the INIT moments would need ~180 VGPRs).  A wave pair shares 64
// columns: the even wave (role 0) owns the even outputs k = 2m (E s, s_j = x_j + x_{NTT-1-j}), the
// odd wave (role 1) the odd ones (O d, d_j = x_j - x_{NTT-1-j}).  Each wave reads the whole column
// itself (the partner's second read of the same lines is an L2 hit), so the forward needs no
// exchange; the inverse exchanges its half sums e_j / o_j through LDS in chunks of 8 rows
// (out_j = e_j + o_j, out_{NTT-1-j} = e_j - o_j).  Per wave the matrix half is wave-uniform
// (E or O: scalar loads), and every plane is read and written as 64 contiguous doubles per
// wave instruction -- the strided FFT this replaces ran at ~1 TB/s (64 planes 8 MB apart per
// block).
constexpr int TP_CH = 8;   // inverse: rows per LDS exchange chunk

// (64 points: 32 folded values + 16 moment sums + the recurrence need ~130 VGPRs: 3 waves per
// SIMD, no spills)
template <int NTT, int MODE>
__global__ __launch_bounds__(TC_NTH) __attribute__((amdgpu_waves_per_eu(NTT > 48 ? 3 : 4))) void k_dct_tp_fwd_init(
        SpecTab T, const double* __restrict__ Ch, const double* __restrict__ in, double* __restrict__ bh, SStep* Sg,
        RedBuf rb, double rtol, int maxiter, double* gath, int rank) {
    constexpr int H = NTT / 2;
    static_assert(NTT % 2 == 0 && H % TP_CH == 0, "even column length, whole exchange chunks");
    const int64_t ncols = (int64_t)T.nyl * T.Nx;
    const int lane = threadIdx.x & 63;
    const int role = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 1);       // 0 even, 1 odd
    const int pair = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
    const int64_t c = ((int64_t)blockIdx.x * (TC_NTH / 128) + pair) * 64 + lane;
    const SStep S0 = *Sg;
    const double c0 = S0.ic0, ic1 = 1.0 / S0.ic1;   // INIT interval (previous solve's b^ measure)
    double acc[NMOM];
#pragma unroll
    for (int m = 0; m < NMOM; ++m) acc[m] = 0.0;
    __shared__ double mts[NTT];
    for (int i = threadIdx.x; i < NTT; i += TC_NTH) mts[i] = T.mt[i];
    __syncthreads();
    if (c < ncols) {
        const int kyl = (int)(c / T.Nx), kx = (int)(c - (int64_t)kyl * T.Nx), ky = T.y0 + kyl;
        const double myv = T.my[ky], mxv = T.mx[kx];
        const double sg = role ? -1.0 : 1.0;
        double v[H];   // s (even wave) or d (odd wave)
#pragma unroll
        for (int j = 0; j < H; ++j) v[j] = in[j * ncols + c] + sg * in[(NTT - 1 - j) * ncols + c];
        const double* M = Ch + role * H * H;   // E or O, wave-uniform
#pragma unroll
        for (int m = 0; m < H; ++m) {
            double X = 0.0;
#pragma unroll
            for (int j = 0; j < H; ++j) X = fma(M[m * H + j], v[j], X);
            const int k = 2 * m + role;
            bh[k * ncols + c] = X;
            if constexpr (MODE == TC_PLAIN) continue;
            const double lam = T.reps + T.r * ((mts[k] + myv) + mxv);   // spec_lam's order
            const double x = (lam - c0) * ic1, x2 = x + x, rr = X * X;
            acc[0] += rr;
            acc[1] = fma(x, rr, acc[1]);
            double tm2 = 1.0, tm1 = x;
#pragma unroll
            for (int mm = 2; mm < NMOM; ++mm) {
                const double t = fma(x2, tm1, -tm2);
                acc[mm] = fma(t, rr, acc[mm]);
                tm2 = tm1;
                tm1 = t;
            }
        }
    }
    if constexpr (MODE == TC_PLAIN) return;
    __shared__ double tot[NACC];
    if (!sp_reduce_last_rs<NMOM, TC_NTH>(acc, rb, tot)) return;
    for (int m = NMOM + threadIdx.x; m < NACC; m += TC_NTH) tot[m] = 0.0;   // q = 0: rq, qq vanish
    __syncthreads();
    if (MODE == TC_GATH) {
        for (int m = threadIdx.x; m < NACC; m += TC_NTH) gath[rank * NACC + m] = tot[m];
        return;
    }
    if (threadIdx.x >= 64) return;
    __shared__ __attribute__((aligned(16))) double xb[3 * NG + 2];
    sstep_plan_wave(Sg, S0, tot, xb, 1, rtol, maxiter);
}

template <int NTT, bool PLAIN = false>
__global__ __launch_bounds__(TC_NTH) __attribute__((amdgpu_waves_per_eu(4))) void k_dct_tp_inv_xhat(
        SpecTab T, const double* __restrict__ Ch, const double* __restrict__ bh, const double* __restrict__ rh,
        const SStep* Sg, double* __restrict__ out) {
    constexpr int H = NTT / 2;
    const int64_t ncols = (int64_t)T.nyl * T.Nx;
    const int lane = threadIdx.x & 63;
    const int role = __builtin_amdgcn_readfirstlane((threadIdx.x >> 6) & 1);
    const int pair = __builtin_amdgcn_readfirstlane(threadIdx.x >> 7);
    const int64_t c = ((int64_t)blockIdx.x * (TC_NTH / 128) + pair) * 64 + lane;
    const bool ok = c < ncols;
    if (!PLAIN && Sg->k == 0) rh = bh;   // no pass ran: r = b^, x^ = 0
    __shared__ double xs[TC_NTH / 128][2][TP_CH][64];   // [pair][role][row of chunk][column]
    double xk[H];   // x^_{2m + role}
    if (ok) {
        const int kyl = (int)(c / T.Nx), kx = (int)(c - (int64_t)kyl * T.Nx), ky = T.y0 + kyl;
#pragma unroll
        for (int m = 0; m < H; ++m) {
            const int k = 2 * m + role;
            if constexpr (PLAIN) {
                xk[m] = bh[k * ncols + c];
            } else {
                const double lam = spec_lam(T, T.mt[k] + T.my[ky], kx);
                xk[m] = (bh[k * ncols + c] - rh[k * ncols + c]) / lam;
            }
        }
    } else {
#pragma unroll
        for (int m = 0; m < H; ++m) xk[m] = 0.0;
    }
    const double* M = Ch + role * H * H;
#pragma unroll
    for (int j0 = 0; j0 < H; j0 += TP_CH) {
#pragma unroll
        for (int jj = 0; jj < TP_CH; ++jj) {
            double e = 0.0;
#pragma unroll
            for (int m = 0; m < H; ++m) e = fma(M[m * H + j0 + jj], xk[m], e);
            xs[pair][role][jj][lane] = e;
        }
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < TP_CH; ++jj) {
            const double e = xs[pair][0][jj][lane], o = xs[pair][1][jj][lane];
            const int j = j0 + jj;
            if (ok) {
                if (role == 0) out[j * ncols + c] = e + o;
                else out[(NTT - 1 - j) * ncols + c] = e - o;
            }
        }
        __syncthreads();
    }
}

#define FOTO_TPAIR_SIZES(X) X(48) X(64)

#define FOTO_TCOL_SIZES(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(20) X(24) X(32)

#include "foto_gauss.inc"

static bool tcol_supported(int n) {
#define FOTO_TCOL_CASE(NN) if (n == NN) return true;
    FOTO_TCOL_SIZES(FOTO_TCOL_CASE)
    FOTO_TPAIR_SIZES(FOTO_TCOL_CASE)
#undef FOTO_TCOL_CASE
    return false;
}
static bool tpair_size(int n) {
#define FOTO_TCOL_CASE(NN) if (n == NN) return true;
    FOTO_TPAIR_SIZES(FOTO_TCOL_CASE)
#undef FOTO_TCOL_CASE
    return false;
}

// ============================================================================ plan

static int split_start_h(int n, int W, int h) {
    const int base = n / W, extra = n % W;
    return h * base + std::min(h, extra);
}

struct SpecImpl {
    Geo g{};
    int rank = 0, world = 1;
    int y0 = 0, nyl = 0;          // spectral box rows (sharded: Ny split over ranks)
    double r = 1, eps = 0;
    double *bh = nullptr, *rh = nullptr, *ph = nullptr, *tmp = nullptr;   // spectral box
    double* tmpp = nullptr;       // physical slab scratch (one halo plane per side: tmpp[-nxy ..])
    double *Cx = nullptr, *Cy = nullptr, *Ct = nullptr, *CxT = nullptr, *CyT = nullptr, *CtT = nullptr;
    double *mx = nullptr, *my = nullptr, *mt = nullptr;
    double *Fx = nullptr, *Fy = nullptr, *Ft = nullptr;   // FFT-DCT tables (nullptr: GEMM path)
    RedBuf rb{};
    double* gath = nullptr;       // s = 1: 2 doubles; s-step sharded: world * NACC
    CGScal* S = nullptr;
    CGScal* hS = nullptr;
    SStep* S2 = nullptr;
    SStep* hS2 = nullptr;
    int nblocks2 = 0;
    bool ring = false;   // s-step passes by the LDS-ring kernel
    int nb_ring = 0;
    double* Cth = nullptr;        // t-axis DCT-II even | odd halves (column kernels)
    bool tcol = false;            // single shard, s-step, Nt in FOTO_TCOL_SIZES
    bool xt = false;              // single shard, Gauss CG: x and t DCTs in one pass (k_dct_xt_fwd / k_dct_tx_inv)
    int tcol_nb = 0;              // column kernels' blocks
    int last_passes = 0;          // passes of the previous s-step solve (first chunk size)
    // deferred solves in flight (solve_deferred -> finish), oldest first: one for the s-step
    // CG, up to two for the Gauss CG (two outer iterations in flight)
    struct Pend {
        int launched = 0, maxiter = 0, hslot = 0;
        double rtol = 0.0;
        double *b = nullptr, *x = nullptr;
    };
    Pend pq[2];
    int npend = 0;
    int sstep = 1;
    bool split_plan = false;
    std::vector<void*> allocs;
    int nblocks = 0;
    double c0 = 0, c1 = 1;
    // Gauss-compressed CG (cg_mode 3, foto_gauss.inc); gauss_active: the solve in flight uses it
    bool gauss = false, gauss_active = false;
    GqState* gq = nullptr;
    GqState* hgq2[2] = {nullptr, nullptr};   // pinned: the header (K, status, conv, done, bn2, rn2) of
    int hslot = 0, hlast = 0;                // the last two solves (hslot: the next one's)
    GqState* dgq2[2] = {nullptr, nullptr};   // their device addresses (coherent host memory)
    GqNodes* gqn = nullptr;
    double* gq_hist = nullptr;    // world histograms (slot rank is this box's)
    bool gq_nodes_wave = true;    // k_gq_nodes_w (FOTO_GQ_NODES=thread: k_gq_nodes, the round-4 form)
    bool gq_tfuse = false;        // x^ inside the inverse t-DCT (k_dct_t_inv_gq; FOTO_GQ_TFUSE)
    double* gq_tab = nullptr;
    GqBins* gq_bins = nullptr;    // bin edges of the measure and the solution table
    GqQCos* gq_qcos = nullptr;    // the solution table's transform constants
    GqPub* gq_pub = nullptr;      // k_gq_cgtab's (alpha, beta) slots
    bool gq_cgtab = true;         // FOTO_GQ_CGTAB=0: k_gq_cg, then k_gq_qtab
    // bin-ordered histogram (k_gq_hist_perm): the box's voxels grouped by bin, chunked
    unsigned* gq_permv = nullptr;
    GqChunk* gq_chunks = nullptr;
    int gq_nch = 0;
    int* gq_cfirst = nullptr;     // [GQ_NB + 1] first chunk of each bin
    double* gq_rowmu = nullptr;   // mu_t + mu_y per box row
    double* gq_ppart = nullptr;   // [chunk id][GQ_NM] chunk sums
    GqExact* gq_exact = nullptr;  // exact bins (the whole grid's distinct eigenvalues)

    // k_spec_s2r LATE: working ring passes plan at their start (single shard unless split;
    // sharded always); the pass a plan finishes marks the solve done in its tail
    int late_plan() const { return (ring && (world > 1 || !split_plan)) ? 1 : 0; }

    int alloc(size_t bytes, void** p) {
        FOTO_HIP_CHECK(hipMalloc(p, bytes));
        allocs.push_back(*p);
        return 0;
    }
    ~SpecImpl() {
        for (void* p : allocs) (void)hipFree(p);
        if (hS) (void)hipHostFree(hS);
        if (hS2) (void)hipHostFree(hS2);
        for (GqState* h : hgq2)
            if (h) (void)hipHostFree(h);
    }
    SpecTab tab() const {
        SpecTab T;
        T.mt = mt; T.my = my; T.mx = mx; T.r = r; T.reps = r * eps;
        T.Nt = g.Nt; T.Ny = g.Ny; T.Nx = g.Nx;
        T.y0 = y0; T.nyl = nyl;
        return T;
    }
    bool vec() const { return (g.Nx % 2) == 0; }
    double nbox() const { return (double)g.Nt * nyl * g.Nx; }
};
static int gq_pub_clear(SpecImpl* P, hipStream_t s);

// orthonormal DCT-II matrix C[k][j] = s_k cos(pi k (2j+1) / (2n)) (long double on the host)
// eigenvalues 2 - 2 cos(pi k / n) of the Neumann second difference (the same values dct_matrix gives)
static void dct_eigen(int n, std::vector<double>& mu) {
    mu.assign(n, 0.0);
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int k = 0; k < n; ++k) mu[k] = (double)(2.0L - 2.0L * cosl(pi * k / n));
}

static void dct_matrix(int n, std::vector<double>& C, std::vector<double>& CT, std::vector<double>& mu) {
    C.assign((size_t)n * n, 0.0);
    CT.assign((size_t)n * n, 0.0);
    mu.assign(n, 0.0);
    const long double pi = 3.141592653589793238462643383279502884L;
    for (int k = 0; k < n; ++k) {
        const long double s = (k == 0) ? sqrtl(1.0L / n) : sqrtl(2.0L / n);
        for (int j = 0; j < n; ++j) {
            const double v = (double)(s * cosl(pi * k * (2.0L * j + 1.0L) / (2.0L * n)));
            C[(size_t)k * n + j] = v;
            CT[(size_t)j * n + k] = v;
        }
        mu[k] = (double)(2.0L - 2.0L * cosl(pi * k / n));
    }
}

static int reset_s2(SpecImpl* P, hipStream_t s);

static int cus_count() {   // CUs of the current device (cached per device ordinal)
    static int cache[64] = {0};
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess) return cus;
    if (dev >= 0 && dev < 64 && cache[dev] > 0) return cache[dev];
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 256;
    if (dev >= 0 && dev < 64) cache[dev] = cus;
    return cus;
}

static int gq_build_perm(SpecImpl* P, hipStream_t s);

int SpectralPlan::init(const Geo& g, int rank, int world, double r, double eps, int sstep, hipStream_t s) {
    // cg_mode 3: the Gauss-compressed CG, with the s-step machinery kept for the (rare) redo
    const bool gauss = (sstep == 3);
    if (gauss) sstep = 2;
    if (sstep != 1 && sstep != 2) {
        set_error("spectral CG: s-step must be 1 or 2");
        return FOTO_ERR_ARG;
    }
    if (world > 1 && sstep != 2) {
        set_error("sharded spectral CG needs cg_mode = 2 (s-step)");
        return FOTO_ERR_ARG;
    }
    if (world > g.Ny) {
        set_error("sharded spectral CG needs Ny >= world (rows are split over ranks)");
        return FOTO_ERR_ARG;
    }
    if (!(eps > 0.0)) {
        set_error("spectral CG needs reg_epsilon > 0 (x = (b - r) / lam)");
        return FOTO_ERR_ARG;
    }
    auto* P = new SpecImpl();
    impl = P;
    P->sstep = sstep;
    P->g = g;
    P->rank = rank;
    P->world = world;
    P->y0 = split_start_h(g.Ny, world, rank);
    P->nyl = split_start_h(g.Ny, world, rank + 1) - P->y0;
    P->r = r;
    P->eps = eps;
    {
        const char* e = getenv("FOTO_S2_SPLIT");   // tuning knob: plan in its own 1-block kernel
        P->split_plan = e && atoi(e) != 0;
    }
    const size_t NB = (size_t)g.Nt * P->nyl * g.Nx;          // spectral box
    const size_t NS = (size_t)g.nloc * g.nxy;                // physical slab
    void* b;
    FOTO_TRY(P->alloc(NB * 8, &b)); P->bh = (double*)b;
    FOTO_TRY(P->alloc(NB * 8, &b)); P->rh = (double*)b;
    FOTO_TRY(P->alloc(NB * 8, &b)); P->ph = (double*)b;
    FOTO_TRY(P->alloc(std::max(NB, NS) * 8, &b)); P->tmp = (double*)b;
    if (world > 1) {
        FOTO_TRY(P->alloc((NS + 2 * (size_t)g.nxy) * 8, &b)); P->tmpp = (double*)b + g.nxy;
    }
    std::vector<double> C, CT, mu;
    if (g_dct_fft < 0) {
        const char* e = getenv("FOTO_DCT_FFT");
        g_dct_fft = e ? atoi(e) : 1;
    }
    // the n x n matrices only for an axis the FFT kernels do not take (dct_fft_axis's rule):
    // 2 x 3.3 MB of host cosines and blocking copies per 640-axis saved at context creation
    auto up = [&](int n, double** Cd, double** CTd, double** mud) -> int {
        int m1, m2;
        const bool fft = g_dct_fft && n >= 64 && fft_factors(n, &m1, &m2);
        if (fft) dct_eigen(n, mu);
        else dct_matrix(n, C, CT, mu);
        void* p;
        if (!fft) {
            FOTO_TRY(P->alloc(C.size() * 8, &p)); *Cd = (double*)p;
            FOTO_TRY(P->alloc(CT.size() * 8, &p)); *CTd = (double*)p;
            FOTO_HIP_CHECK(hipMemcpy(*Cd, C.data(), C.size() * 8, hipMemcpyHostToDevice));
            FOTO_HIP_CHECK(hipMemcpy(*CTd, CT.data(), CT.size() * 8, hipMemcpyHostToDevice));
        }
        FOTO_TRY(P->alloc(mu.size() * 8, &p)); *mud = (double*)p;
        FOTO_HIP_CHECK(hipMemcpy(*mud, mu.data(), mu.size() * 8, hipMemcpyHostToDevice));
        return (int)0;
    };
    FOTO_TRY(up(g.Nx, &P->Cx, &P->CxT, &P->mx));
    const double mx_max = mu.back();
    FOTO_TRY(up(g.Ny, &P->Cy, &P->CyT, &P->my));
    const double my_max = mu.back();
    FOTO_TRY(up(g.Nt, &P->Ct, &P->CtT, &P->mt));
    const double mt_max = mu.back();
    auto upf = [&](int n, double** Fd) -> int {
        int m1, m2;
        if (!fft_factors(n, &m1, &m2)) return 0;
        const std::vector<double> t = fft_table(n);
        void* p;
        FOTO_TRY(P->alloc(t.size() * 8, &p));
        *Fd = (double*)p;
        FOTO_HIP_CHECK(hipMemcpy(*Fd, t.data(), t.size() * 8, hipMemcpyHostToDevice));
        return 0;
    };
    FOTO_TRY(upf(g.Nx, &P->Fx));
    FOTO_TRY(upf(g.Ny, &P->Fy));
    FOTO_TRY(upf(g.Nt, &P->Ft));
    // Chebyshev scaling of lam: global spectrum bounds (identical on every rank)
    const double lmin = r * eps, lmax = r * eps + r * (mt_max + my_max + mx_max);
    P->c0 = 0.5 * (lmax + lmin);
    P->c1 = 0.5 * (lmax - lmin);
    const int rows = g.Nt * P->nyl;
    const int ntiles = ((g.Nx + 127) / 128) * ((rows + 3) / 4);
    P->nblocks = std::min(ntiles, 2048);
    {
        // one resident wave of blocks: blocks per CU at the pass kernel's occupancy x CUs
        const int ntiles2 = ((g.Nx + 127) / 128) * ((rows + S2_NTH / 64 - 1) / (S2_NTH / 64));
        int dev = 0, cus = 256, per_cu = 0;
        FOTO_HIP_CHECK(hipGetDevice(&dev));
        FOTO_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        FOTO_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spec_s2<true, false, true>, S2_NTH, 0));
        const char* e = getenv("FOTO_S2_BLOCKS");   // tuning knob for A/B runs
        const int want = e ? std::max(1, atoi(e)) : std::max(1, per_cu) * cus;
        P->nblocks2 = std::min(ntiles2, want);
        // ring-fed pass (k_spec_s2r): one 1024-thread block per CU (its LDS ring), at most one
        // block per 16 wave tiles; FOTO_RING=0 selects the register-fed pass (A/B runs)
        const char* er = getenv("FOTO_RING");
        P->ring = ring_ok(P->tab()) && !(er && atoi(er) == 0);
        const int nwt = ((g.Nx + 127) / 128) * rows;
        P->nb_ring = std::max(1, std::min({P->nblocks2, cus, (nwt + RING_NW - 1) / RING_NW}));
    }
    {
        const char* e = getenv("FOTO_TCOL");   // 0: t axis by dct_pass + separate INIT / xhat passes (A/B runs)
        P->tcol = sstep == 2 && tcol_supported(g.Nt) && !(e && atoi(e) == 0);
    }
    if (P->tcol) {
        const int H = g.Nt / 2;
        dct_matrix(g.Nt, C, CT, mu);
        std::vector<double> ch((size_t)2 * H * H);
        for (int m = 0; m < H; ++m)
            for (int j = 0; j < H; ++j) {
                ch[(size_t)m * H + j] = C[(size_t)(2 * m) * g.Nt + j];
                ch[(size_t)H * H + m * H + j] = C[(size_t)(2 * m + 1) * g.Nt + j];
            }
        FOTO_TRY(P->alloc(ch.size() * 8, &b));
        P->Cth = (double*)b;
        FOTO_HIP_CHECK(hipMemcpy(P->Cth, ch.data(), ch.size() * 8, hipMemcpyHostToDevice));
        const int per_block = tpair_size(g.Nt) ? TC_NTH / 2 : TC_NTH;   // wave pairs: 64 columns per 2 waves
        P->tcol_nb = (int)(((int64_t)P->nyl * g.Nx + per_block - 1) / per_block);
    }
    const int cap = std::max({2 * P->nblocks, NACC * P->nblocks2, NMOM * P->tcol_nb});
    FOTO_TRY(P->alloc(sizeof(double) * (cap + 8), &b));
    P->rb.partials = (double*)b;
    P->rb.ticket = (unsigned*)((double*)b + cap);
    P->rb.cap = cap;
    FOTO_HIP_CHECK(hipMemsetAsync(P->rb.ticket, 0, 8 * sizeof(double), s));
    FOTO_TRY(P->alloc(sizeof(double) * std::max(4, NACC * world), &b)); P->gath = (double*)b;
    FOTO_TRY(P->alloc(sizeof(CGScal), &b)); P->S = (CGScal*)b;
    FOTO_HIP_CHECK(hipHostMalloc((void**)&P->hS, sizeof(CGScal)));
    FOTO_TRY(P->alloc(sizeof(SStep), &b)); P->S2 = (SStep*)b;
    FOTO_HIP_CHECK(hipHostMalloc((void**)&P->hS2, sizeof(SStep)));
    FOTO_TRY(reset_s2(P, s));   // c0, c1 for the fused INIT (solve_tcol)
    // the Gauss-compressed CG needs the bin-ordered voxel list; boxes its packing does not
    // cover run the s-step CG (decided on the whole grid, so every rank agrees)
    P->gauss = gauss && gq_perm_ok(g.Nx, g.Nt * g.Ny);
    {   // (x, t) / (t, x) in one pass: single shard, the column kernels' t sizes, an FFT x plan.
        // Opt-in (FOTO_DCT_XT=1): correct (the whole GPU suite passes with it) but measured 2.2x
        // slower than the two passes it replaces -- 151 / 165 us against 69 / 72 us at the bench
        // grid (profiles/r05_xt_ab.txt): a row slab's t-sums (164 KB) pin one 512-thread block
        // per CU, whose load / FFT / accumulate phases then run without overlap.
        const char* e = getenv("FOTO_DCT_XT");
        P->xt = P->gauss && P->tcol && world == 1 && P->Fx && g_dct_fft && xt_supported(g.Nx, g.Nt) &&
                (e && atoi(e) == 1);
    }
    if (P->gauss) {
        FOTO_TRY(P->alloc(sizeof(GqState), &b)); P->gq = (GqState*)b;
        FOTO_HIP_CHECK(hipMemsetAsync(P->gq, 0, sizeof(GqState), s));
        for (int k = 0; k < 2; ++k) {
            FOTO_HIP_CHECK(hipHostMalloc((void**)&P->hgq2[k], sizeof(GqState), hipHostMallocMapped | hipHostMallocCoherent));
            std::memset((void*)P->hgq2[k], 0, sizeof(GqState));
            FOTO_HIP_CHECK(hipHostGetDevicePointer((void**)&P->dgq2[k], P->hgq2[k], 0));
        }
        FOTO_TRY(P->alloc(sizeof(GqNodes), &b)); P->gqn = (GqNodes*)b;
        FOTO_TRY(P->alloc(sizeof(double) * GQ_HIST * world, &b)); P->gq_hist = (double*)b;
        const char* gn = getenv("FOTO_GQ_NODES");
        P->gq_nodes_wave = !(gn && std::strcmp(gn, "thread") == 0);
        const char* tf = getenv("FOTO_GQ_TFUSE");
        P->gq_tfuse = tf && atoi(tf) != 0;
        FOTO_TRY(P->alloc(GQ_TAB_BYTES, &b)); P->gq_tab = (double*)b;
        // k_gq_xhat holds the whole table (128 KB) in dynamic LDS, beside its 10 KB bin tables
        FOTO_HIP_CHECK(hipFuncSetAttribute((const void*)k_gq_xhat, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)GQ_TAB_BYTES));
        FOTO_TRY(P->alloc(sizeof(GqBins), &b)); P->gq_bins = (GqBins*)b;
        k_gq_bins<<<1, 256, 0, s>>>(P->gq_bins);
        FOTO_TRY(P->alloc(sizeof(GqQCos), &b)); P->gq_qcos = (GqQCos*)b;
        k_gq_qcos<<<1, 256, 0, s>>>(P->gq_qcos);
        FOTO_TRY(P->alloc(sizeof(GqPub), &b)); P->gq_pub = (GqPub*)b;
        FOTO_TRY(gq_pub_clear(P, s));
        const char* ct = getenv("FOTO_GQ_CGTAB");
        P->gq_cgtab = !(ct && atoi(ct) == 0);
        FOTO_HIP_CHECK(hipGetLastError());
        FOTO_TRY(P->alloc(sizeof(GqExact), &b)); P->gq_exact = (GqExact*)b;
        FOTO_TRY(gq_build_perm(P, s));
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
    }
    return 0;
}

// The bin-ordered voxel list of a box T (k_gq_hist_perm): per-row run counts by bin, a scan
// over the rows of each bin, the bins' first entries (host and device), then every row writes
// its runs.  perm (rows * Nx), rowmu (rows), first_d / tot_d (GQ_NB + 1 / GQ_NB) are the
// caller's; the count table is scratch.
static int gq_perm_lists(SpecImpl* P, const SpecTab& T, unsigned* perm, double* rowmu, int* first_d, int* tot_d,
                         std::vector<int>& htot, std::vector<int>& hfirst, hipStream_t s) {
    const int rows = T.Nt * T.nyl;
    const int64_t N = (int64_t)rows * T.Nx;
    k_gq_rowmu<<<(rows + 255) / 256, 256, 0, s>>>(T, rowmu);
    FOTO_HIP_CHECK(hipGetLastError());
    int* cnt = nullptr;
    const size_t ncnt = (size_t)GQ_NB * rows;
    FOTO_HIP_CHECK(hipMalloc((void**)&cnt, sizeof(int) * ncnt));
    int rc = 0;
    htot.assign(GQ_NB, 0);
    hfirst.assign(GQ_NB + 1, 0);
    do {
        if (hipMemsetAsync(cnt, 0, sizeof(int) * ncnt, s) != hipSuccess) { rc = -1; break; }
        k_gq_perm_count<<<(rows + 255) / 256, 256, 0, s>>>(T, P->gq_bins, rowmu, 1.0 / P->c1, cnt);
        k_gq_perm_scan<<<GQ_NB, 256, 0, s>>>(rows, cnt, tot_d);
        if (hipMemcpyAsync(htot.data(), tot_d, sizeof(int) * GQ_NB, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess) { rc = -1; break; }
        int64_t acc = 0;
        for (int bb = 0; bb < GQ_NB; ++bb) {
            hfirst[bb] = (int)acc;
            acc += htot[bb];
        }
        hfirst[GQ_NB] = (int)acc;
        if (acc != N) {
            set_error("gauss perm: %lld voxels binned, box has %lld", (long long)acc, (long long)N);
            rc = -1;
            break;
        }
        if (hipMemcpyAsync(first_d, hfirst.data(), sizeof(int) * (GQ_NB + 1), hipMemcpyHostToDevice, s) != hipSuccess) {
            rc = -1;
            break;
        }
        k_gq_perm_fill<<<(rows + 255) / 256, 256, 0, s>>>(T, P->gq_bins, rowmu, 1.0 / P->c1, cnt, first_d, perm);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) rc = -1;
    } while (false);
    (void)hipFree(cnt);
    if (rc) set_error("gauss perm build failed");
    return rc ? -1 : 0;
}

// The chunk list in dispatch order.  Neighbouring bins share the cache lines of b^ (a 16-voxel
// line holds runs of ~2 bins of a row), and a bin's chunks walk the rows in order, so the chunks
// of all bins over the same rows read the same lines at about the same time -- from the same L2
// only if they run on the same XCD.  Workgroups go round-robin to the 8 XCDs (block k to XCD
// k % 8) and a block's 4 waves take slots 4k .. 4k + 3: slot lists are filled so that XCD x
// gets the chunks whose first row lies in the x-th eighth of the rows (FOTO_GQ_XCD=0: bin order).
// The sums go to part[chunk id] either way, so the histogram is bit-identical.
static int gq_order_chunks(SpecImpl* P, std::vector<GqChunk>& ch, int rows, hipStream_t s) {
    const char* e = getenv("FOTO_GQ_XCD");
    const int nx = 8;
    const int n = (int)ch.size();
    if ((e && atoi(e) == 0) || n < 4 * nx) return 0;
    void* b = nullptr;
    GqChunk* dch = nullptr;
    int* drow = nullptr;
    FOTO_HIP_CHECK(hipMalloc(&b, sizeof(GqChunk) * n + sizeof(int) * n));
    dch = (GqChunk*)b;
    drow = (int*)(dch + n);
    std::vector<int> row(n);
    int rc = 0;
    if (hipMemcpyAsync(dch, ch.data(), sizeof(GqChunk) * n, hipMemcpyHostToDevice, s) != hipSuccess) rc = -1;
    if (!rc) {
        k_gq_chunk_rows<<<(n + 255) / 256, 256, 0, s>>>(dch, n, P->gq_permv, drow);
        if (hipGetLastError() != hipSuccess ||
            hipMemcpyAsync(row.data(), drow, sizeof(int) * n, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            rc = -1;
    }
    (void)hipFree(b);
    if (rc) {
        set_error("gauss chunk order: device step failed");
        return FOTO_ERR_HIP;
    }
    std::vector<std::vector<int>> L(nx);
    for (int c = 0; c < n; ++c) L[std::min(nx - 1, (int)((int64_t)row[c] * nx / std::max(1, rows)))].push_back(c);
    std::vector<size_t> at(nx, 0);
    const int nb = (n + 3) / 4;
    std::vector<GqChunk> out((size_t)nb * 4, GqChunk{0, 0, 0, -1});
    for (int k = 0; k < nb; ++k)
        for (int w = 0; w < 4; ++w) {
            int x = k % nx;
            if (at[x] == L[x].size()) {   // this XCD's share is used up: the longest remaining list
                size_t best = 0;
                x = -1;
                for (int y = 0; y < nx; ++y)
                    if (L[y].size() - at[y] > best) { best = L[y].size() - at[y]; x = y; }
                if (x < 0) continue;
            }
            out[(size_t)k * 4 + w] = ch[L[x][at[x]++]];
        }
    ch.swap(out);
    return 0;
}

// this box's list and chunks, and the exact bins of the whole grid (from the box's list when the
// box is the grid, else from a scratch list of the grid: every rank derives the same table)
static int gq_build_perm(SpecImpl* P, hipStream_t s) {
    const SpecTab T = P->tab();
    // exact bins of at most GQ_M points (their points are the rule).  FOTO_GQ_EXACT (A/B): -1
    // none; up to GQ_XS = 16 also takes bins of 9-16 points through the Stieltjes procedure --
    // measured less accurate (the 5-step iterate of an 8x24x20 grid 1.6e-10 from scipy's against
    // 2.3e-12; the node / weight solve loses digits on clustered points), not the default
    const char* ex = getenv("FOTO_GQ_EXACT");
    const int xmax = ex ? std::min(atoi(ex), GQ_XS) : GQ_M;
    const int rows = P->g.Nt * P->nyl;
    const int64_t N = (int64_t)rows * P->g.Nx;
    void* b = nullptr;
    FOTO_TRY(P->alloc(sizeof(double) * rows, &b)); P->gq_rowmu = (double*)b;
    FOTO_TRY(P->alloc(sizeof(unsigned) * N, &b)); P->gq_permv = (unsigned*)b;
    FOTO_TRY(P->alloc(sizeof(int) * (2 * GQ_NB + 1), &b));
    int* first_d = (int*)b;
    int* tot_d = first_d + GQ_NB + 1;
    std::vector<int> htot, hfirst;
    FOTO_TRY(gq_perm_lists(P, T, P->gq_permv, P->gq_rowmu, first_d, tot_d, htot, hfirst, s));
    std::vector<GqChunk> ch;
    std::vector<int> cfirst(GQ_NB + 1);
    for (int bb = 0; bb < GQ_NB; ++bb) {
        cfirst[bb] = (int)ch.size();
        for (int st = 0; st < htot[bb]; st += GQ_PCH)
            ch.push_back(GqChunk{bb, hfirst[bb] + st, std::min(GQ_PCH, htot[bb] - st), (int)ch.size()});
    }
    cfirst[GQ_NB] = (int)ch.size();
    const int nch = (int)ch.size();
    FOTO_TRY(P->alloc(sizeof(int) * (GQ_NB + 1), &b)); P->gq_cfirst = (int*)b;
    FOTO_TRY(P->alloc(sizeof(double) * GQ_NM * std::max(1, nch), &b)); P->gq_ppart = (double*)b;
    FOTO_TRY(gq_order_chunks(P, ch, rows, s));
    P->gq_nch = (int)ch.size();
    FOTO_TRY(P->alloc(sizeof(GqChunk) * std::max<size_t>(1, ch.size()), &b)); P->gq_chunks = (GqChunk*)b;
    FOTO_HIP_CHECK(hipMemcpyAsync(P->gq_chunks, ch.data(), sizeof(GqChunk) * ch.size(), hipMemcpyHostToDevice, s));
    FOTO_HIP_CHECK(hipMemcpyAsync(P->gq_cfirst, cfirst.data(), sizeof(int) * (GQ_NB + 1), hipMemcpyHostToDevice, s));
    if (P->nyl == P->g.Ny) {
        k_gq_exact<<<GQ_NB / 64, 64, 0, s>>>(T, P->gq_permv, first_d, tot_d, P->gq_rowmu, 1.0 / P->c1, xmax, P->gq_exact);
        FOTO_HIP_CHECK(hipGetLastError());
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        return 0;
    }
    SpecTab TG = T;   // the whole grid
    TG.y0 = 0;
    TG.nyl = P->g.Ny;
    const int grows = P->g.Nt * P->g.Ny;
    unsigned* gperm = nullptr;
    double* growmu = nullptr;
    int* gidx = nullptr;
    int rc = 0;
    if (hipMalloc((void**)&gperm, sizeof(unsigned) * (size_t)grows * P->g.Nx) != hipSuccess ||
        hipMalloc((void**)&growmu, sizeof(double) * grows) != hipSuccess ||
        hipMalloc((void**)&gidx, sizeof(int) * (2 * GQ_NB + 1)) != hipSuccess) {
        set_error("gauss exact bins: scratch allocation failed");
        rc = -1;
    }
    if (!rc) rc = gq_perm_lists(P, TG, gperm, growmu, gidx, gidx + GQ_NB + 1, htot, hfirst, s);
    if (!rc) {
        k_gq_exact<<<GQ_NB / 64, 64, 0, s>>>(TG, gperm, gidx, gidx + GQ_NB + 1, growmu, 1.0 / P->c1, xmax, P->gq_exact);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
            set_error("gauss exact bins: kernel failed");
            rc = -1;
        }
    }
    if (gperm) (void)hipFree(gperm);
    if (growmu) (void)hipFree(growmu);
    if (gidx) (void)hipFree(gidx);
    return rc ? -1 : 0;
}

SpectralPlan::~SpectralPlan() { delete (SpecImpl*)impl; }

// one axis of [outer][n][inner]: FFT kernels where the length has an instantiation, GEMM otherwise
static hipError_t dct_pass(const SpecImpl* P, int axis, bool inv, int outer, int inner, const double* in, double* out,
                           hipStream_t s) {
    const double* tab = axis == 0 ? P->Fx : axis == 1 ? P->Fy : P->Ft;
    const int n = axis == 0 ? P->g.Nx : axis == 1 ? P->g.Ny : P->g.Nt;
    const hipError_t e = dct_fft_axis(outer, n, inner, inv, tab, in, out, s);
    if (e != hipErrorNotSupported) return e;
    const double* C = axis == 0 ? (inv ? P->CxT : P->Cx) : axis == 1 ? (inv ? P->CyT : P->Cy) : (inv ? P->CtT : P->Ct);
    return dct_axis(outer, n, inner, C, in, out, s);
}

// 3-D transforms of a single shard: forward = (Ct (x) Cy (x) Cx), inverse = transpose.
static int forward3(SpecImpl* P, double* in, double* scratch, double* out, KTimer* kt, hipStream_t s) {
    const Geo& g = P->g;
    const double N = (double)g.Nt * (double)g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    // in -x-> scratch -y-> in -t-> out   (in is clobbered)
    FOTO_HIP_CHECK(dct_pass(P, 0, false, g.Nt * g.Ny, 1, in, scratch, s));
    FOTO_HIP_CHECK(dct_pass(P, 1, false, g.Nt, g.Nx, scratch, in, s));
    FOTO_HIP_CHECK(dct_pass(P, 2, false, 1, (int)g.nxy, in, out, s));
    if (kt) kt->stop(e, s, FOTO_K_DCT, 6.0 * 8.0 * N);
    return 0;
}

static int inverse3(SpecImpl* P, double* in, double* scratch, double* out, KTimer* kt, hipStream_t s) {
    const Geo& g = P->g;
    const double N = (double)g.Nt * (double)g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    // in -t-> scratch -y-> in -x-> out   (in is clobbered)
    FOTO_HIP_CHECK(dct_pass(P, 2, true, 1, (int)g.nxy, in, scratch, s));
    FOTO_HIP_CHECK(dct_pass(P, 1, true, g.Nt, g.Nx, scratch, in, s));
    FOTO_HIP_CHECK(dct_pass(P, 0, true, g.Nt * g.Ny, 1, in, out, s));
    if (kt) kt->stop(e, s, FOTO_K_DCT, 6.0 * 8.0 * N);
    return 0;
}

static hipError_t launch_s2(SpecImpl* P, bool init, double rtol, int maxiter, double* gath, hipStream_t s) {
    const SpecTab T = P->tab();
    const int nb = P->nblocks2;
    // gath == nullptr: single shard, fused plan (or the separate plan kernel, FOTO_S2_SPLIT=1)
    const bool fuse = (gath == nullptr) && !P->split_plan;
    double* gw = gath ? gath : P->gath;
    if (P->ring) {
        const hipError_t e = launch_s2_ring(T, P->rh, P->ph, P->bh, P->S2, P->rb, rtol, maxiter, gw, P->rank, init, fuse,
                                            FOTO_RING_D, P->nb_ring, s);
        if (e != hipSuccess || gath != nullptr || fuse) return e;
        k_spec_s2_plan<<<1, 64, 0, s>>>(P->S2, P->gath, 1, init ? 1 : 0, rtol, maxiter);
        return hipGetLastError();
    }
#define FOTO_S2_LAUNCH(V, I, F) \
    k_spec_s2<V, I, F><<<nb, S2_NTH, 0, s>>>(T, P->rh, P->ph, P->bh, P->S2, P->rb, rtol, maxiter, gw, P->rank)
    if (P->vec()) {
        if (init) { if (fuse) FOTO_S2_LAUNCH(true, true, true); else FOTO_S2_LAUNCH(true, true, false); }
        else { if (fuse) FOTO_S2_LAUNCH(true, false, true); else FOTO_S2_LAUNCH(true, false, false); }
    } else {
        if (init) { if (fuse) FOTO_S2_LAUNCH(false, true, true); else FOTO_S2_LAUNCH(false, true, false); }
        else { if (fuse) FOTO_S2_LAUNCH(false, false, true); else FOTO_S2_LAUNCH(false, false, false); }
    }
#undef FOTO_S2_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || gath != nullptr || fuse) return e;
    // single shard, split plan: world = 1 plan kernel right behind the pass
    k_spec_s2_plan<<<1, 64, 0, s>>>(P->S2, P->gath, 1, init ? 1 : 0, rtol, maxiter);
    return hipGetLastError();
}

static int reset_s2(SpecImpl* P, hipStream_t s) {
    SStep h{};
    h.c0 = P->c0;
    h.c1 = P->c1;
    h.gc0 = P->c0;
    h.gc1 = P->c1;
    h.ic0 = P->c0;   // the first solve's INIT moments: the whole spectrum
    h.ic1 = P->c1;
    {
        const char* e = getenv("FOTO_SADAPT");   // 0: whole-spectrum interval for every pass (A/B runs)
        h.flags = (e && atoi(e) == 0) ? 1 : 0;
    }
    *P->hS2 = h;
    FOTO_HIP_CHECK(hipMemcpyAsync(P->S2, P->hS2, sizeof(SStep), hipMemcpyHostToDevice, s));
    FOTO_HIP_CHECK(hipStreamSynchronize(s));   // hS2 is reused by polling
    return 0;
}

// init_done: the fused t-axis kernel already reset the state, took r_0's moments and planned
static int solve_s2(SpecImpl* P, double rtol, int maxiter, int predicted, int* iters, int* info, KTimer* kt,
                    hipStream_t s, bool init_done = false) {
    const double N = P->nbox();
    if (!init_done) {
        hipEvent_t e = kt ? kt->start(s) : nullptr;
        FOTO_HIP_CHECK(launch_s2(P, true, rtol, maxiter, nullptr, s));
        if (kt) kt->stop(e, s, FOTO_K_SPEC, 16.0 * N);
    }
    // Host polls the done flag between chunks.  A poll idles the GPU for the host's wake-up
    // (measured up to ~1 ms per solve when polling every pass), while a pass launched after
    // the solve finished exits in a few us -- so over-predict: the first chunk is the previous
    // solve's pass count + 2, then chunks of 2.
    int passes = 0;
    (void)predicted;
    const int first = P->last_passes > 0 ? P->last_passes + 2 : 8;
    while (true) {
        const int chunk = (passes == 0) ? first : 2;
        for (int j = 0; j < chunk; ++j, ++passes) {
            hipEvent_t e = kt ? kt->start(s) : nullptr;
            FOTO_HIP_CHECK(launch_s2(P, false, rtol, maxiter, nullptr, s));
            if (kt) kt->stop(e, s, FOTO_K_SPEC, 32.0 * N);
        }
        FOTO_HIP_CHECK(hipMemcpyAsync(P->hS2, P->S2, sizeof(SStep), hipMemcpyDeviceToHost, s));
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        if (P->hS2->done) break;
        if (passes > maxiter + 4) {
            set_error("spectral s-step CG did not terminate");
            return FOTO_ERR_STATE;
        }
    }
    *iters = P->hS2->iters;
    *info = (P->hS2->done == 1) ? 0 : maxiter;
    P->last_passes = P->hS2->passes;
    // S.passes counts the plans (INIT's and every working pass's but the last), i.e. the
    // passes that applied steps; the launches beyond them exited at once -- keep them out of
    // the per-kernel timing
    if (kt) kt->discard_last(FOTO_K_SPEC, std::max(0, passes - P->hS2->passes));
    return 0;
}

static hipError_t launch_xhat(SpecImpl* P, hipStream_t s) {
    const SpecTab T = P->tab();
    if (P->vec()) k_spec_xhat<true><<<P->nblocks, NT, 0, s>>>(T, P->bh, P->rh, P->tmp);
    else k_spec_xhat<false><<<P->nblocks, NT, 0, s>>>(T, P->bh, P->rh, P->tmp);
    return hipGetLastError();
}

// plan (forward): single shard, the kernel plans the first pass; sharded, it leaves this rank's INIT
// moments in gath for the all-gather
// x^ = Q(lam) b^ (the Gauss-compressed CG's solution table) into a box buffer: persistent
// 1024-thread blocks, the table in LDS.  Sized for the whole table (32 rows, 128 KB) one block
// fits a CU; sized for the first FOTO_GQ_XQL rows (default 17: 68 KB, what K <= ~200 needs;
// the table kernel's qn is not known when this launch is enqueued) two fit, and any rows beyond
// are read from the global table.  (FOTO_GQ_XQL=0: the whole table, one block per CU.)
static hipError_t gq_xhat(SpecImpl* P, double* out, hipStream_t s) {
    const SpecTab T = P->tab();
    const int rows = P->g.Nt * P->nyl;
    static const int xql = [] {
        const char* e = getenv("FOTO_GQ_XQL");
        return e ? atoi(e) : 17;
    }();
    const int ql = (xql > 0 && xql < GQ_QN) ? xql : GQ_QN;
    const int per_cu = (ql < GQ_QN) ? 2 : 1;
    const int nb = std::max(1, std::min(per_cu * cus_count(), (rows + GQ_XNTH / 64 - 1) / (GQ_XNTH / 64)));
    k_gq_xhat<<<nb, GQ_XNTH, (size_t)ql * GQ_QB * sizeof(double), s>>>(T, P->bh, P->gq_tab, P->gq, P->gq_bins,
                                                                       1.0 / P->c1, out, ql);
    return hipGetLastError();
}

// inv: x^ = (b^ - r^)/lam (s-step) or, with P->gauss, Q(lam) b^ from the Gauss-compressed CG's table
static hipError_t launch_tcol(SpecImpl* P, bool inv, const double* in, double* out, double rtol, int maxiter,
                              hipStream_t s, int mode = TC_PLAN) {
    const SpecTab T = P->tab();
    const int nb = P->tcol_nb;
    const bool gq = inv && P->gauss_active;
    // one thread per column with the table in LDS: x^ = Q(lam) b^ inside the inverse t-DCT
    bool tfuse = false;
#define FOTO_TFUSE_NT(NN) tfuse = tfuse || P->g.Nt == NN;
    FOTO_TCOL_SIZES(FOTO_TFUSE_NT)   // (one thread per column: Nt <= 32)
#undef FOTO_TFUSE_NT
    tfuse = tfuse && gq && P->gq_tfuse;
    if (gq && !tfuse) {   // x^ -> rh, then the plain inverse below
        const hipError_t e = gq_xhat(P, P->rh, s);
        if (e != hipSuccess) return e;
    }
    if (tfuse) {
        const int ql = 17;   // 2 blocks of 512 per CU (<= 80 KB of LDS each); rows beyond from the global table
        const int nbf = (int)(((int64_t)P->nyl * P->g.Nx + GQ_TFNTH - 1) / GQ_TFNTH);
#define FOTO_TFUSE_LAUNCH(NN)                                                                                      \
        if (P->g.Nt == NN) {                                                                                       \
            k_dct_t_inv_gq<NN><<<nbf, GQ_TFNTH, (size_t)ql * GQ_QB * sizeof(double), s>>>(                         \
                    T, P->Cth, P->bh, P->gq_tab, P->gq, P->gq_bins, 1.0 / P->c1, out, ql);                       \
            return hipGetLastError();                                                                              \
        }
        FOTO_TCOL_SIZES(FOTO_TFUSE_LAUNCH)
#undef FOTO_TFUSE_LAUNCH
        return hipErrorNotSupported;
    }
#define FOTO_TCOL_FWD(NN, K, M) K<NN, M><<<nb, TC_NTH, 0, s>>>(T, P->Cth, in, P->bh, P->S2, P->rb, rtol, maxiter, \
                                                                P->gath, P->rank)
#define FOTO_TCOL_LAUNCH(NN)                                                                                       \
    if (P->g.Nt == NN) {                                                                                           \
        if (gq) k_dct_t_inv_xhat<NN, true><<<nb, TC_NTH, 0, s>>>(T, P->Cth, P->rh, nullptr, nullptr, out);         \
        else if (inv) k_dct_t_inv_xhat<NN><<<nb, TC_NTH, 0, s>>>(T, P->Cth, P->bh, P->rh, P->S2, out);             \
        else if (mode == TC_PLAN) FOTO_TCOL_FWD(NN, k_dct_t_fwd_init, TC_PLAN);                                    \
        else if (mode == TC_GATH) FOTO_TCOL_FWD(NN, k_dct_t_fwd_init, TC_GATH);                                    \
        else FOTO_TCOL_FWD(NN, k_dct_t_fwd_init, TC_PLAIN);                                                        \
        return hipGetLastError();                                                                                  \
    }
    FOTO_TCOL_SIZES(FOTO_TCOL_LAUNCH)
#undef FOTO_TCOL_LAUNCH
#define FOTO_TPAIR_LAUNCH(NN)                                                                                      \
    if (P->g.Nt == NN) {                                                                                           \
        if (gq) k_dct_tp_inv_xhat<NN, true><<<nb, TC_NTH, 0, s>>>(T, P->Cth, P->rh, nullptr, nullptr, out);        \
        else if (inv) k_dct_tp_inv_xhat<NN><<<nb, TC_NTH, 0, s>>>(T, P->Cth, P->bh, P->rh, P->S2, out);            \
        else if (mode == TC_PLAN) FOTO_TCOL_FWD(NN, k_dct_tp_fwd_init, TC_PLAN);                                   \
        else if (mode == TC_GATH) FOTO_TCOL_FWD(NN, k_dct_tp_fwd_init, TC_GATH);                                   \
        else FOTO_TCOL_FWD(NN, k_dct_tp_fwd_init, TC_PLAIN);                                                       \
        return hipGetLastError();                                                                                  \
    }
    FOTO_TPAIR_SIZES(FOTO_TPAIR_LAUNCH)
#undef FOTO_TPAIR_LAUNCH
#undef FOTO_TCOL_FWD
    return hipErrorNotSupported;
}

// (b^, r^) -t(+xhat)-> b -y-> tmp -x-> x
static int tcol_inverse(SpecImpl* P, double* b, double* x, double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    const Geo& g = P->g;
    const double N = (double)g.Nt * (double)g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    FOTO_HIP_CHECK(launch_tcol(P, true, nullptr, b, rtol, maxiter, s));
    FOTO_HIP_CHECK(dct_pass(P, 1, true, g.Nt, g.Nx, b, P->tmp, s));
    FOTO_HIP_CHECK(dct_pass(P, 0, true, g.Nt * g.Ny, 1, P->tmp, x, s));
    if (kt) kt->stop(e, s, FOTO_K_DCT, 7.0 * 8.0 * N);
    return 0;
}

// ---------------------------------------------------------------------------- Gauss-compressed CG (host)
// one shard, wave-per-bin nodes: k_gq_nodes_w sums the chunk sums itself (no histogram pass)
static bool gq_fused_reduce(const SpecImpl* P) { return P->gq_nodes_wave && P->world == 1; }

// b^ -> this box's histogram (slot rank of gq_hist)
static int gq_measure(SpecImpl* P, KTimer* kt, hipStream_t s) {
    const SpecTab T = P->tab();
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    const int nbk = std::max(1, (P->gq_nch + 3) / 4);
    k_gq_hist_perm<<<nbk, 256, 0, s>>>(T, P->bh, P->gq_permv, P->gq_chunks, P->gq_nch, P->gq_bins, P->gq_exact,
                                       P->gq_rowmu, 1.0 / P->c1, P->gq_ppart);
    FOTO_HIP_CHECK(hipGetLastError());
    // (one shard with the wave-per-bin node kernel: the bin sums are taken there, from the chunk sums)
    if (!gq_fused_reduce(P)) {
        k_gq_perm_reduce<<<GQ_HIST / 4, 256, 0, s>>>(P->gq_ppart, P->gq_cfirst, P->gq_hist + (size_t)P->rank * GQ_HIST);
        FOTO_HIP_CHECK(hipGetLastError());
    }
    if (kt) kt->stop(e, s, FOTO_K_SPEC, 8.0 * P->nbox());
    return 0;
}

// k_gq_cgtab's slots as a fresh plan has them: every (alpha, beta) NaN, kdone -1, ticket 0
static int gq_pub_clear(SpecImpl* P, hipStream_t s) {
    if (!P->gq_pub) return 0;
    FOTO_HIP_CHECK(hipMemsetAsync(P->gq_pub, 0xff, sizeof(GqPub), s));   // (all-ones: NaN, -1)
    FOTO_HIP_CHECK(hipMemsetAsync(&P->gq_pub->ticket, 0, sizeof(unsigned), s));
    return 0;
}

// the world histograms -> Gauss nodes -> CG coefficients -> solution table; header to host
static int gq_solve(SpecImpl* P, double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    if (!P->gq_nodes_wave)
        k_gq_nodes<<<GQ_NODES / 64, 64, 0, s>>>(P->gq_hist, P->gq_bins, P->gq_exact, P->world, P->r * P->eps, P->c1, P->gqn);
    else if (gq_fused_reduce(P))
        k_gq_nodes_w<<<GQ_NB / 4, 256, 0, s>>>(nullptr, P->gq_ppart, P->gq_cfirst, P->gq_bins, P->gq_exact, 1,
                                               P->r * P->eps, P->c1, P->gqn);
    else
        k_gq_nodes_w<<<GQ_NB / 4, 256, 0, s>>>(P->gq_hist, nullptr, nullptr, P->gq_bins, P->gq_exact, P->world,
                                               P->r * P->eps, P->c1, P->gqn);
    FOTO_HIP_CHECK(hipGetLastError());
    const char* kl = getenv("FOTO_GQ_KLIM");   // (tests: force the s-step redo path)
    const int klim = kl ? std::max(0, std::min(GQ_KMAX, atoi(kl))) : GQ_KMAX;
    // the header to the host slot: stored by the CG kernel itself (FOTO_HOST_CRIT=0: a copy)
    P->hlast = P->hslot;
    P->hslot ^= 1;
    const char* hc = getenv("FOTO_HOST_CRIT");
    const bool direct = !(hc && atoi(hc) == 0);
    if (P->gq_cgtab) {
        k_gq_cgtab<<<1 + GQ_TAB / 256, 256, 0, s>>>(P->gqn, rtol, maxiter, klim, P->gq,
                                                    direct ? P->dgq2[P->hlast] : nullptr, P->gq_pub, P->gq_bins,
                                                    P->gq_qcos, P->r * P->eps, P->c1, P->gq_tab);
        FOTO_HIP_CHECK(hipGetLastError());
    } else {
        k_gq_cg<<<1, GQ_CGNTH, 0, s>>>(P->gqn, rtol, maxiter, klim, P->gq, direct ? P->dgq2[P->hlast] : nullptr);
        FOTO_HIP_CHECK(hipGetLastError());
        k_gq_qtab<<<GQ_TAB / 256, 256, 0, s>>>(P->gq, P->gq_bins, P->gq_qcos, P->r * P->eps, P->c1, P->gq_tab);
        FOTO_HIP_CHECK(hipGetLastError());
    }
    if (kt) kt->stop(e, s, FOTO_K_SPEC, 0.0);
    if (!direct)
        FOTO_HIP_CHECK(hipMemcpyAsync(P->hgq2[P->hlast], P->gq, offsetof(GqState, alpha), hipMemcpyDeviceToHost, s));
    P->gauss_active = true;
    return 0;
}

// a failed solve broke the done chain (k_gq_cg); once it is redone, later solves may run again
static int gq_unbreak(SpecImpl* P, hipStream_t s) {
    FOTO_HIP_CHECK(hipMemsetAsync(&P->gq->broken, 0, sizeof(int), s));
    return 0;
}


// single shard: b (physical) -> b^ -> measure -> CG -> x, all enqueued.  b is only read: the
// transforms run through the box buffers (b -x-> tmp -y-> rh -t-> b^; x^ -> rh / tmp ... -> x),
// so F survives a solve whose prox was skipped -- a failed solve with the next outer iteration
// already enqueued behind it (foto_bb.cpp) then finds its right-hand side intact.
static int gq_enqueue(SpecImpl* P, const double* b, double* x, double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    const Geo& g = P->g;
    const double N = (double)g.Nt * (double)g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    if (P->xt) {   // b -(x, t)-> tmp -y-> b^: two passes (k_dct_xt_fwd)
        FOTO_HIP_CHECK(dct_xt(g.Nt, g.Ny, g.Nx, false, P->Fx, P->Cth, b, P->tmp, s));
        FOTO_HIP_CHECK(dct_pass(P, 1, false, g.Nt, g.Nx, P->tmp, P->bh, s));
        if (kt) kt->stop(e, s, FOTO_K_DCT, 4.0 * 8.0 * N);
    } else {
        FOTO_HIP_CHECK(dct_pass(P, 0, false, g.Nt * g.Ny, 1, b, P->tmp, s));
        FOTO_HIP_CHECK(dct_pass(P, 1, false, g.Nt, g.Nx, P->tmp, P->rh, s));
        if (P->tcol) FOTO_HIP_CHECK(launch_tcol(P, false, P->rh, nullptr, rtol, maxiter, s, TC_PLAIN));
        else FOTO_HIP_CHECK(dct_pass(P, 2, false, 1, (int)g.nxy, P->rh, P->bh, s));
        if (kt) kt->stop(e, s, FOTO_K_DCT, 6.0 * 8.0 * N);
    }
    FOTO_TRY(gq_measure(P, kt, s));
    FOTO_TRY(gq_solve(P, rtol, maxiter, kt, s));
    e = kt ? kt->start(s) : nullptr;
    if (P->xt) {   // x^ -> rh -y-> tmp -(t, x)-> x (k_dct_tx_inv)
        FOTO_HIP_CHECK(gq_xhat(P, P->rh, s));
        FOTO_HIP_CHECK(dct_pass(P, 1, true, g.Nt, g.Nx, P->rh, P->tmp, s));
        FOTO_HIP_CHECK(dct_xt(g.Nt, g.Ny, g.Nx, true, P->Fx, P->Cth, P->tmp, x, s));
        if (kt) kt->stop(e, s, FOTO_K_DCT, 6.0 * 8.0 * N);
        return 0;
    }
    if (P->tcol) {
        FOTO_HIP_CHECK(launch_tcol(P, true, nullptr, P->tmp, rtol, maxiter, s));   // x^ -> rh, t^-1 -> tmp
    } else {
        FOTO_HIP_CHECK(gq_xhat(P, P->rh, s));
        FOTO_HIP_CHECK(dct_pass(P, 2, true, 1, (int)g.nxy, P->rh, P->tmp, s));
    }
    FOTO_HIP_CHECK(dct_pass(P, 1, true, g.Nt, g.Nx, P->tmp, P->rh, s));
    FOTO_HIP_CHECK(dct_pass(P, 0, true, g.Nt * g.Ny, 1, P->rh, x, s));
    if (kt) kt->stop(e, s, FOTO_K_DCT, 7.0 * 8.0 * N);
    return 0;
}

// the s-step CG from b^ (still intact) when the tables could not represent the solve
static int gq_redo(SpecImpl* P, double* b, double* x, double rtol, int maxiter, int* iters, int* info, KTimer* kt,
                   hipStream_t s) {
    P->gauss_active = false;
    FOTO_TRY(gq_unbreak(P, s));
    FOTO_TRY(solve_s2(P, rtol, maxiter, 0, iters, info, kt, s, false));
    if (P->tcol) return tcol_inverse(P, b, x, rtol, maxiter, kt, s);
    FOTO_HIP_CHECK(launch_xhat(P, s));
    return inverse3(P, P->tmp, b, x, kt, s);
}

// after the stream has passed the header copy of the solve in ring slot h
static void gq_result(const SpecImpl* P, int h, int maxiter, int* iters, int* info) {
    *iters = P->hgq2[h]->K;
    *info = P->hgq2[h]->conv ? 0 : maxiter;
}

// single shard, s-step, column-kernel t axis: b -x-> tmp -y-> b -t(+INIT)-> b^; CG passes;
// (b^, r^) -t(+xhat)-> b -y-> tmp -x-> x
static int solve_tcol(SpecImpl* P, double* b, double* x, double rtol, int maxiter, int predicted, int* iters,
                      int* info, KTimer* kt, hipStream_t s) {
    const Geo& g = P->g;
    const double N = (double)g.Nt * (double)g.nxy;
    // no reset_s2 here (a host wait per solve): the INIT plan rewrites every field but the
    // constant c0, c1, which init() set
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    FOTO_HIP_CHECK(dct_pass(P, 0, false, g.Nt * g.Ny, 1, b, P->tmp, s));
    FOTO_HIP_CHECK(dct_pass(P, 1, false, g.Nt, g.Nx, P->tmp, b, s));
    FOTO_HIP_CHECK(launch_tcol(P, false, b, nullptr, rtol, maxiter, s));
    if (kt) kt->stop(e, s, FOTO_K_DCT, 6.0 * 8.0 * N);
    FOTO_TRY(solve_s2(P, rtol, maxiter, predicted, iters, info, kt, s, true));
    return tcol_inverse(P, b, x, rtol, maxiter, kt, s);
}

bool SpectralPlan::deferrable() const {
    const SpecImpl* P = (const SpecImpl*)impl;
    if (P->gauss) return P->world == 1 && P->npend < 2;   // fixed work: nothing to predict
    return P->tcol && P->sstep == 2 && P->world == 1 && P->last_passes > 0 && P->npend == 0;
}

const int* SpectralPlan::done_flag() const {
    const SpecImpl* P = (const SpecImpl*)impl;
    return P->gauss ? &P->gq->done : &P->S2->done;
}

int SpectralPlan::pending() const { return ((const SpecImpl*)impl)->npend; }

int SpectralPlan::solve_deferred(double* b, double* x, double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    if (!deferrable()) {
        set_error("spectral CG: deferred solve needs a single-shard plan with a free slot (s-step: after a finished solve)");
        return FOTO_ERR_STATE;
    }
    SpecImpl::Pend& d = P->pq[P->npend];
    d.b = b;
    d.x = x;
    d.rtol = rtol;
    d.maxiter = maxiter;
    d.launched = 0;
    if (P->gauss) {
        FOTO_TRY(gq_enqueue(P, b, x, rtol, maxiter, kt, s));
        d.hslot = P->hlast;
        ++P->npend;
        return 0;
    }
    const Geo& g = P->g;
    const double N = (double)g.Nt * (double)g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    FOTO_HIP_CHECK(dct_pass(P, 0, false, g.Nt * g.Ny, 1, b, P->tmp, s));
    FOTO_HIP_CHECK(dct_pass(P, 1, false, g.Nt, g.Nx, P->tmp, b, s));
    FOTO_HIP_CHECK(launch_tcol(P, false, b, nullptr, rtol, maxiter, s));
    if (kt) kt->stop(e, s, FOTO_K_DCT, 6.0 * 8.0 * N);
    // the previous solve's pass count + margin (passes past the end exit at once);
    // FOTO_CG_MARGIN overrides the default 2 (tests force the redo path with a negative one)
    const char* me = getenv("FOTO_CG_MARGIN");
    const int margin = me ? atoi(me) : 2;
    const int n = std::max(1, P->last_passes + margin);
    for (int j = 0; j < n; ++j) {
        hipEvent_t ep = kt ? kt->start(s) : nullptr;
        FOTO_HIP_CHECK(launch_s2(P, false, rtol, maxiter, nullptr, s));
        if (kt) kt->stop(ep, s, FOTO_K_SPEC, 32.0 * N);
    }
    FOTO_HIP_CHECK(hipMemcpyAsync(P->hS2, P->S2, sizeof(SStep), hipMemcpyDeviceToHost, s));
    FOTO_TRY(tcol_inverse(P, b, x, rtol, maxiter, kt, s));
    d.launched = n;
    ++P->npend;
    return 0;
}

bool SpectralPlan::oldest_needs_redo() const {
    const SpecImpl* P = (const SpecImpl*)impl;
    if (P->npend == 0) return false;
    if (P->gauss) return P->hgq2[P->pq[0].hslot]->status != 0;
    return !P->hS2->done;
}

int SpectralPlan::drop_newest(hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    if (P->npend == 0 || !P->gauss) {
        set_error("spectral CG: no Gauss solve in flight to drop");
        return FOTO_ERR_STATE;
    }
    --P->npend;
    // the dropped solve may have failed or followed a failed one: its flags mean nothing now
    return gq_unbreak(P, s);
}

int SpectralPlan::finish(int* iters, int* info, int* redo, KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    if (P->npend == 0) {
        set_error("spectral CG: no deferred solve to finish");
        return FOTO_ERR_STATE;
    }
    const SpecImpl::Pend d = P->pq[0];
    P->pq[0] = P->pq[1];
    --P->npend;
    *redo = 0;
    if (P->gauss) {
        if (P->hgq2[d.hslot]->status != 0) {   // K beyond the table or a breakdown: the s-step CG from b^
            if (P->npend != 0) {
                set_error("spectral CG: a failed solve must be redone before the next one runs (drop it first)");
                return FOTO_ERR_STATE;
            }
            *redo = 1;
            return gq_redo(P, d.b, d.x, d.rtol, d.maxiter, iters, info, kt, s);
        }
        gq_result(P, d.hslot, d.maxiter, iters, info);
        if (P->npend == 0) P->gauss_active = false;
        return 0;
    }
    int passes = d.launched;
    if (!P->hS2->done) {   // the predicted passes were not enough: continue, polling, and redo x
        *redo = 1;
        const double N = P->nbox();
        while (!P->hS2->done) {
            for (int j = 0; j < 2; ++j, ++passes) {
                hipEvent_t e = kt ? kt->start(s) : nullptr;
                FOTO_HIP_CHECK(launch_s2(P, false, d.rtol, d.maxiter, nullptr, s));
                if (kt) kt->stop(e, s, FOTO_K_SPEC, 32.0 * N);
            }
            FOTO_HIP_CHECK(hipMemcpyAsync(P->hS2, P->S2, sizeof(SStep), hipMemcpyDeviceToHost, s));
            FOTO_HIP_CHECK(hipStreamSynchronize(s));
            if (passes > d.maxiter + 4) {
                set_error("spectral s-step CG did not terminate");
                return FOTO_ERR_STATE;
            }
        }
        FOTO_TRY(tcol_inverse(P, d.b, d.x, d.rtol, d.maxiter, kt, s));
    }
    *iters = P->hS2->iters;
    *info = (P->hS2->done == 1) ? 0 : d.maxiter;
    P->last_passes = P->hS2->passes;
    if (kt) kt->discard_last(FOTO_K_SPEC, std::max(0, passes - P->hS2->passes));
    return 0;
}

int SpectralPlan::solve(double* b, double* x, double rtol, int maxiter, int predicted, int* iters, int* info,
                        KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    const Geo& g = P->g;
    const SpecTab T = P->tab();
    const double N = (double)g.Nt * (double)g.nxy;
    const bool vec = P->vec();
    if (P->gauss) {
        FOTO_TRY(gq_enqueue(P, b, x, rtol, maxiter, kt, s));
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        if (P->hgq2[P->hlast]->status != 0) return gq_redo(P, b, x, rtol, maxiter, iters, info, kt, s);
        gq_result(P, P->hlast, maxiter, iters, info);
        P->gauss_active = false;
        return 0;
    }
    if (P->tcol) return solve_tcol(P, b, x, rtol, maxiter, predicted, iters, info, kt, s);
    // b (physical) -> b^ ; b is scratch afterwards
    FOTO_TRY(forward3(P, b, P->tmp, P->bh, kt, s));
    if (P->sstep == 2) {
        FOTO_TRY(solve_s2(P, rtol, maxiter, predicted, iters, info, kt, s));
        FOTO_HIP_CHECK(launch_xhat(P, s));
        FOTO_TRY(inverse3(P, P->tmp, b, x, kt, s));
        return 0;
    }
    if (vec) k_spec_init<true><<<P->nblocks, NT, 0, s>>>(T, P->bh, P->rh, P->rb, P->gath);
    else k_spec_init<false><<<P->nblocks, NT, 0, s>>>(T, P->bh, P->rh, P->rb, P->gath);
    FOTO_HIP_CHECK(hipGetLastError());
    FOTO_HIP_CHECK(hipMemsetAsync(P->S, 0, sizeof(CGScal), s));
    int k = 0;
    bool done = false;
    const int first = predicted > 4 ? predicted - 3 : 8;
    while (k < maxiter) {
        int chunk = (k == 0) ? first : 2;
        chunk = std::min(chunk, maxiter - k);
        for (int j = 0; j < chunk; ++j, ++k) {
            hipEvent_t e = kt ? kt->start(s) : nullptr;
            if (vec) k_spec_cg<true><<<P->nblocks, NT, 0, s>>>(T, k, P->rh, P->ph, P->S, P->rb, P->gath, rtol);
            else k_spec_cg<false><<<P->nblocks, NT, 0, s>>>(T, k, P->rh, P->ph, P->S, P->rb, P->gath, rtol);
            FOTO_HIP_CHECK(hipGetLastError());
            if (kt) kt->stop(e, s, FOTO_K_SPEC, (k == 0 ? 24.0 : 32.0) * N);
        }
        FOTO_HIP_CHECK(hipMemcpyAsync(P->hS, P->S, sizeof(CGScal), hipMemcpyDeviceToHost, s));
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        if (P->hS->done) { done = true; break; }
    }
    *iters = done ? P->hS->iters : maxiter;
    *info = done ? 0 : maxiter;
    if (vec) k_spec_xhat<true><<<P->nblocks, NT, 0, s>>>(T, P->bh, P->rh, P->tmp);
    else k_spec_xhat<false><<<P->nblocks, NT, 0, s>>>(T, P->bh, P->rh, P->tmp);
    FOTO_HIP_CHECK(hipGetLastError());
    FOTO_TRY(inverse3(P, P->tmp, b, x, kt, s));
    return 0;
}

// ----------------------------------------------------------------------------- sharded phases
// Physical slab [tl][y][x] (planes t0..t0+nloc) <-> spectral box [kt][ky - y0][kx].

int SpectralPlan::fwd_local(double* b, int lo, int hi, KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    const Geo& g = P->g;
    if (lo < 0 || hi > g.nloc || hi <= lo) {
        set_error("spectral CG: fwd_local planes [%d, %d) outside the slab", lo, hi);
        return FOTO_ERR_ARG;
    }
    const int np = hi - lo;
    const int64_t o = (int64_t)lo * g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    FOTO_HIP_CHECK(dct_pass(P, 0, false, np * g.Ny, 1, b + o, P->tmpp + o, s));   // x
    FOTO_HIP_CHECK(dct_pass(P, 1, false, np, g.Nx, P->tmpp + o, b + o, s));       // y (b: the all-to-all's source)
    if (kt) kt->stop(e, s, FOTO_K_SLAB, 4.0 * 8.0 * (double)np * (double)g.nxy);
    return 0;
}

int SpectralPlan::fwd_t(KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    const Geo& g = P->g;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    if (P->tcol)   // box tmp -> b^ and this rank's INIT moments -> gath (cg_begin then launches nothing)
        FOTO_HIP_CHECK(launch_tcol(P, false, P->tmp, nullptr, 0.0, 0, s, P->gauss ? TC_PLAIN : TC_GATH));
    else
        FOTO_HIP_CHECK(dct_pass(P, 2, false, 1, P->nyl * g.Nx, P->tmp, P->bh, s));   // box tmp -> b^
    if (kt) kt->stop(e, s, FOTO_K_DCT, 2.0 * 8.0 * P->nbox());
    return 0;
}

int SpectralPlan::cg_begin(double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    if (P->tcol && !P->gauss) return 0;   // the column kernel of fwd_t took the INIT moments
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    FOTO_HIP_CHECK(launch_s2(P, true, rtol, maxiter, P->gath, s));
    if (kt) kt->stop(e, s, FOTO_K_SPEC, 16.0 * P->nbox());
    return 0;
}

int SpectralPlan::cg_pass(double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    if (P->late_plan())   // plans at its start from the all-gathered moments (no cg_plan after it)
        FOTO_HIP_CHECK(launch_s2_ring(P->tab(), P->rh, P->ph, P->bh, P->S2, P->rb, rtol, maxiter, P->gath, P->rank,
                                      false, true, FOTO_RING_D, P->nb_ring, s, P->world));
    else
        FOTO_HIP_CHECK(launch_s2(P, false, rtol, maxiter, P->gath, s));
    if (kt) kt->stop(e, s, FOTO_K_SPEC, 32.0 * P->nbox());
    return 0;
}

int SpectralPlan::cg_plan(int init, double rtol, int maxiter, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    if (!init && P->late_plan()) return 0;   // the next cg_pass plans at its start
    k_spec_s2_plan<<<1, 64, 0, s>>>(P->S2, P->gath, P->world, init, rtol, maxiter);
    FOTO_HIP_CHECK(hipGetLastError());
    return 0;
}

int SpectralPlan::poll(int* done, int* iters, int* passes, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    FOTO_HIP_CHECK(hipMemcpyAsync(P->hS2, P->S2, sizeof(SStep), hipMemcpyDeviceToHost, s));
    FOTO_HIP_CHECK(hipStreamSynchronize(s));
    *done = P->hS2->done;
    *iters = P->hS2->iters;
    *passes = P->hS2->passes;
    return 0;
}

int SpectralPlan::inv_t(KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    const Geo& g = P->g;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    if (P->tcol) {   // x^ and the inverse t-DCT in one column kernel: tmp = box of x~ (box_out)
        FOTO_HIP_CHECK(launch_tcol(P, true, nullptr, P->tmp, 0.0, 0, s));
        if (kt) kt->stop(e, s, FOTO_K_DCT, 3.0 * 8.0 * P->nbox());
        return 0;
    }
    if (P->gauss_active) FOTO_HIP_CHECK(gq_xhat(P, P->tmp, s));                     // tmp = x^
    else FOTO_HIP_CHECK(launch_xhat(P, s));
    FOTO_HIP_CHECK(dct_pass(P, 2, true, 1, P->nyl * g.Nx, P->tmp, P->rh, s));    // rh = box of x~
    if (kt) kt->stop(e, s, FOTO_K_DCT, 2.0 * 8.0 * P->nbox());
    return 0;
}

int SpectralPlan::inv_local(double* scratch, double* x, int lo, int hi, KTimer* kt, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    const Geo& g = P->g;
    if (lo < -1 || hi > g.nloc + 1 || hi <= lo) {   // (one halo plane per side: phi's halo)
        set_error("spectral CG: inv_local planes [%d, %d) outside the slab and its halo", lo, hi);
        return FOTO_ERR_ARG;
    }
    const int np = hi - lo;
    const int64_t o = (int64_t)lo * g.nxy;
    hipEvent_t e = kt ? kt->start(s) : nullptr;
    FOTO_HIP_CHECK(dct_pass(P, 1, true, np, g.Nx, scratch + o, P->tmpp + o, s));   // y (scratch: the all-to-all's target)
    FOTO_HIP_CHECK(dct_pass(P, 0, true, np * g.Ny, 1, P->tmpp + o, x + o, s));     // x
    if (kt) kt->stop(e, s, FOTO_K_SLAB, 4.0 * 8.0 * (double)np * (double)g.nxy);
    return 0;
}

bool SpectralPlan::gauss() const { return ((const SpecImpl*)impl)->gauss; }
int SpectralPlan::gauss_hist_size() { return GQ_HIST; }
double* SpectralPlan::gauss_hist() const { return ((const SpecImpl*)impl)->gq_hist; }

int SpectralPlan::gauss_measure(KTimer* kt, hipStream_t s) { return gq_measure((SpecImpl*)impl, kt, s); }

int SpectralPlan::gauss_solve(double rtol, int maxiter, KTimer* kt, hipStream_t s) {
    return gq_solve((SpecImpl*)impl, rtol, maxiter, kt, s);
}

int SpectralPlan::gauss_wait(int maxiter, int* ok, int* iters, int* info, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    FOTO_HIP_CHECK(hipStreamSynchronize(s));
    *ok = P->hgq2[P->hlast]->status == 0;
    gq_result(P, P->hlast, maxiter, iters, info);
    if (!*ok) {
        P->gauss_active = false;
        FOTO_TRY(gq_unbreak(P, s));   // the s-step CG redoes this solve (foto_bb.cpp)
    }
    return 0;
}

int SpectralPlan::gauss_result(int maxiter, int* ok, int* iters, int* info, hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    *ok = P->hgq2[P->hlast]->status == 0;
    gq_result(P, P->hlast, maxiter, iters, info);
    P->gauss_active = false;
    if (!*ok) FOTO_TRY(gq_unbreak(P, s));
    return 0;
}

void SpectralPlan::gauss_end() { ((SpecImpl*)impl)->gauss_active = false; }

int SpectralPlan::reset(hipStream_t s) {
    SpecImpl* P = (SpecImpl*)impl;
    P->npend = 0;
    P->gauss_active = false;
    if (P->gq) FOTO_HIP_CHECK(hipMemsetAsync(P->gq, 0, sizeof(GqState), s));
    FOTO_TRY(gq_pub_clear(P, s));
    P->last_passes = 0;
    FOTO_HIP_CHECK(hipMemsetAsync(P->S, 0, sizeof(CGScal), s));
    FOTO_HIP_CHECK(hipMemsetAsync(P->rb.ticket, 0, 8 * sizeof(double), s));
    return reset_s2(P, s);
}

double* SpectralPlan::box_in() const { return ((SpecImpl*)impl)->tmp; }
double* SpectralPlan::box_out() const {
    const SpecImpl* P = (const SpecImpl*)impl;
    return P->tcol ? P->tmp : P->rh;
}
double* SpectralPlan::gath() const { return ((SpecImpl*)impl)->gath; }
int SpectralPlan::moments() { return NACC; }
int SpectralPlan::y0() const { return ((SpecImpl*)impl)->y0; }
int SpectralPlan::nyl() const { return ((SpecImpl*)impl)->nyl; }

}  // namespace foto

// ============================================================================ C ABI: one DCT axis (test entry)

extern "C" int foto_dct(const double* in, int outer, int n, int inner, int inverse, int path, double* out) {
    using namespace foto;
    if (!in || !out || outer < 1 || n < 2 || inner < 1 || path < 0 || path > 2) {
        set_error("foto_dct: bad arguments");
        return FOTO_ERR_ARG;
    }
    const size_t tot = (size_t)outer * n * inner;
    hipStream_t s = nullptr;
    FOTO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<void*> bufs;
    auto dev = [&](size_t nd, double** p) -> int {
        FOTO_HIP_CHECK(hipMalloc((void**)p, std::max<size_t>(nd, 1) * 8));
        bufs.push_back(*p);
        return 0;
    };
    auto body = [&]() -> int {
        double *din, *dout, *dtab = nullptr, *dC;
        FOTO_TRY(dev(tot, &din));
        FOTO_TRY(dev(tot, &dout));
        FOTO_HIP_CHECK(hipMemcpyAsync(din, in, tot * 8, hipMemcpyHostToDevice, s));
        int m1, m2;
        hipError_t e = hipErrorNotSupported;
        if (path != 2 && fft_factors(n, &m1, &m2)) {
            const std::vector<double> t = fft_table(n);
            FOTO_TRY(dev(t.size(), &dtab));
            FOTO_HIP_CHECK(hipMemcpyAsync(dtab, t.data(), t.size() * 8, hipMemcpyHostToDevice, s));
            FOTO_HIP_CHECK(hipStreamSynchronize(s));
            e = dct_fft_axis(outer, n, inner, inverse != 0, dtab, din, dout, s);
        }
        if (e == hipErrorNotSupported) {
            if (path == 1) { set_error("foto_dct: no FFT plan for n = %d", n); return FOTO_ERR_ARG; }
            std::vector<double> C, CT, mu;
            dct_matrix(n, C, CT, mu);
            FOTO_TRY(dev(C.size(), &dC));
            FOTO_HIP_CHECK(hipMemcpyAsync(dC, inverse ? CT.data() : C.data(), C.size() * 8, hipMemcpyHostToDevice, s));
            FOTO_HIP_CHECK(hipStreamSynchronize(s));
            e = dct_axis(outer, n, inner, dC, din, dout, s);
        }
        FOTO_HIP_CHECK(e);
        FOTO_HIP_CHECK(hipMemcpyAsync(out, dout, tot * 8, hipMemcpyDeviceToHost, s));
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        return 0;
    };
    const int rc = body();
    (void)hipStreamSynchronize(s);
    for (void* p : bufs) (void)hipFree(p);
    (void)hipStreamDestroy(s);
    return rc;
}

// ============================================================================ C ABI: stream ceiling probe
// The s-step pass's memory traffic alone -- read r, q (16 B per lane), write r, q -- with no
// moments, no plan and no reduction: what the dominant kernel could reach on this device.
// bench.py reports the pass against it (roofline.stream_frac) beside the HBM-peak fraction,
// because the pass's 157 MB working set sits in the 256 MiB Infinity Cache.

namespace foto {
__global__ __launch_bounds__(256) void k_stream_fill(double* __restrict__ r, double* __restrict__ q, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        r[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5;
        q[i] = 1e-3 * (double)((i * 40503u + 7) % 1000) - 0.5;
    }
}

template <bool WT>
__global__ __launch_bounds__(256) void k_stream_rq(double* __restrict__ r, double* __restrict__ q, int64_t n2,
                                                   double a, double b) {
    const __amdgpu_buffer_rsrc_t rr = wt_rsrc(r), rq = wt_rsrc(q);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        const dbl2 rv = reinterpret_cast<const dbl2*>(r)[i], qv = reinterpret_cast<const dbl2*>(q)[i];
        const dbl2 pn = b * qv + rv, rn = rv - a * pn;
        if (WT) {
            st_wt16(rr, (int)(i * 16), rn);
            st_wt16(rq, (int)(i * 16), pn);
        } else {
            reinterpret_cast<dbl2*>(r)[i] = rn;
            reinterpret_cast<dbl2*>(q)[i] = pn;
        }
    }
}
// the prox + RHS traffic: 4 fields in, 4 out, 16 B per lane per field (ping-pong between the
// two sets of four so every launch streams from HBM)
__global__ __launch_bounds__(256) void k_stream_4x4(const double* __restrict__ a0, const double* __restrict__ a1,
                                                    const double* __restrict__ a2, const double* __restrict__ a3,
                                                    double* __restrict__ b0, double* __restrict__ b1,
                                                    double* __restrict__ b2, double* __restrict__ b3, int64_t n2, double c) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n2; i += (int64_t)gridDim.x * 256) {
        const dbl2 x0 = reinterpret_cast<const dbl2*>(a0)[i], x1 = reinterpret_cast<const dbl2*>(a1)[i];
        const dbl2 x2 = reinterpret_cast<const dbl2*>(a2)[i], x3 = reinterpret_cast<const dbl2*>(a3)[i];
        reinterpret_cast<dbl2*>(b0)[i] = x1 + c * x0;
        reinterpret_cast<dbl2*>(b1)[i] = x2 + c * x0;
        reinterpret_cast<dbl2*>(b2)[i] = x3 + c * x0;
        reinterpret_cast<dbl2*>(b3)[i] = x0 - c * (x1 + x2);
    }
}
}  // namespace foto

extern "C" int foto_stream_probe4(int64_t n, int reps, double* us) {
    using namespace foto;
    if (!us || n < 2 || n % 2 || reps < 1) {
        set_error("foto_stream_probe4: bad arguments (n even)");
        return FOTO_ERR_ARG;
    }
    hipStream_t s = nullptr;
    double* f[8] = {nullptr};
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto body = [&]() -> int {
        FOTO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        for (int i = 0; i < 8; ++i) FOTO_HIP_CHECK(hipMalloc((void**)&f[i], n * 8));
        for (int i = 0; i < 8; i += 2) k_stream_fill<<<1024, 256, 0, s>>>(f[i], f[i + 1], n);   // non-zero data
        FOTO_HIP_CHECK(hipGetLastError());
        FOTO_HIP_CHECK(hipEventCreate(&e0));
        FOTO_HIP_CHECK(hipEventCreate(&e1));
        const int nb = 4 * cus_count();
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            FOTO_HIP_CHECK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) {
                double** A = (k & 1) ? f + 4 : f;
                double** B = (k & 1) ? f : f + 4;
                k_stream_4x4<<<nb, 256, 0, s>>>(A[0], A[1], A[2], A[3], B[0], B[1], B[2], B[3], n / 2, 1e-9);
            }
            FOTO_HIP_CHECK(hipGetLastError());
            FOTO_HIP_CHECK(hipEventRecord(e1, s));
            FOTO_HIP_CHECK(hipEventSynchronize(e1));
            float t = 0.f;
            FOTO_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
            best = std::min(best, t);
        }
        us[0] = 1e3 * best / reps;
        return 0;
    };
    const int rc = body();
    if (s) (void)hipStreamSynchronize(s);
    for (double* p : f)
        if (p) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (s) (void)hipStreamDestroy(s);
    return rc;
}

extern "C" int foto_stream_probe(int64_t n, int reps, double* us) {
    using namespace foto;
    if (!us || n < 2 || n % 2 || reps < 1 || n * 8 >= (int64_t(1) << 31)) {
        set_error("foto_stream_probe: bad arguments (n even, n * 8 < 2^31)");
        return FOTO_ERR_ARG;
    }
    hipStream_t s = nullptr;
    double *r = nullptr, *q = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    auto body = [&]() -> int {
        FOTO_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        FOTO_HIP_CHECK(hipMalloc((void**)&r, n * 8));
        FOTO_HIP_CHECK(hipMalloc((void**)&q, n * 8));
        // non-zero data: zero-filled buffers let the chip hold a higher clock (MI355X_MICROARCH.md,
        // DVFS give-back) and read 15-20 % faster than the solver's vectors do
        k_stream_fill<<<1024, 256, 0, s>>>(r, q, n);
        FOTO_HIP_CHECK(hipGetLastError());
        FOTO_HIP_CHECK(hipEventCreate(&e0));
        FOTO_HIP_CHECK(hipEventCreate(&e1));
        for (int wt = 0; wt < 2; ++wt) {
            float best = 1e30f;
            for (int rep = 0; rep < 3; ++rep) {
                FOTO_HIP_CHECK(hipEventRecord(e0, s));
                for (int k = 0; k < reps; ++k) {
                    if (wt) k_stream_rq<true><<<1024, 256, 0, s>>>(r, q, n / 2, 1e-9, 1e-9);
                    else k_stream_rq<false><<<1024, 256, 0, s>>>(r, q, n / 2, 1e-9, 1e-9);
                }
                FOTO_HIP_CHECK(hipGetLastError());
                FOTO_HIP_CHECK(hipEventRecord(e1, s));
                FOTO_HIP_CHECK(hipEventSynchronize(e1));
                float t = 0.f;
                FOTO_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
                best = std::min(best, t);
            }
            us[wt] = 1e3 * best / reps;
        }
        return 0;
    };
    const int rc = body();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (r) (void)hipFree(r);
    if (q) (void)hipFree(q);
    if (s) (void)hipStreamDestroy(s);
    return rc;
}
