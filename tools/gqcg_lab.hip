// Node-CG lab: scipy's CG recurrence on the 2048-node Gauss measure (k_gq_cg, foto_gauss.inc)
// against variants that change where a step's time goes.  A synthetic measure (positive
// weights decaying with lam, lam spread like the DCT spectrum of the bench grid), maxiter steps
// (rtol = 0 so every variant runs the same count), each variant launched back to back; alpha
// and beta compared with the product kernel's.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//       -I../optical-flow-optimal-transport_amd/csrc gqcg_lab.hip -o gqcg_lab
#include "../optical-flow-optimal-transport_amd/csrc/foto_spectral.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
namespace foto { void set_error(const char*, ...) {} }
using namespace foto;

// ---- variant: NTH threads, NPT nodes per thread, the "lr / ap" form (5 VALU ops per node per
// step: ap = beta ap + lam r, r -= alpha ap, lr = lam r, rr += r r, rd += lr r); block sum by
// DPP + an LDS slot per wave; BCAST = 1: every lane reads the wave slots (LDS broadcast),
// BCAST = 0: lane 0 reads them and readlane broadcasts
template <int NTH, int BCAST, int NACCV = 4>
__global__ __launch_bounds__(NTH) void k_cg_var(const GqNodes* __restrict__ nd, double rtol, int maxiter,
                                                GqState* __restrict__ S) {
    constexpr int NW = NTH / 64;
    constexpr int NPT = GQ_NODES / NTH;
    constexpr int NACC = NPT >= NACCV ? NACCV : NPT;
    __shared__ __attribute__((aligned(16))) dbl2 red[2][NW > 0 ? NW : 1];
    __shared__ __attribute__((aligned(16))) dbl2 redr[2][4 * (NW > 0 ? NW : 1)];
    __shared__ double abL[2][GQ_KMAX];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double lam[NPT], r[NPT], ap[NPT], lr[NPT];
    double mass = 0.0;
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const int id = threadIdx.x * NPT + j;
        lam[j] = nd->lam[id];
        const double w = nd->w[id];
        r[j] = sqrt(w);
        ap[j] = 0.0;
        lr[j] = lam[j] * r[j];
        mass += w;
    }
    auto reduce2 = [&](double a, double b, int slot, double* ra, double* rb) {
        a += dbl_dpp<0x111>(a);
        b += dbl_dpp<0x111>(b);
        a += dbl_dpp<0x112>(a);
        b += dbl_dpp<0x112>(b);
        a += dbl_dpp<0x114>(a);
        b += dbl_dpp<0x114>(b);
        a += dbl_dpp<0x118>(a);
        b += dbl_dpp<0x118>(b);
        if constexpr (BCAST == 2) {   // row totals (lanes 15, 31, 47, 63) through LDS
            if ((lane & 15) == 15) redr[slot][wv * 4 + (lane >> 4)] = dbl2{a, b};
            __syncthreads();
            dbl2 t = redr[slot][0];
#pragma unroll
            for (int q = 1; q < 4 * NW; ++q) t += redr[slot][q];
            *ra = t[0];
            *rb = t[1];
            return;
        }
        a += dbl_dpp_rows<0x142, 0xa>(a);
        b += dbl_dpp_rows<0x142, 0xa>(b);
        a += dbl_dpp_rows<0x143, 0xc>(a);
        b += dbl_dpp_rows<0x143, 0xc>(b);
        if constexpr (NW == 1) {
            *ra = dbl_readlane(a, 63);
            *rb = dbl_readlane(b, 63);
        } else {
            if (lane == 63) red[slot][wv] = dbl2{a, b};
            __syncthreads();
            if constexpr (BCAST) {
                dbl2 t = red[slot][0];
#pragma unroll
                for (int q = 1; q < NW; ++q) t += red[slot][q];
                *ra = t[0];
                *rb = t[1];
            } else {
                dbl2 v[NW];
                if (lane == 0) {
#pragma unroll
                    for (int q = 0; q < NW; ++q) v[q] = red[slot][q];
                }
                double ta = dbl_readlane(v[0][0], 0), tb = dbl_readlane(v[0][1], 0);
#pragma unroll
                for (int q = 1; q < NW; ++q) {
                    ta += dbl_readlane(v[q][0], 0);
                    tb += dbl_readlane(v[q][1], 0);
                }
                *ra = ta;
                *rb = tb;
            }
        }
    };
    double bn2, unused;
    reduce2(mass, 0.0, 1, &bn2, &unused);
    const double atol = rtol * sqrt(bn2);
    const double atol2 = atol * atol;
    int status = 0, conv = 0, K = maxiter;
    double rho = bn2, irho_prev = 1.0, sigma_prev = 1.0;
    // the first step's sums (r0 = sqrt(w))
    double sa[NACC], sd[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) { sa[q] = 0.0; sd[q] = 0.0; }
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        sa[j % NACC] = fma(r[j], r[j], sa[j % NACC]);
        sd[j % NACC] = fma(lr[j], r[j], sd[j % NACC]);
    }
    for (int k = 0; k < maxiter; ++k) {
#pragma unroll
        for (int h = NACC / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int q = 0; q < h; ++q) { sa[q] += sa[q + h]; sd[q] += sd[q + h]; }
        double delta;
        reduce2(sa[0], sd[0], k & 1, &rho, &delta);
        if (rho < atol2) { K = k; conv = 1; break; }
        if (k >= GQ_KMAX) { K = k; status = 2; break; }
        const double beta = (k == 0) ? 0.0 : rho * irho_prev;
        const double sigma = (k == 0) ? delta : fma(-beta * beta, sigma_prev, delta);
        if (!(sigma > 0.0) || !isfinite(sigma)) { K = k; status = 1; break; }
        double y = __builtin_amdgcn_rcp(sigma);
        y = fma(y, fma(-sigma, y, 1.0), y);
        y = fma(y, fma(-sigma, y, 1.0), y);
        double alpha = rho * y;
        alpha = fma(fma(-sigma, alpha, rho), y, alpha);
        irho_prev = 1.0 / rho;
#pragma unroll
        for (int q = 0; q < NACC; ++q) { sa[q] = 0.0; sd[q] = 0.0; }
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
            ap[j] = fma(beta, ap[j], lr[j]);
            r[j] = fma(-alpha, ap[j], r[j]);
            lr[j] = lam[j] * r[j];
            sa[j % NACC] = fma(r[j], r[j], sa[j % NACC]);
            sd[j % NACC] = fma(lr[j], r[j], sd[j % NACC]);
        }
        if (threadIdx.x == 0) {
            abL[0][k] = alpha;
            abL[1][k] = beta;
        }
        sigma_prev = sigma;
    }
    __syncthreads();
    const int kst = (K < GQ_KMAX) ? K : GQ_KMAX;
    for (int e = threadIdx.x; e < kst; e += NTH) {
        S->alpha[e] = abL[0][e];
        S->beta[e] = abL[1][e];
    }
    if (threadIdx.x == 0) {
        S->K = K;
        S->status = status;
        S->conv = conv;
        S->rn2 = rho;
    }
}

// ---- lower bound: the same loop with no cross-lane reduction at all (each lane's own sums
// stand in for the totals), to price the reduction + barrier part of a step
template <int NTH>
__global__ __launch_bounds__(NTH) void k_cg_noreduce(const GqNodes* __restrict__ nd, int maxiter, GqState* __restrict__ S) {
    constexpr int NPT = GQ_NODES / NTH;
    constexpr int NACC = NPT >= 4 ? 4 : NPT;
    double lam[NPT], r[NPT], ap[NPT], lr[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const int id = threadIdx.x * NPT + j;
        lam[j] = nd->lam[id];
        r[j] = sqrt(nd->w[id]);
        ap[j] = 0.0;
        lr[j] = lam[j] * r[j];
    }
    double sa[NACC], sd[NACC];
    double irho_prev = 1.0, sigma_prev = 1.0;
#pragma unroll
    for (int q = 0; q < NACC; ++q) { sa[q] = 0.0; sd[q] = 0.0; }
#pragma unroll
    for (int j = 0; j < NPT; ++j) { sa[j % NACC] = fma(r[j], r[j], sa[j % NACC]); sd[j % NACC] = fma(lr[j], r[j], sd[j % NACC]); }
    for (int k = 0; k < maxiter; ++k) {
#pragma unroll
        for (int h = NACC / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int q = 0; q < h; ++q) { sa[q] += sa[q + h]; sd[q] += sd[q + h]; }
        const double rho = sa[0] * 2048.0, delta = sd[0] * 2048.0;
        const double beta = (k == 0) ? 0.0 : rho * irho_prev;
        const double sigma = (k == 0) ? delta : fma(-beta * beta, sigma_prev, delta);
        double y = __builtin_amdgcn_rcp(sigma);
        y = fma(y, fma(-sigma, y, 1.0), y);
        y = fma(y, fma(-sigma, y, 1.0), y);
        double alpha = rho * y;
        alpha = fma(fma(-sigma, alpha, rho), y, alpha);
        irho_prev = 1.0 / rho;
#pragma unroll
        for (int q = 0; q < NACC; ++q) { sa[q] = 0.0; sd[q] = 0.0; }
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
            ap[j] = fma(beta, ap[j], lr[j]);
            r[j] = fma(-alpha, ap[j], r[j]);
            lr[j] = lam[j] * r[j];
            sa[j % NACC] = fma(r[j], r[j], sa[j % NACC]);
            sd[j % NACC] = fma(lr[j], r[j], sd[j % NACC]);
        }
        sigma_prev = sigma;
    }
    if (threadIdx.x == 0) S->rn2 = sa[0];
}

// ---- two steps per reduction (round 5).  At the top of a pair the lanes hold r = r_k and
// a = A p_{k-1}; step k's alpha, beta come from rho = r.r and delta = r.Ar as in k_gq_cg, and
// step k + 1's from the same reduction: r_{k+1} = (1 - alpha lam) r - alpha beta a, so
//   rho'   = Srr  - 2 al Slrr  + al^2 Sl2rr - 2 al be (Sra  - al Slra)  + (al be)^2 Saa
//   delta' = Slrr - 2 al Sl2rr + al^2 Sl3rr - 2 al be (Slra - al Sl2ra) + (al be)^2 Slaa
// -- nine sums, one barrier per two steps.  RED 0: each sum by its own DPP tree (as reduce2);
// RED 1: a butterfly reduce-scatter inside each 16-lane row (mirror, half-mirror, quad xor 2,
// quad xor 1: 5 + 3 + 2 + 1 exchanges for the nine sums), then xor 16 / xor 32 by gfx950's
// permlane swaps, the 4 waves' rows through LDS, and readlanes.
constexpr int C2N = 9;
__device__ __forceinline__ double dbl_pl16(double v) {   // v of lane l ^ 16
    const long long b = __double_as_longlong(v);
    const unsigned l = threadIdx.x & 63;
    auto lo = __builtin_amdgcn_permlane16_swap((unsigned)b, (unsigned)b, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    const unsigned rl = (l & 16) ? lo[0] : lo[1], rh = (l & 16) ? hi[0] : hi[1];
    return __longlong_as_double(((long long)rh << 32) | rl);
}
__device__ __forceinline__ double dbl_pl32(double v) {   // v of lane l ^ 32
    const long long b = __double_as_longlong(v);
    const unsigned l = threadIdx.x & 63;
    auto lo = __builtin_amdgcn_permlane32_swap((unsigned)b, (unsigned)b, false, false);
    auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
    const unsigned rl = (l & 32) ? lo[0] : lo[1], rh = (l & 32) ? hi[0] : hi[1];
    return __longlong_as_double(((long long)rh << 32) | rl);
}
template <int CIN, int CTRL>
__device__ __forceinline__ void bfly(double (&v)[C2N], bool bit) {
    constexpr int H = (CIN + 1) / 2;
#pragma unroll
    for (int i = 0; i < H; ++i) {
        const double lo = v[i], hi = (H + i < CIN) ? v[H + i] : 0.0;
        const double send = bit ? lo : hi, keep = bit ? hi : lo;
        v[i] = keep + dbl_dpp<CTRL>(send);
    }
}
// the sum a row lane holds after the four stages (-1: padding), from the same halving
struct BflyMap {
    int lane_of[C2N];
    constexpr BflyMap() : lane_of{} {
        for (int l = 0; l < 16; ++l) {
            const int bits[4] = {(l >> 3) & 1, (l >> 2) & 1, (l >> 1) & 1, l & 1};
            const int cin[4] = {9, 5, 3, 2};
            int base = 0, cnt = 9;
            for (int st = 0; st < 4; ++st) {
                const int H = (cin[st] + 1) / 2;
                if (bits[st]) { base += H; cnt = cnt - H; }
                else cnt = cnt < H ? cnt : H;
            }
            if (cnt >= 1 && base < C2N) lane_of[base] = l;
        }
    }
};
constexpr BflyMap BFLY{};

template <int RED>
__global__ __launch_bounds__(256) void k_cg2(const GqNodes* __restrict__ nd, double rtol, int maxiter, int klim,
                                             GqState* __restrict__ S) {
    constexpr int NTH = 256, NW = 4, NPT = GQ_NODES / NTH;
    __shared__ __attribute__((aligned(16))) double red[2][NW][16];
    __shared__ double abL[2][GQ_KMAX];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double lam[NPT], r[NPT], a[NPT];
    double mass = 0.0;
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const int id = threadIdx.x * NPT + j;
        lam[j] = nd->lam[id];
        const double w = nd->w[id];
        r[j] = sqrt(w);
        a[j] = 0.0;
        mass += w;
    }
    auto sums = [&](double (&s)[C2N]) {
#pragma unroll
        for (int q = 0; q < C2N; ++q) s[q] = 0.0;
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
            const double lr = lam[j] * r[j], la = lam[j] * a[j], lr2 = lr * lr;
            s[0] = fma(r[j], r[j], s[0]);
            s[1] = fma(lr, r[j], s[1]);
            s[2] += lr2;
            s[3] = fma(lam[j], lr2, s[3]);
            s[4] = fma(r[j], a[j], s[4]);
            s[5] = fma(lr, a[j], s[5]);
            s[6] = fma(lr, la, s[6]);
            s[7] = fma(a[j], a[j], s[7]);
            s[8] = fma(la, a[j], s[8]);
        }
    };
    // block totals of v[0 .. C2N), the same bits in every lane
    auto reduce9 = [&](double (&v)[C2N], int slot, double (&t)[C2N]) {
        if constexpr (RED == 0) {
#pragma unroll
            for (int q = 0; q < C2N; ++q) v[q] += dbl_dpp<0x111>(v[q]);
#pragma unroll
            for (int q = 0; q < C2N; ++q) v[q] += dbl_dpp<0x112>(v[q]);
#pragma unroll
            for (int q = 0; q < C2N; ++q) v[q] += dbl_dpp<0x114>(v[q]);
#pragma unroll
            for (int q = 0; q < C2N; ++q) v[q] += dbl_dpp<0x118>(v[q]);
#pragma unroll
            for (int q = 0; q < C2N; ++q) v[q] += dbl_dpp_rows<0x142, 0xa>(v[q]);
#pragma unroll
            for (int q = 0; q < C2N; ++q) v[q] += dbl_dpp_rows<0x143, 0xc>(v[q]);
            if (lane == 63) {
#pragma unroll
                for (int q = 0; q < C2N; ++q) red[slot][wv][q] = v[q];
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < C2N; ++q) {
                double x = red[slot][0][q];
#pragma unroll
                for (int w = 1; w < NW; ++w) x += red[slot][w][q];
                t[q] = x;
            }
        } else {
            const int l = lane & 15;
            bfly<9, 0x140>(v, (l >> 3) & 1);   // row_mirror: l <-> 15 - l
            bfly<5, 0x141>(v, (l >> 2) & 1);   // row_half_mirror: l <-> 7 - l in each half row
            bfly<3, 0x4E>(v, (l >> 1) & 1);    // quad_perm [2, 3, 0, 1]
            bfly<2, 0xB1>(v, l & 1);           // quad_perm [1, 0, 3, 2]
            double x = v[0];
            x += dbl_pl16(x);
            x += dbl_pl32(x);
            if (lane < 16) red[slot][wv][lane] = x;
            __syncthreads();
            double y = red[slot][0][l];
#pragma unroll
            for (int w = 1; w < NW; ++w) y += red[slot][w][l];
#pragma unroll
            for (int q = 0; q < C2N; ++q) t[q] = dbl_readlane(y, BFLY.lane_of[q]);
        }
    };
    double tt[C2N], ss[C2N];
    {
        double m[C2N];
#pragma unroll
        for (int q = 0; q < C2N; ++q) m[q] = 0.0;
        m[0] = mass;
        reduce9(m, 1, tt);
    }
    const double bn2 = tt[0];
    const double atol = rtol * sqrt(bn2);
    const double atol2 = atol * atol;
    int status = 0, conv = 0, K = maxiter;
    double rho = bn2, irho_prev = 1.0, sigma_prev = 1.0;
    auto rdiv = [](double num, double den) {
        double y = __builtin_amdgcn_rcp(den);
        y = fma(y, fma(-den, y, 1.0), y);
        y = fma(y, fma(-den, y, 1.0), y);
        double q = num * y;
        return fma(fma(-den, q, num), y, q);
    };
    sums(ss);
    for (int k = 0; k < maxiter; k += 2) {
        reduce9(ss, (k >> 1) & 1, tt);
        rho = tt[0];
        const double delta = tt[1];
        if (rho < atol2) { K = k; conv = 1; break; }
        if (k >= klim) { K = k; status = 2; break; }
        const double beta = (k == 0) ? 0.0 : rho * irho_prev;
        const double sigma = (k == 0) ? delta : fma(-beta * beta, sigma_prev, delta);
        if (!(sigma > 0.0) || !isfinite(sigma)) { K = k; status = 1; break; }
        const double alpha = rdiv(rho, sigma);
        if (threadIdx.x == 0) { abL[0][k] = alpha; abL[1][k] = beta; }
        const double ab = alpha * beta, ab2 = ab * ab, a2 = alpha * alpha;
        const double rho1 = fma(ab2, tt[7], fma(-2.0 * ab, fma(-alpha, tt[5], tt[4]), fma(a2, tt[2], fma(-2.0 * alpha, tt[1], tt[0]))));
        const double delta1 = fma(ab2, tt[8], fma(-2.0 * ab, fma(-alpha, tt[6], tt[5]), fma(a2, tt[3], fma(-2.0 * alpha, tt[2], tt[1]))));
        // step k + 1 (unless the pair ends after step k)
        int fin = 0;   // 1: K = k + 1 after step k's update
        double beta1 = 0.0, alpha1 = 0.0, sigma1 = 0.0;
        if (k + 1 >= maxiter) { fin = 1; K = k + 1; rho = rho; }
        else if (rho1 < atol2) { fin = 1; K = k + 1; conv = 1; rho = rho1; }
        else if (k + 1 >= klim) { fin = 1; K = k + 1; status = 2; rho = rho1; }
        else {
            beta1 = rho1 * (1.0 / rho);
            sigma1 = fma(-beta1 * beta1, sigma, delta1);
            if (!(sigma1 > 0.0) || !isfinite(sigma1)) { fin = 1; K = k + 1; status = 1; rho = rho1; }
            else alpha1 = rdiv(rho1, sigma1);
        }
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
            a[j] = fma(beta, a[j], lam[j] * r[j]);
            r[j] = fma(-alpha, a[j], r[j]);
        }
        if (fin) break;
        if (threadIdx.x == 0) { abL[0][k + 1] = alpha1; abL[1][k + 1] = beta1; }
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
            a[j] = fma(beta1, a[j], lam[j] * r[j]);
            r[j] = fma(-alpha1, a[j], r[j]);
        }
        rho = rho1;
        irho_prev = 1.0 / rho1;
        sigma_prev = sigma1;
        sums(ss);
    }
    __syncthreads();
    const int kst = (K < GQ_KMAX) ? K : GQ_KMAX;
    for (int e = threadIdx.x; e < kst; e += NTH) {
        S->alpha[e] = abL[0][e];
        S->beta[e] = abL[1][e];
    }
    if (threadIdx.x == 0) {
        S->K = K;
        S->status = status;
        S->conv = conv;
        S->bn2 = bn2;
        S->rn2 = rho;
    }
}

// ---- round 6: where the reduction's time goes, and a shorter one.  RED 0: the product's two
// interleaved DPP trees (row_shr 1/2/4/8, row_bcast 15/31); RED 1: a reduce-scatter by one
// v_permlane32_swap pair (lanes 0-31 end with a_l + a_l+32, lanes 32-63 with b_l-32 + b_l), then
// two f64 MFMAs against 0/1 matrices (the first sums the four k-slices of each column, a in
// columns 0-7 and b in 8-15 by the mask B; the second sums its lane-group totals), both totals
// in every lane; RED 2: none (a lane's own sums x 64, timing only).  XW 0: the wave totals
// through LDS + barrier (product); XW 1: none (a wave's total x 4, timing only).  IRHO 1:
// 1 / rho by rcp + two Newton steps instead of the IEEE division sequence.
template <int RED, int XW, int IRHO>
__global__ __launch_bounds__(256) void k_cg_r6(const GqNodes* __restrict__ nd, double rtol, int maxiter,
                                               GqState* __restrict__ S) {
    constexpr int NTH = 256, NW = 4, NPT = GQ_NODES / NTH, NACC = 2;
    __shared__ __attribute__((aligned(16))) dbl2 red[2][NW];
    __shared__ double abL[2][GQ_KMAX];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const double bmask = (((lane >> 4) < 2) == ((lane & 15) < 8)) ? 1.0 : 0.0;
    double lam[NPT], r[NPT], ap[NPT], lr[NPT];
    double mass = 0.0;
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        const int id = threadIdx.x * NPT + j;
        lam[j] = nd->lam[id];
        const double w = nd->w[id];
        r[j] = sqrt(w);
        ap[j] = 0.0;
        lr[j] = lam[j] * r[j];
        mass += w;
    }
    auto wave2 = [&](double a, double b, double* wa, double* wb) {
        if constexpr (RED == 0) {
            a += dbl_dpp<0x111>(a);
            b += dbl_dpp<0x111>(b);
            a += dbl_dpp<0x112>(a);
            b += dbl_dpp<0x112>(b);
            a += dbl_dpp<0x114>(a);
            b += dbl_dpp<0x114>(b);
            a += dbl_dpp<0x118>(a);
            b += dbl_dpp<0x118>(b);
            a += dbl_dpp_rows<0x142, 0xa>(a);
            b += dbl_dpp_rows<0x142, 0xa>(b);
            a += dbl_dpp_rows<0x143, 0xc>(a);
            b += dbl_dpp_rows<0x143, 0xc>(b);
            *wa = dbl_readlane(a, 63);
            *wb = dbl_readlane(b, 63);
        } else if constexpr (RED == 1) {
            const long long ba = __double_as_longlong(a), bb = __double_as_longlong(b);
            auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ba, (unsigned)bb, false, false);
            auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ba >> 32), (unsigned)(bb >> 32), false, false);
            const double x0 = __longlong_as_double(((long long)hi[0] << 32) | lo[0]);
            const double x1 = __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
            const double s = x0 + x1;
            const dbl4 d1 = __builtin_amdgcn_mfma_f64_16x16x4f64(s, bmask, dbl4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
            const double u = (d1[0] + d1[1]) + (d1[2] + d1[3]);
            const dbl4 d2 = __builtin_amdgcn_mfma_f64_16x16x4f64(u, 1.0, dbl4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0);
            *wa = d2[0];
            *wb = d2[2];
        } else if constexpr (RED == 3) {
            // reduce-scatter by one permlane32 swap pair (a-partials in lanes 0-31, b-partials in
            // 32-63), xor 16 by permlane16 swaps, then an all-reduce inside each 16-lane row by
            // DPP rotations (8, 4, 2, 1): every lane of the low half ends with the a total, of the
            // high half with the b total -- one double per level after the first
            const long long ba = __double_as_longlong(a), bb = __double_as_longlong(b);
            auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ba, (unsigned)bb, false, false);
            auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ba >> 32), (unsigned)(bb >> 32), false, false);
            double t = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) +
                       __longlong_as_double(((long long)hi[1] << 32) | lo[1]);
            t += dbl_pl16(t);
            t += dbl_dpp<0x128>(t);   // row_ror:8
            t += dbl_dpp<0x124>(t);   // row_ror:4
            t += dbl_dpp<0x122>(t);   // row_ror:2
            t += dbl_dpp<0x121>(t);   // row_ror:1
            *wa = dbl_readlane(t, 0);
            *wb = dbl_readlane(t, 32);
        } else {
            *wa = 64.0 * a;
            *wb = 64.0 * b;
        }
    };
    auto reduce2 = [&](double a, double b, int slot, double* ra, double* rb) {
        double wa, wb;
        wave2(a, b, &wa, &wb);
        if constexpr (XW == 0) {
            if (lane == 63) red[slot][wv] = dbl2{wa, wb};
            __syncthreads();
            dbl2 t = red[slot][0];
#pragma unroll
            for (int q = 1; q < NW; ++q) t += red[slot][q];
            *ra = t[0];
            *rb = t[1];
        } else {
            *ra = 4.0 * wa;
            *rb = 4.0 * wb;
        }
    };
    double bn2, unused;
    reduce2(mass, 0.0, 1, &bn2, &unused);
    const double atol = rtol * sqrt(bn2);
    const double atol2 = atol * atol;
    int status = 0, conv = 0, K = maxiter;
    double rho = bn2, irho_prev = 1.0, sigma_prev = 1.0;
    double sa[NACC], sd[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) { sa[q] = 0.0; sd[q] = 0.0; }
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
        sa[j % NACC] = fma(r[j], r[j], sa[j % NACC]);
        sd[j % NACC] = fma(lr[j], r[j], sd[j % NACC]);
    }
    for (int k = 0; k < maxiter; ++k) {
        sa[0] += sa[1];
        sd[0] += sd[1];
        double delta;
        reduce2(sa[0], sd[0], k & 1, &rho, &delta);
        if (rho < atol2) { K = k; conv = 1; break; }
        if (k >= GQ_KMAX) { K = k; status = 2; break; }
        const double beta = (k == 0) ? 0.0 : rho * irho_prev;
        const double sigma = (k == 0) ? delta : fma(-beta * beta, sigma_prev, delta);
        if (!(sigma > 0.0) || !isfinite(sigma)) { K = k; status = 1; break; }
        double y = __builtin_amdgcn_rcp(sigma);
        y = fma(y, fma(-sigma, y, 1.0), y);
        y = fma(y, fma(-sigma, y, 1.0), y);
        double alpha = rho * y;
        alpha = fma(fma(-sigma, alpha, rho), y, alpha);
        if constexpr (IRHO) {
            double z = __builtin_amdgcn_rcp(rho);
            z = fma(z, fma(-rho, z, 1.0), z);
            irho_prev = fma(z, fma(-rho, z, 1.0), z);
        } else {
            irho_prev = 1.0 / rho;
        }
#pragma unroll
        for (int q = 0; q < NACC; ++q) { sa[q] = 0.0; sd[q] = 0.0; }
#pragma unroll
        for (int j = 0; j < NPT; ++j) {
            ap[j] = fma(beta, ap[j], lr[j]);
            r[j] = fma(-alpha, ap[j], r[j]);
            lr[j] = lam[j] * r[j];
            sa[j % NACC] = fma(r[j], r[j], sa[j % NACC]);
            sd[j % NACC] = fma(lr[j], r[j], sd[j % NACC]);
        }
        if (threadIdx.x == 0) {
            abL[0][k] = alpha;
            abL[1][k] = beta;
        }
        sigma_prev = sigma;
    }
    __syncthreads();
    const int kst = (K < GQ_KMAX) ? K : GQ_KMAX;
    for (int e = threadIdx.x; e < kst; e += NTH) {
        S->alpha[e] = abL[0][e];
        S->beta[e] = abL[1][e];
    }
    if (threadIdx.x == 0) {
        S->K = K;
        S->status = status;
        S->conv = conv;
        S->bn2 = bn2;
        S->rn2 = rho;
    }
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int maxiter = argc > 1 ? atoi(argv[1]) : 180;
    const int reps = argc > 2 ? atoi(argv[2]) : 50;
    // synthetic measure: the bench grid's spectrum spans [r eps, ~12 r]; weights decay with lam
    std::vector<double> lam(GQ_NODES), w(GQ_NODES);
    srand(7);
    for (int i = 0; i < GQ_NODES; ++i) {
        const double t = (i + 0.5) / GQ_NODES;
        lam[i] = 1e-2 + 12.0 * t * t * (1.0 + 0.01 * (rand() / (double)RAND_MAX));
        w[i] = exp(-3.0 * lam[i]) * (0.5 + rand() / (double)RAND_MAX) + 1e-12;
    }
    GqNodes* nd;
    GqState *S0, *S1;
    CK(hipMalloc(&nd, sizeof(GqNodes)));
    CK(hipMalloc(&S0, sizeof(GqState)));
    CK(hipMalloc(&S1, sizeof(GqState)));
    CK(hipMemcpy(nd->lam, lam.data(), sizeof(double) * GQ_NODES, hipMemcpyHostToDevice));
    CK(hipMemcpy(nd->w, w.data(), sizeof(double) * GQ_NODES, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    GqState h0, h1;
    auto timeit = [&](const char* name, auto launch, bool cmp) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; ++i) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        double err = 0;
        int K = -1, st = -1;
        if (cmp) {
            CK(hipMemcpy(&h1, S1, sizeof(GqState), hipMemcpyDeviceToHost));
            K = h1.K;
            st = h1.status;
            for (int k = 0; k < std::min(h0.K, h1.K) && k < GQ_KMAX; ++k) {
                err = std::max(err, fabs(h1.alpha[k] - h0.alpha[k]) / fabs(h0.alpha[k]));
                if (k) err = std::max(err, fabs(h1.beta[k] - h0.beta[k]) / fabs(h0.beta[k]));
            }
        }
        printf("%-28s %8.2f us/solve  %6.3f us/step  K %d status %d  max rel d(alpha,beta) %.2e\n", name,
               1e3 * ms / reps, 1e3 * ms / reps / maxiter, K, st, err);
    };
    timeit("product k_gq_cg (256)", [&] { k_gq_cg<<<1, GQ_CGNTH>>>(nd, 0.0, maxiter, GQ_KMAX, S0, nullptr); }, false);
    CK(hipMemcpy(&h0, S0, sizeof(GqState), hipMemcpyDeviceToHost));
    printf("  product: K %d status %d rn2/bn2 %.3e\n", h0.K, h0.status, h0.rn2 / h0.bn2);
    if (argc > 3 && atoi(argv[3]) == 6) {   // round 6 rows only
        timeit("r6 dpp+lds (product form)", [&] { k_cg_r6<0, 0, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
        timeit("r6 dpp+lds fast 1/rho", [&] { k_cg_r6<0, 0, 1><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
        timeit("r6 mfma+lds", [&] { k_cg_r6<1, 0, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
        timeit("r6 mfma+lds fast 1/rho", [&] { k_cg_r6<1, 0, 1><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
        timeit("r6 rotate+lds", [&] { k_cg_r6<3, 0, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
        timeit("r6 rotate only (no lds)", [&] { k_cg_r6<3, 1, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, false);
        timeit("r6 dpp only (no lds)", [&] { k_cg_r6<0, 1, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, false);
        timeit("r6 mfma only (no lds)", [&] { k_cg_r6<1, 1, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, false);
        timeit("r6 lds only (no wave red)", [&] { k_cg_r6<2, 0, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, false);
        timeit("r6 neither", [&] { k_cg_r6<2, 1, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, false);
        const double rtols[3] = {1e-3, 1e-5, 1e-7};
        for (double rt : rtols) {
            k_gq_cg<<<1, GQ_CGNTH>>>(nd, rt, 100000, GQ_KMAX, S0, nullptr);
            k_cg_r6<1, 0, 1><<<1, 256>>>(nd, rt, 100000, S1);
            CK(hipMemcpy(&h0, S0, sizeof(GqState), hipMemcpyDeviceToHost));
            CK(hipMemcpy(&h1, S1, sizeof(GqState), hipMemcpyDeviceToHost));
            double err = 0;
            for (int k = 0; k < std::min(h0.K, h1.K) && k < GQ_KMAX; ++k) {
                err = std::max(err, fabs(h1.alpha[k] - h0.alpha[k]) / fabs(h0.alpha[k]));
                if (k) err = std::max(err, fabs(h1.beta[k] - h0.beta[k]) / fabs(h0.beta[k]));
            }
            printf("  rtol %.0e: product K %d rn2 %.9e | mfma+fast K %d conv %d rn2 %.9e | d(alpha,beta) %.2e\n", rt, h0.K,
                   h0.rn2, h1.K, h1.conv, h1.rn2, err);
        }
        return 0;
    }
    timeit("lr/ap 64 (one wave)", [&] { k_cg_var<64, 0><<<1, 64>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 128 readlane", [&] { k_cg_var<128, 0><<<1, 128>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 128 bcast", [&] { k_cg_var<128, 1><<<1, 128>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 256 readlane", [&] { k_cg_var<256, 0><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 256 bcast", [&] { k_cg_var<256, 1><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 256 rows-LDS", [&] { k_cg_var<256, 2><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 128 rows-LDS", [&] { k_cg_var<128, 2><<<1, 128>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 256 bcast nacc2", [&] { k_cg_var<256, 1, 2><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 256 bcast nacc8", [&] { k_cg_var<256, 1, 8><<<1, 256>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 512 rows-LDS", [&] { k_cg_var<512, 2><<<1, 512>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("lr/ap 512 bcast", [&] { k_cg_var<512, 1><<<1, 512>>>(nd, 0.0, maxiter, S1); }, true);
    timeit("2-step naive DPP", [&] { k_cg2<0><<<1, 256>>>(nd, 0.0, maxiter, GQ_KMAX, S1); }, true);
    timeit("2-step butterfly", [&] { k_cg2<1><<<1, 256>>>(nd, 0.0, maxiter, GQ_KMAX, S1); }, true);
    {   // with a stop test: the iteration count against the product's
        const double rtols[3] = {1e-3, 1e-5, 1e-7};
        for (double rt : rtols) {
            k_gq_cg<<<1, GQ_CGNTH>>>(nd, rt, 100000, GQ_KMAX, S0, nullptr);
            k_cg2<1><<<1, 256>>>(nd, rt, 100000, GQ_KMAX, S1);
            CK(hipMemcpy(&h0, S0, sizeof(GqState), hipMemcpyDeviceToHost));
            CK(hipMemcpy(&h1, S1, sizeof(GqState), hipMemcpyDeviceToHost));
            double err = 0;
            for (int k = 0; k < std::min(h0.K, h1.K) && k < GQ_KMAX; ++k) {
                err = std::max(err, fabs(h1.alpha[k] - h0.alpha[k]) / fabs(h0.alpha[k]));
                if (k) err = std::max(err, fabs(h1.beta[k] - h0.beta[k]) / fabs(h0.beta[k]));
            }
            printf("  rtol %.0e: product K %d conv %d status %d rn2 %.6e | 2-step K %d conv %d status %d rn2 %.6e | d(alpha,beta) %.2e\n",
                   rt, h0.K, h0.conv, h0.status, h0.rn2, h1.K, h1.conv, h1.status, h1.rn2, err);
        }
    }
    timeit("no reduction 64", [&] { k_cg_noreduce<64><<<1, 64>>>(nd, maxiter, S1); }, false);
    timeit("no reduction 128", [&] { k_cg_noreduce<128><<<1, 128>>>(nd, maxiter, S1); }, false);
    timeit("no reduction 512", [&] { k_cg_noreduce<512><<<1, 512>>>(nd, maxiter, S1); }, false);
    timeit("no reduction 256", [&] { k_cg_noreduce<256><<<1, 256>>>(nd, maxiter, S1); }, false);
    timeit("empty launch", [&] { k_cg_noreduce<64><<<1, 64>>>(nd, 0, S1); }, false);
    return 0;
}
