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
    timeit("no reduction 64", [&] { k_cg_noreduce<64><<<1, 64>>>(nd, maxiter, S1); }, false);
    timeit("no reduction 128", [&] { k_cg_noreduce<128><<<1, 128>>>(nd, maxiter, S1); }, false);
    timeit("no reduction 512", [&] { k_cg_noreduce<512><<<1, 512>>>(nd, maxiter, S1); }, false);
    timeit("no reduction 256", [&] { k_cg_noreduce<256><<<1, 256>>>(nd, maxiter, S1); }, false);
    timeit("empty launch", [&] { k_cg_noreduce<64><<<1, 64>>>(nd, 0, S1); }, false);
    return 0;
}
