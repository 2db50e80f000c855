// Modified-Chebyshev lab (round 6): the per-step latency of Gautschi's modified Chebyshev algorithm
// on ONE wave -- the candidate replacement of the node CG's block reduction per step (DESIGN.md 6,
// tools/modmom_proto.py for the numerics).  tau_k[m] = sigma_{k, k+m} lives E entries per lane
// (lane j: m = jE .. jE+E-1); a step needs lane j+1's first two entries of tau_{k-1} and
// tau_{k-2} (wave_shl DPP), the auxiliary coefficients of l = k + m (LDS), and lane 0's tau_k[0],
// tau_k[1] (readlane) for a_k, b_k; CG's alpha, beta and rho follow from them in every lane.
// Checked against a host double-precision run of the same recurrence.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off mc_lab.hip -o mc_lab
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

template <int CTRL>
__device__ __forceinline__ double dpp64(double v) {   // (lanes without a source read 0)
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffLL), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double rl64(double v, int lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// lane j gets lane j + 1's value (lane 63 gets 0): wave_shl:1
__device__ __forceinline__ double from_next(double v) { return dpp64<0x130>(v); }

__device__ __forceinline__ double rcp2(double d) {
    double y = __builtin_amdgcn_rcp(d);
    y = fma(y, fma(-d, y, 1.0), y);
    return fma(y, fma(-d, y, 1.0), y);
}

// one wave: n steps from L = 2n moments; out: a[n], b[n], alpha[n], beta[n], K
template <int E>
__global__ __launch_bounds__(64) void k_mc(const double* __restrict__ nu, const double* __restrict__ ahat,
                                           const double* __restrict__ bhat, int n, double atol2, double* out,
                                           int* Kout) {
    __shared__ double A[64 * E + 520], B[64 * E + 520];   // l = k + m < n + 64E
    const int lane = threadIdx.x;
    for (int e = lane; e < 64 * E + 520; e += 64) {
        A[e] = ahat[e];
        B[e] = bhat[e];
    }
    __syncthreads();
    double cur[E], prv[E];   // tau_{k-1}, tau_{k-2}
#pragma unroll
    for (int i = 0; i < E; ++i) {
        cur[i] = nu[lane * E + i];   // tau_0[m] = sigma_{0, m} = nu_m
        prv[i] = 0.0;
    }
    const double nu0 = rl64(cur[0], 0), nu1 = rl64(cur[1], 0);
    double ak = A[0] + nu1 / nu0, bk = nu0;   // a_0, b_0
    double ratio_prev = nu1 / nu0;             // tau_0[1] / tau_0[0]
    double inv_prev = 1.0 / nu0;               // 1 / tau_0[0]
    // CG: alpha_0 = 1 / a_0, rho_0 = b_0
    double alpha = 1.0 / ak, beta = 0.0, rho = bk;
    int K = n;
    if (lane == 0) { out[0] = ak; out[n] = bk; out[2 * n] = alpha; out[3 * n] = 0.0; }
    for (int k = 1; k < n; ++k) {
        // neighbours: tau_{k-1}[m + 1], [m + 2] and tau_{k-2}[m + 2] for the lane's last entries
        const double c0n = from_next(cur[0]), c1n = from_next(cur[1]);
        const double p0n = from_next(prv[0]), p1n = from_next(prv[1]);
        double nw[E];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const int l = k + lane * E + i;
            const double c_m = cur[i];
            const double c_m1 = (i + 1 < E) ? cur[i + 1] : c0n;
            const double c_m2 = (i + 2 < E) ? cur[i + 2] : ((i + 2 == E) ? c0n : c1n);
            const double p_m2 = (i + 2 < E) ? prv[i + 2] : ((i + 2 == E) ? p0n : p1n);
            nw[i] = c_m2 - (ak - A[l]) * c_m1 - bk * p_m2 + B[l] * c_m;
        }
        const double t0 = rl64(nw[0], 0), t1 = rl64(nw[1], 0);
        const double inv = rcp2(t0);
        const double ratio = t1 * inv;
        const double a_new = A[k] + ratio - ratio_prev;
        const double b_new = t0 * inv_prev;
        // CG from the Jacobi matrix: beta_k = b_k alpha_{k-1}^2, alpha_k = 1 / (a_k - beta_k / alpha_{k-1})
        const double be = b_new * alpha * alpha;
        rho = rho * be;
        if (rho < atol2) { K = k; break; }
        const double al = rcp2(a_new - be * rcp2(alpha));
        if (lane == 0) { out[k] = a_new; out[n + k] = b_new; out[2 * n + k] = al; out[3 * n + k] = be; }
        alpha = al;
        beta = be;
        ak = a_new;
        bk = b_new;
        ratio_prev = ratio;
        inv_prev = inv;
#pragma unroll
        for (int i = 0; i < E; ++i) { prv[i] = cur[i]; cur[i] = nw[i]; }
    }
    if (lane == 0) *Kout = K;
    (void)beta;
}


// variant 2: the sigma recurrence alone in the loop (a_k, b_k to LDS), the auxiliary coefficients
// as shift registers (one new LDS read per step, issued a step ahead), CG's alpha, beta, rho and
// the stop index in a serial pass afterwards
template <int E>
__global__ __launch_bounds__(64) void k_mc2(const double* __restrict__ nu, const double* __restrict__ ahat,
                                            const double* __restrict__ bhat, int n, double atol2, double* out,
                                            int* Kout) {
    __shared__ double A[64 * E + 520], B[64 * E + 520];
    __shared__ double ja[520], jb[520];
    const int lane = threadIdx.x;
    for (int e = lane; e < 64 * E + 520; e += 64) {
        A[e] = ahat[e];
        B[e] = bhat[e];
    }
    __syncthreads();
    double cur[E], prv[E], ra[E], rb[E];
#pragma unroll
    for (int i = 0; i < E; ++i) {
        cur[i] = nu[lane * E + i];
        prv[i] = 0.0;
        ra[i] = A[1 + lane * E + i];   // step 1's l = 1 + m
        rb[i] = B[1 + lane * E + i];
    }
    const double nu0 = rl64(cur[0], 0), nu1 = rl64(cur[1], 0);
    double ak = A[0] + nu1 / nu0, bk = nu0;
    double ratio_prev = nu1 / nu0, inv_prev = 1.0 / nu0;
    if (lane == 0) { ja[0] = ak; jb[0] = bk; }
    double na = A[2 + lane * E + E - 1], nb = B[2 + lane * E + E - 1];   // step 2's last entry
    double Ak = A[1];
    for (int k = 1; k < n; ++k) {
        const double c0n = from_next(cur[0]), c1n = from_next(cur[1]);
        const double p0n = from_next(prv[0]), p1n = from_next(prv[1]);
        double nw[E];
#pragma unroll
        for (int i = 0; i < E; ++i) {
            const double c_m = cur[i];
            const double c_m1 = (i + 1 < E) ? cur[i + 1] : c0n;
            const double c_m2 = (i + 2 < E) ? cur[i + 2] : ((i + 2 == E) ? c0n : c1n);
            const double p_m2 = (i + 2 < E) ? prv[i + 2] : ((i + 2 == E) ? p0n : p1n);
            nw[i] = fma(rb[i], c_m, fma(-bk, p_m2, fma(ra[i] - ak, c_m1, c_m2)));
        }
        const double t0 = rl64(nw[0], 0), t1 = rl64(nw[1], 0);
        const double inv = rcp2(t0);
        const double ratio = t1 * inv;
        const double a_new = Ak + ratio - ratio_prev;
        const double b_new = t0 * inv_prev;
        if (lane == 0) { ja[k] = a_new; jb[k] = b_new; }
        // shift the auxiliary registers: step k + 1's entry i is step k's entry i + 1
#pragma unroll
        for (int i = 0; i + 1 < E; ++i) { ra[i] = ra[i + 1]; rb[i] = rb[i + 1]; }
        ra[E - 1] = na;
        rb[E - 1] = nb;
        Ak = ra[0] ;   // A[k + 1] lives in lane 0's entry 0 (l = k + 1 + 0)
        Ak = rl64(Ak, 0);
        na = A[k + 2 + lane * E + E - 1];
        nb = B[k + 2 + lane * E + E - 1];
        ak = a_new;
        bk = b_new;
        ratio_prev = ratio;
        inv_prev = inv;
#pragma unroll
        for (int i = 0; i < E; ++i) { prv[i] = cur[i]; cur[i] = nw[i]; }
    }
    __syncthreads();
    if (lane == 0) {
        double alpha = 1.0 / ja[0], rho = jb[0];
        int K = n;
        out[0] = ja[0]; out[n] = jb[0]; out[2 * n] = alpha; out[3 * n] = 0.0;
        for (int k = 1; k < n; ++k) {
            const double be = jb[k] * alpha * alpha;
            rho *= be;
            if (rho < atol2) { K = k; break; }
            const double al = 1.0 / (ja[k] - be / alpha);
            out[k] = ja[k]; out[n + k] = jb[k]; out[2 * n + k] = al; out[3 * n + k] = be;
            alpha = al;
        }
        *Kout = K;
    }
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 200;
    const int reps = argc > 2 ? atoi(argv[2]) : 50;
    const int var = argc > 3 ? atoi(argv[3]) : 1;
    constexpr int E = 8;   // L = 2n <= 512
    const int L = 64 * E + 520;
    // synthetic measure: nodes spread like the bench grid's spectrum, weights decaying with lam
    const int NN = 2048;
    std::vector<double> lam(NN), w(NN);
    srand(7);
    for (int i = 0; i < NN; ++i) {
        const double t = (i + 0.5) / NN;
        lam[i] = 1e-2 + 12.0 * t * t * (1.0 + 0.01 * (rand() / (double)RAND_MAX));
        w[i] = exp(-3.0 * lam[i]) * (0.5 + rand() / (double)RAND_MAX) + 1e-12;
    }
    // auxiliary family: the monic orthogonal polynomials of a perturbed measure (Stieltjes, long
    // double), continued by Chebyshev asymptotics past 2n (as the GPU path would)
    std::vector<double> ah(L, 6.005), bh(L, 36.0 / 4.0);
    {
        std::vector<long double> pm(NN, 0.0L), p(NN, 1.0L), wp(NN);
        for (int i = 0; i < NN; ++i) wp[i] = w[i] * (1.0L + 0.05L * sinl(3.0L * lam[i]));
        long double nrm_prev = 1;
        for (int k = 0; k < 2 * n + 4 && k < L; ++k) {
            long double nrm = 0, num = 0;
            for (int i = 0; i < NN; ++i) { nrm += wp[i] * p[i] * p[i]; num += wp[i] * lam[i] * p[i] * p[i]; }
            ah[k] = (double)(num / nrm);
            bh[k] = (double)(k == 0 ? nrm : nrm / nrm_prev);
            for (int i = 0; i < NN; ++i) {
                const long double pn = (lam[i] - ah[k]) * p[i] - (k > 0 ? bh[k] * pm[i] : 0.0L);
                pm[i] = p[i];
                p[i] = pn;
            }
            nrm_prev = nrm;
        }
    }
    // modified moments (host, double)
    std::vector<double> nu(64 * E, 0.0);
    {
        std::vector<double> pm(NN, 0.0), p(NN, 1.0);
        for (int l = 0; l < 2 * n && l < 64 * E; ++l) {
            double s = 0;
            for (int i = 0; i < NN; ++i) s += w[i] * p[i];
            nu[l] = s;
            for (int i = 0; i < NN; ++i) {
                const double pn = (lam[i] - ah[l]) * p[i] - (l > 0 ? bh[l] * pm[i] : 0.0);
                pm[i] = p[i];
                p[i] = pn;
            }
        }
    }
    double mass = 0;
    for (double v : w) mass += v;
    const double atol2 = 1e-12 * mass;
    double *dnu, *da, *db, *dout;
    int* dK;
    CK(hipMalloc(&dnu, sizeof(double) * nu.size()));
    CK(hipMalloc(&da, sizeof(double) * L));
    CK(hipMalloc(&db, sizeof(double) * L));
    CK(hipMalloc(&dout, sizeof(double) * 4 * n));
    CK(hipMalloc(&dK, sizeof(int)));
    CK(hipMemcpy(dnu, nu.data(), sizeof(double) * nu.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(da, ah.data(), sizeof(double) * L, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bh.data(), sizeof(double) * L, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto launch = [&]() {
        if (var == 2) k_mc2<E><<<1, 64>>>(dnu, da, db, n, atol2, dout, dK);
        else k_mc<E><<<1, 64>>>(dnu, da, db, n, atol2, dout, dK);
    };
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<double> out(4 * n);
    int K = 0;
    CK(hipMemcpy(out.data(), dout, sizeof(double) * 4 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&K, dK, sizeof(int), hipMemcpyDeviceToHost));
    // reference: scipy's CG recurrence on the nodes (long double)
    std::vector<long double> r(NN), pp(NN, 0.0L);
    for (int i = 0; i < NN; ++i) r[i] = sqrtl((long double)w[i]);
    long double rho = 0;
    for (int i = 0; i < NN; ++i) rho += r[i] * r[i];
    long double rho_prev = 1;
    int Kr = n;
    double err = 0;
    for (int k = 0; k < n; ++k) {
        long double rr = 0;
        for (int i = 0; i < NN; ++i) rr += r[i] * r[i];
        if (rr < atol2) { Kr = k; break; }
        const long double be = (k == 0) ? 0.0L : rr / rho_prev;
        long double pap = 0;
        for (int i = 0; i < NN; ++i) { pp[i] = r[i] + be * pp[i]; pap += pp[i] * lam[i] * pp[i]; }
        const long double al = rr / pap;
        for (int i = 0; i < NN; ++i) r[i] -= al * lam[i] * pp[i];
        rho_prev = rr;
        if (k < K) err = fmax(err, fabs((double)((out[2 * n + k] - al) / al)));
    }
    printf("modified Chebyshev v%d, one wave, E = %d: %.2f us per run of n = %d (%.3f us/step); K %d (reference %d); "
           "max rel d(alpha) %.2e\n", var, E, 1e3 * ms / reps, n, 1e3 * ms / reps / n, K, Kr, err);
    return 0;
}
