// Node-kernel lab: k_gq_nodes (foto_gauss.inc: per bin, the 8-point Gauss rule of its 16
// Chebyshev moments) on a synthetic measure shaped like the bench grid's (every bin populated by
// random points, weights decaying with lam over many orders of magnitude), timed back to back,
// plus an instrumented copy of its root finder that records per thread how many Sturm
// bisections and Newton steps it took and whether it fell back to bisection to rounding -- the
// wave takes the slowest lane's count.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//       -I../optical-flow-optimal-transport_amd/csrc gqnodes_lab.hip -o gqnodes_lab
#include "../optical-flow-optimal-transport_amd/csrc/foto_spectral.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>
namespace foto { void set_error(const char*, ...) {} }
using namespace foto;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// the root finder of k_gq_nodes with counters: out[id] = bisections | newton << 10 | fallback << 20
__global__ __launch_bounds__(64) void k_nodes_count(const double* __restrict__ hist, const GqExact* __restrict__ X,
                                                    int* __restrict__ out, long long* __restrict__ clk) {
    const int id = blockIdx.x * 64 + threadIdx.x;
    if (id >= GQ_NODES) return;
    const long long c0 = __builtin_amdgcn_s_memtime();
    const int bin = id / GQ_M, k = id - bin * GQ_M;
    double mu[GQ_NM];
#pragma unroll
    for (int j = 0; j < GQ_NM; ++j) mu[j] = hist[j * GQ_NB + bin];
    if (X->n[bin] <= GQ_XS) { out[id] = -1; return; }
    double al[GQ_M], be[GQ_M];
    double msum = 0.0;
#pragma unroll
    for (int j = 0; j < GQ_NM; ++j) msum += mu[j];
    const long long c1 = __builtin_amdgcn_s_memtime() + (msum == 12345.678 ? 1 : 0);
    const int n = gq_mcheb(mu, al, be);
    const long long c2 = __builtin_amdgcn_s_memtime() + (al[GQ_M - 1] == 12345.678 ? 1 : 0);
    long long c3 = c2, c4 = c2;
    int nb = 0, nn = 0, fb = 0;
    if (k < n) {
        double sb[GQ_M];
#pragma unroll
        for (int i = 0; i < GQ_M; ++i) sb[i] = (i < n) ? sqrt(be[i]) : 0.0;
        double lo = 1e300, hi = -1e300;
#pragma unroll
        for (int i = 0; i < GQ_M; ++i) {
            if (i < n) {
                const double r = ((i > 0) ? sb[i] : 0.0) + ((i + 1 < n) ? sb[i + 1] : 0.0);
                lo = fmin(lo, al[i] - r);
                hi = fmax(hi, al[i] + r);
            }
        }
        int clo = 0, chi = n;
        auto bisect = [&](int itmin, int itmax) {
            for (int it = 0; it < itmax; ++it) {
                if (it >= itmin && chi - clo == 1) break;
                const double mid = 0.5 * (lo + hi);
                if (mid <= lo || mid >= hi) break;
                ++nb;
                const int c = gq_sturm(al, be, n, mid);
                if (c > k) { hi = mid; chi = c; }
                else { lo = mid; clo = c; }
            }
        };
        bisect(24, 96);
        c3 = __builtin_amdgcn_s_memtime() + (lo == 12345.678 ? 1 : 0);
        double u = 0.5 * (lo + hi);
        bool ok = true;
        for (int it = 0; it < 6; ++it) {
            double pm = 1.0, p = al[0] - u, dm = 0.0, d = -1.0;
#pragma unroll
            for (int i = 1; i < GQ_M; ++i) {
                if (i < n) {
                    const double pn = (al[i] - u) * p - be[i] * pm;
                    const double dn = (al[i] - u) * d - p - be[i] * dm;
                    pm = p; p = pn; dm = d; d = dn;
                }
            }
            ++nn;
            if (d == 0.0 || p == 0.0) break;
            const double un = u - p / d;
            if (!(un > lo && un < hi)) { ok = false; break; }
            if (un == u) break;
            u = un;
        }
        if (!ok) { fb = 1; bisect(200, 200); }
        c4 = __builtin_amdgcn_s_memtime() + (u == 12345.678 ? 1 : 0);
    }
    out[id] = nb | (nn << 10) | (fb << 20);
    if (id == 0) { clk[0] = c1 - c0; clk[1] = c2 - c1; clk[2] = c3 - c2; clk[3] = c4 - c3; }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    const double decay = argc > 2 ? atof(argv[2]) : 3.0;   // weights exp(-decay * lam)
    // bins on the host (k_gq_bins's edges), points per bin with s inside it
    std::vector<double> hi(GQ_NB + 1);
    for (int b = 0; b <= GQ_NB; ++b) {
        const double c = cos(M_PI * b / (2.0 * GQ_NB));
        hi[b] = (b == GQ_NB) ? 0.0 : 2.0 * c * c;
    }
    const double lmin = 1e-2, c1 = 6.0;   // lam = lmin + c1 s, s in [0, 2]
    std::vector<double> hist(GQ_HIST, 0.0);
    // chunk sums too (k_gq_hist_perm's output: [chunk][moment], chunks of a bin consecutive),
    // 8 .. 71 chunks per bin, for k_gq_nodes_w's fused reduction
    std::vector<int> cfirst(GQ_NB + 1, 0);
    std::vector<double> part;
    srand(11);
    for (int b = 0; b < GQ_NB; ++b) {
        const double mid = 0.5 * (hi[b] + hi[b + 1]), hw = 0.5 * (hi[b] - hi[b + 1]);
        const int np = 200 + rand() % 400;
        const int nch = 8 + rand() % 64;
        cfirst[b + 1] = cfirst[b] + nch;
        part.resize((size_t)cfirst[b + 1] * GQ_NM, 0.0);
        for (int q = 0; q < np; ++q) {
            double* pc = &part[(size_t)(cfirst[b] + q % nch) * GQ_NM];
            const double u = 2.0 * rand() / (double)RAND_MAX - 1.0;
            const double s = mid + hw * u, lam = lmin + c1 * s;
            const double w = exp(-decay * lam) * (0.1 + rand() / (double)RAND_MAX);
            double tm2 = 1.0, tm1 = u;
            hist[0 * GQ_NB + b] += w;
            hist[1 * GQ_NB + b] += w * u;
            pc[0] += w;
            pc[1] += w * u;
            for (int m = 2; m < GQ_NM; ++m) {
                const double t = 2.0 * u * tm1 - tm2;
                hist[m * GQ_NB + b] += w * t;
                pc[m] += w * t;
                tm2 = tm1;
                tm1 = t;
            }
        }
    }
    double* dh;
    GqBins* B;
    GqExact* X;
    GqNodes* nd;
    int* cnt;
    CK(hipMalloc(&dh, sizeof(double) * GQ_HIST));
    CK(hipMalloc(&B, sizeof(GqBins)));
    CK(hipMalloc(&X, sizeof(GqExact)));
    CK(hipMalloc(&nd, sizeof(GqNodes)));
    CK(hipMalloc(&cnt, sizeof(int) * GQ_NODES));
    CK(hipMemcpy(dh, hist.data(), sizeof(double) * GQ_HIST, hipMemcpyHostToDevice));
    k_gq_bins<<<1, 256>>>(B);
    std::vector<int> xn(GQ_NB, GQ_XS + 1);
    CK(hipMemcpy(X->n, xn.data(), sizeof(int) * GQ_NB, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    hipEvent_t a, e;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&e));
    k_gq_nodes<<<GQ_NODES / 64, 64>>>(dh, B, X, 1, lmin, c1, nd);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < reps; ++i) k_gq_nodes<<<GQ_NODES / 64, 64>>>(dh, B, X, 1, lmin, c1, nd);
    CK(hipEventRecord(e, 0));
    CK(hipEventSynchronize(e));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, e));
    printf("k_gq_nodes: %.2f us per launch (decay %.1f)\n", 1e3 * ms / reps, decay);
    // the wave-per-bin form, from the histogram and from the chunk sums (+ k_gq_perm_reduce's
    // output for the bitwise check of the fused reduction)
    {
        double *dpart, *dh2;
        int* dcf;
        GqNodes* nd2;
        GqNodes* nd3;
        const int nch = cfirst[GQ_NB];
        CK(hipMalloc(&dpart, sizeof(double) * part.size()));
        CK(hipMalloc(&dh2, sizeof(double) * GQ_HIST));
        CK(hipMalloc(&dcf, sizeof(int) * (GQ_NB + 1)));
        CK(hipMalloc(&nd2, sizeof(GqNodes)));
        CK(hipMalloc(&nd3, sizeof(GqNodes)));
        CK(hipMemcpy(dpart, part.data(), sizeof(double) * part.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(dcf, cfirst.data(), sizeof(int) * (GQ_NB + 1), hipMemcpyHostToDevice));
        k_gq_perm_reduce<<<GQ_HIST / 4, 256>>>(dpart, dcf, dh2);
        k_gq_nodes<<<GQ_NODES / 64, 64>>>(dh2, B, X, 1, lmin, c1, nd);
        k_gq_nodes_w<<<GQ_NB / 4, 256>>>(dh2, nullptr, nullptr, B, X, 1, lmin, c1, nd2);
        k_gq_nodes_w<<<GQ_NB / 4, 256>>>(nullptr, dpart, dcf, B, X, 1, lmin, c1, nd3);
        CK(hipDeviceSynchronize());
        std::vector<double> l1(GQ_NODES), w1(GQ_NODES), l2(GQ_NODES), w2(GQ_NODES), l3(GQ_NODES), w3(GQ_NODES);
        CK(hipMemcpy(l1.data(), nd->lam, sizeof(double) * GQ_NODES, hipMemcpyDeviceToHost));
        CK(hipMemcpy(w1.data(), nd->w, sizeof(double) * GQ_NODES, hipMemcpyDeviceToHost));
        CK(hipMemcpy(l2.data(), nd2->lam, sizeof(double) * GQ_NODES, hipMemcpyDeviceToHost));
        CK(hipMemcpy(w2.data(), nd2->w, sizeof(double) * GQ_NODES, hipMemcpyDeviceToHost));
        CK(hipMemcpy(l3.data(), nd3->lam, sizeof(double) * GQ_NODES, hipMemcpyDeviceToHost));
        CK(hipMemcpy(w3.data(), nd3->w, sizeof(double) * GQ_NODES, hipMemcpyDeviceToHost));
        double dl = 0, dw = 0;
        int same23 = 1, nz = 0;
        for (int i = 0; i < GQ_NODES; ++i) {
            dl = std::max(dl, fabs(l2[i] - l1[i]) / fabs(l1[i]));
            if (w1[i] != 0.0) dw = std::max(dw, fabs(w2[i] - w1[i]) / fabs(w1[i]));
            nz += (w1[i] != 0.0);
            same23 &= (l2[i] == l3[i] && w2[i] == w3[i]);
        }
        printf("nodes_w vs nodes: max rel d lam %.2e, d w %.2e (%d weighted nodes); fused reduction bitwise %s\n",
               dl, dw, nz, same23 ? "equal" : "DIFFERENT");
        for (int pass = 0; pass < 2; ++pass) {
            CK(hipEventRecord(a, 0));
            for (int i = 0; i < reps; ++i) {
                if (pass == 0) k_gq_nodes_w<<<GQ_NB / 4, 256>>>(dh2, nullptr, nullptr, B, X, 1, lmin, c1, nd2);
                else k_gq_nodes_w<<<GQ_NB / 4, 256>>>(nullptr, dpart, dcf, B, X, 1, lmin, c1, nd3);
            }
            CK(hipEventRecord(e, 0));
            CK(hipEventSynchronize(e));
            CK(hipEventElapsedTime(&ms, a, e));
            printf("k_gq_nodes_w (%s): %.2f us per launch\n", pass ? "chunk sums, fused reduction" : "histogram",
                   1e3 * ms / reps);
        }
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < reps; ++i) k_gq_perm_reduce<<<GQ_HIST / 4, 256>>>(dpart, dcf, dh2);
        CK(hipEventRecord(e, 0));
        CK(hipEventSynchronize(e));
        CK(hipEventElapsedTime(&ms, a, e));
        printf("k_gq_perm_reduce: %.2f us per launch (%d chunks)\n", 1e3 * ms / reps, nch);
    }
    long long* clk;
    CK(hipMalloc(&clk, 4 * sizeof(long long)));
    k_nodes_count<<<GQ_NODES / 64, 64>>>(dh, X, cnt, clk);
    long long hc[4];
    CK(hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost));
    printf("thread 0 cycles (s_memtime): loads %lld, mcheb %lld, bisect %lld, newton %lld\n", hc[0], hc[1], hc[2], hc[3]);
    std::vector<int> c(GQ_NODES);
    CK(hipMemcpy(c.data(), cnt, sizeof(int) * GQ_NODES, hipMemcpyDeviceToHost));
    int hb[8] = {0}, fbs = 0, maxb = 0, maxn = 0, wave_max_sum = 0;
    for (int w = 0; w < GQ_NODES / 64; ++w) {
        int wm = 0;
        for (int l = 0; l < 64; ++l) {
            const int v = c[w * 64 + l];
            if (v < 0) continue;
            const int nb = v & 1023, nn = (v >> 10) & 1023, fb = v >> 20;
            maxb = std::max(maxb, nb);
            maxn = std::max(maxn, nn);
            fbs += fb;
            hb[std::min(7, nb / 16)]++;
            wm = std::max(wm, nb + 8 * nn);
        }
        wave_max_sum += wm;
    }
    printf("bisections: max %d; histogram by 16s:", maxb);
    for (int i = 0; i < 8; ++i) printf(" %d", hb[i]);
    printf("; newton max %d; fallbacks %d; mean per-wave max (bisect + 8 newton) %.1f\n", maxn, fbs,
           wave_max_sum / (double)(GQ_NODES / 64));
    return 0;
}
