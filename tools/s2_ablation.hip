// Times the real spectral s-step pass (k_spec_s2, compiled from the product source) at the
// bench grid in isolation, to split its duration into streaming body, cross-block reduction
// and single-thread planning.  Each rep restores the same SStep (two steps, not finished).
#include "../optical-flow-optimal-transport_amd/csrc/foto_spectral.hip"
#include <cstdio>
#include <vector>
namespace foto { void set_error(const char*, ...) {} }
using namespace foto;


template <int MOM>
__global__ __launch_bounds__(256) void spass(double* __restrict__ r, double* __restrict__ p, const double* mt,
                                             const double* my, const double* mx, int Nt, int Ny, int Nx, double a0,
                                             double b0, double a1, double b1, double* out) {
    const int rows = Nt * Ny, ntx = (Nx + 127) / 128, ntiles = ntx * ((rows + 3) / 4);
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    double acc[12];
    for (int m = 0; m < 12; ++m) acc[m] = 0.0;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int row = (t / ntx) * 4 + ty, kx = (t % ntx) * 128 + 2 * tx;
        if (row >= rows || kx >= Nx) continue;
        const int kt = row / Ny, ky = row - kt * Ny;
        const double rm = mt[kt] + my[ky];
        const double l0 = 0.01 + (rm + mx[kx]), l1 = 0.01 + (rm + mx[kx + 1]);
        const size_t i = (size_t)row * Nx + kx;
        dbl2 rv = *(const dbl2*)(r + i), qv = *(const dbl2*)(p + i);
        double r0 = rv[0], r1 = rv[1], q0 = qv[0], q1 = qv[1];
        double p0 = b0 * q0 + r0, p1 = b0 * q1 + r1;
        r0 = r0 - a0 * (l0 * p0); r1 = r1 - a0 * (l1 * p1); q0 = p0; q1 = p1;
        p0 = b1 * q0 + r0; p1 = b1 * q1 + r1;
        r0 = r0 - a1 * (l0 * p0); r1 = r1 - a1 * (l1 * p1); q0 = p0; q1 = p1;
        *(dbl2*)(r + i) = dbl2{r0, r1};
        *(dbl2*)(p + i) = dbl2{q0, q1};
        if (MOM) {
            double ls[2] = {l0, l1}, rs[2] = {r0, r1}, qs[2] = {q0, q1};
            for (int e = 0; e < 2; ++e) {
                const double x = (ls[e] - 6.0) * 0.16;
                double T[4] = {1.0, x, 0, 0};
                T[2] = 2.0 * x * T[1] - T[0];
                T[3] = 2.0 * x * T[2] - T[1];
                const double rr = rs[e] * rs[e], rq = rs[e] * qs[e], qq = qs[e] * qs[e];
                for (int m = 0; m < 4; ++m) { acc[m] += T[m] * rr; acc[4 + m] += T[m] * rq; acc[8 + m] += T[m] * qq; }
            }
        }
    }
    double s = 0;
    for (int m = 0; m < 12; ++m) s += acc[m];
    if (s == 1.2345) out[0] = s;
}


// ---- candidate reduction: block sums by LDS transpose (no shuffles), partials laid out
// [block][16] (one 128-B line per block), optional two-level tickets (groups of GS blocks).
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// sum of v[k] over the block's NTH threads into out[k] (valid in threads 0..K-1 via LDS)
template <int K, int NTH>
__device__ __forceinline__ void blk_sum_lds(const double (&v)[K], double* red /* K*NTH */, double* red2 /* K*16 */) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; ++k) red[k * NTH + tid] = v[k];
    __syncthreads();
    constexpr int SEG = NTH / 16;
    if (tid < K * 16) {
        const int k = tid >> 4, sg = tid & 15;
        const double* a = red + k * NTH + sg * SEG;
        double s = a[0];
#pragma unroll
        for (int j = 1; j < SEG; ++j) s += a[j];
        red2[k * 16 + sg] = s;
    }
    __syncthreads();
}
template <int K, int NTH, int MODE0>   // MODE 2: no ticket; 3: one ticket; 4: two-level (GS = 32)
__device__ bool red_new(double (&v)[K], double* part, unsigned* tickets, double* tot) {
    static_assert(K <= 16, "");
    constexpr bool KM = (MODE0 == 8);
    constexpr int MODE = KM ? 3 : MODE0;
    __shared__ double red[K * NTH];
    __shared__ double red2[K * 16];
    __shared__ int is_last;
    const int tid = threadIdx.x, nb = gridDim.x, b = blockIdx.x;
    blk_sum_lds<K, NTH>(v, red, red2);
    auto fin16 = [&](int k) {
        double s = red2[k * 16];
#pragma unroll
        for (int j = 1; j < 16; ++j) s += red2[k * 16 + j];
        return s;
    };
    if (tid < K) st_sc1(KM ? part + (int64_t)tid * nb + b : part + (int64_t)b * 16 + tid, fin16(tid));
    if (MODE == 2) return false;
    if (MODE >= 5) {   // 5: wait + single atomic, 6: wait only, 7: atomic only; no tail
        if (tid < 64) {
            if (MODE != 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (tid == 0 && MODE != 6) {
                const unsigned t = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                is_last = (t == (unsigned)(nb - 1));
                if (is_last) __hip_atomic_store(tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        return false;
    }
    constexpr int GS = 32;
    const int ng = (nb + GS - 1) / GS, g = b / GS, gs = min(GS, nb - g * GS);
    if (tid < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) {
            unsigned* tk = (MODE == 3) ? tickets : tickets + 32 * (1 + g);
            const unsigned t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            is_last = (t == (unsigned)((MODE == 3 ? nb : gs) - 1));
            if (is_last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (!is_last) return false;
    // reduce n rows of part (stride 16) starting at row r0 into tot[K] (fixed order)
    auto reduce_rows = [&](const double* src, int n) {
        double x[K];
#pragma unroll
        for (int k = 0; k < K; ++k) x[k] = 0.0;
        constexpr int RPT = 4;   // rows per thread per round trip
        for (int base = 0; base < n; base += RPT * NTH) {
            double y[RPT][K];
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const int rr = min(base + tid + j * NTH, n - 1);   // unconditional loads: one round trip
#pragma unroll
                for (int k = 0; k < K; ++k) y[j][k] = ld_sc1(KM ? src + (int64_t)k * n + rr : src + (int64_t)rr * 16 + k);
            }
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
                const bool ok = base + tid + j * NTH < n;
#pragma unroll
                for (int k = 0; k < K; ++k) x[k] += ok ? y[j][k] : 0.0;
            }
        }
        __syncthreads();
        blk_sum_lds<K, NTH>(x, red, red2);
        if (tid < K) tot[tid] = fin16(tid);
        __syncthreads();
    };
    if (MODE == 3) {
        reduce_rows(part, nb);
        return true;
    }
    reduce_rows(part + (int64_t)g * GS * 16, gs);
    double* gpart = part + (int64_t)nb * 16;   // group partials [g][16]
    if (tid < K) st_sc1(gpart + (int64_t)g * 16 + tid, tot[tid]);
    if (tid < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0) {
            const unsigned t = __hip_atomic_fetch_add(tickets, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            is_last = (t == (unsigned)(ng - 1));
            if (is_last) __hip_atomic_store(tickets, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    if (!is_last) return false;
    reduce_rows(gpart, ng);
    return true;
}

// Copy of k_spec_s2 (FUSE = false) with knobs: RED 0 = skip the cross-block reduction
// (keep accumulators live), 1 = sp_reduce_last_wide; PIPE 0 = plain tile loop.
template <int RED, int PIPE>
__global__ __launch_bounds__(S2_NTH) void k_abl(SpecTab T, double* __restrict__ rh, double* __restrict__ ph,
                                               SStep* Sg, RedBuf rb, double* gath) {
    constexpr int TR = S2_NTH / 64;
    __shared__ SStep SS;
    if (threadIdx.x == 0) SS = *Sg;
    __syncthreads();
    const int k = SS.k, ns = SS.nsteps;
    const double a0 = SS.a[0], b0 = SS.b[0], a1 = SS.a[1], b1 = SS.b[1];
    const double c0 = SS.c0, ic1 = 1.0 / SS.c1;
    double acc[3 * SM];
    for (int m = 0; m < 3 * SM; ++m) acc[m] = 0.0;
    auto moments = [&](double lam, double r, double q) {
        double Tm[SM];
        cheb_all((lam - c0) * ic1, Tm);
        const double rr = r * r, rq = r * q, qq = q * q;
        for (int m = 0; m < SM; ++m) { acc[m] += Tm[m] * rr; acc[SM + m] += Tm[m] * rq; acc[2 * SM + m] += Tm[m] * qq; }
    };
    auto body = [&](const SpElem& e, double r0, double r1, double q0, double q1) {
        double p0 = b0 * q0 + r0, p1 = b0 * q1 + r1;
        r0 = r0 - a0 * (e.l0 * p0); r1 = r1 - a0 * (e.l1 * p1); q0 = p0; q1 = p1;
        if (ns == 2) { p0 = b1 * q0 + r0; p1 = b1 * q1 + r1; r0 = r0 - a1 * (e.l0 * p0); r1 = r1 - a1 * (e.l1 * p1); q0 = p0; q1 = p1; }
        st2<true>(rh, e.i, e.n2, r0, r1);
        st2<true>(ph, e.i, e.n2, q0, q1);
        moments(e.l0, r0, q0);
        if (e.n2 == 2) moments(e.l1, r1, q1);
    };
    const int rows = T.Nt * T.nyl, ntx = (T.Nx + 127) / 128, ntiles = ntx * ((rows + TR - 1) / TR);
    if (PIPE) {
        int t = blockIdx.x;
        SpElem e = spec_elem<TR>(T, t < ntiles ? t : 0, ntx, rows);
        if (t >= ntiles) e.n2 = 0;
        double r0 = 0, r1 = 0, q0 = 0, q1 = 0;
        if (e.n2) { ld2<true>(rh, e.i, e.n2, r0, r1); ld2<true>(ph, e.i, e.n2, q0, q1); }
        while (t < ntiles) {
            const int tn = t + gridDim.x;
            SpElem en = spec_elem<TR>(T, tn < ntiles ? tn : 0, ntx, rows);
            if (tn >= ntiles) en.n2 = 0;
            double nr0 = 0, nr1 = 0, nq0 = 0, nq1 = 0;
            if (en.n2) { ld2<true>(rh, en.i, en.n2, nr0, nr1); ld2<true>(ph, en.i, en.n2, nq0, nq1); }
            if (e.n2) body(e, r0, r1, q0, q1);
            e = en; r0 = nr0; r1 = nr1; q0 = nq0; q1 = nq1; t = tn;
        }
    } else {
        for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
            SpElem e = spec_elem<TR>(T, t, ntx, rows);
            if (!e.n2) continue;
            double r0, r1, q0, q1;
            ld2<true>(rh, e.i, e.n2, r0, r1); ld2<true>(ph, e.i, e.n2, q0, q1);
            body(e, r0, r1, q0, q1);
        }
    }
    if (RED >= 2) {
        __shared__ double tot[3 * SM];
        if (red_new<3 * SM, S2_NTH, RED>(acc, rb.partials, rb.ticket, tot) && threadIdx.x == 0)
            for (int m = 0; m < 3 * SM; ++m) gath[m] = tot[m];
    } else if (RED) {
        __shared__ double tot[3 * SM];
        if (sp_reduce_last_wide<3 * SM, S2_NTH>(acc, rb, tot) && threadIdx.x == 0)
            for (int m = 0; m < 3 * SM; ++m) gath[m] = tot[m];
    } else {
        double s = 0;
        for (int m = 0; m < 3 * SM; ++m) s += acc[m];
        if (s == 1.2345) gath[0] = s;
    }
}

int main() {
    const int Nt = 32, Ny = 480, Nx = 640;
    const size_t n = (size_t)Nt * Ny * Nx;
    std::vector<double> mt(Nt), my(Ny), mx(Nx);
    for (int k = 0; k < Nt; ++k) mt[k] = 2 - 2 * cos(M_PI * k / Nt);
    for (int k = 0; k < Ny; ++k) my[k] = 2 - 2 * cos(M_PI * k / Ny);
    for (int k = 0; k < Nx; ++k) mx[k] = 2 - 2 * cos(M_PI * k / Nx);
    double *r, *p, *b, *dmt, *dmy, *dmx, *part, *gath;
    unsigned* ticket;
    SStep* Sg;
    if (hipMalloc(&r, n * 8) || hipMalloc(&p, n * 8) || hipMalloc(&b, n * 8) || hipMalloc(&dmt, 8 * Nt) ||
        hipMalloc(&dmy, 8 * Ny) || hipMalloc(&dmx, 8 * Nx) || hipMalloc(&part, 8 * 12 * 65536) ||
        hipMalloc(&gath, 8 * 64) || hipMalloc(&ticket, 65536) || hipMalloc(&Sg, sizeof(SStep)))
        return 1;
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5;
    (void)hipMemcpy(r, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(p, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmt, mt.data(), 8 * Nt, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmy, my.data(), 8 * Ny, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmx, mx.data(), 8 * Nx, hipMemcpyHostToDevice);
    (void)hipMemset(ticket, 0, 65536);
    SpecTab T{dmt, dmy, dmx, 1.0, 1e-2, Nt, Ny, Nx, 0, Ny};
    SStep S0{};
    S0.k = 10; S0.nsteps = 2; S0.a[0] = S0.a[1] = 1e-9; S0.b[0] = S0.b[1] = 1e-9;
    S0.rho_prev = 1.0; S0.atol = 1e-30; S0.c0 = 6.0; S0.c1 = 6.0;
    RedBuf rb{part, ticket, 12 * 65536};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int grids[5] = {256, 512, 1024, 2048, 4096};
    for (int gi = 0; gi < 5; ++gi) {
        for (int fuse = 0; fuse < 2; ++fuse) {
            float best = 1e9, sum = 0;
            for (int rep = 0; rep < 30; ++rep) {
                (void)hipMemcpy(Sg, &S0, sizeof(SStep), hipMemcpyHostToDevice);
                (void)hipEventRecord(e0);
                if (fuse) k_spec_s2<true, false, true><<<grids[gi], S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, nullptr, 0);
                else k_spec_s2<true, false, false><<<grids[gi], S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0);
                (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
                float t; (void)hipEventElapsedTime(&t, e0, e1);
                if (t < best) best = t;
                if (rep >= 10) sum += t;
            }
            printf("k_spec_s2 grid=%d fuse=%d best %6.1f us  mean %6.1f us\n", grids[gi], fuse, best * 1e3, sum / 20 * 1e3);
        }
    }
    for (int gi = 0; gi < 5; ++gi) {
        for (int v = 0; v < 11; ++v) {
            float best = 1e9, sum = 0;
            for (int rep = 0; rep < 30; ++rep) {
                if (rep == 0) (void)hipMemcpy(Sg, &S0, sizeof(SStep), hipMemcpyHostToDevice);
                (void)hipEventRecord(e0);
                const int G = grids[gi];
                if (v == 0) k_abl<0, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 1) k_abl<0, 1><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 2) k_abl<1, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 3) k_abl<1, 1><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 4) k_abl<2, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 5) k_abl<3, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 6) k_abl<4, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 7) k_abl<5, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 8) k_abl<6, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 9) k_abl<7, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                if (v == 10) k_abl<8, 0><<<G, S2_NTH>>>(T, r, p, Sg, rb, gath);
                (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
                float t; (void)hipEventElapsedTime(&t, e0, e1);
                if (t < best) best = t;
                if (rep >= 10) sum += t;
            }
            printf("k_abl grid=%d red=%d pipe=%d best %6.1f us  mean %6.1f us\n", grids[gi], v < 4 ? v >> 1 : v - 2, v < 4 ? v & 1 : 0, best * 1e3, sum / 20 * 1e3);
        }
    }
    {
        double h1[12], h3[12], h4[12];
        k_abl<1, 0><<<1024, S2_NTH>>>(T, r, p, Sg, rb, gath);
        (void)hipMemcpy(h1, gath, 96, hipMemcpyDeviceToHost);
        k_abl<3, 0><<<1024, S2_NTH>>>(T, r, p, Sg, rb, gath);
        (void)hipMemcpy(h3, gath, 96, hipMemcpyDeviceToHost);
        k_abl<4, 0><<<1000, S2_NTH>>>(T, r, p, Sg, rb, gath);
        (void)hipMemcpy(h4, gath, 96, hipMemcpyDeviceToHost);
        double m3 = 0, m4 = 0;
        for (int m = 0; m < 12; ++m) { m3 = fmax(m3, fabs(h3[m] - h1[m]) / fabs(h1[m])); m4 = fmax(m4, fabs(h4[m] - h1[m]) / fabs(h1[m])); }
        printf("check rel diff red3 %.3e red4 %.3e (h1[0]=%.6e)\n", m3, m4, h1[0]);
    }
    double* z;
    (void)hipMalloc(&z, 2 * n * 8);
    (void)hipMemset(z, 0, 2 * n * 8);
    for (int zero = 0; zero < 2; ++zero) {
        double* rr = zero ? z : r;
        double* pp = zero ? z + n : p;
        float best = 1e9;
        for (int rep = 0; rep < 30; ++rep) {
            (void)hipEventRecord(e0);
            spass<1><<<1024, 256>>>(rr, pp, dmt, dmy, dmx, Nt, Ny, Nx, 1e-9, 1e-9, 1e-9, 1e-9, gath);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float t; (void)hipEventElapsedTime(&t, e0, e1);
            if (t < best) best = t;
        }
        printf("spass zero=%d best %6.1f us\n", zero, best * 1e3);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}
