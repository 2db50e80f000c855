// Pass-design lab: the spectral s-step pass (k_spec_s2, compiled from the product source)
// against a variant that streams r, q through a per-wave LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4, D tiles in flight per wave, counted vmcnt waits), at the bench
// grid.  Checks that both produce bit-identical r, q and the same moments (to rounding),
// and times them.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//       -I../optical-flow-optimal-transport_amd/csrc pass_lab.hip -o pass_lab
#include "../optical-flow-optimal-transport_amd/csrc/foto_spectral.hip"
#include <cstdio>
#include <vector>
namespace foto { void set_error(const char*, ...) {} }
using namespace foto;

__global__ __launch_bounds__(256) void stream_rq(double* __restrict__ r, double* __restrict__ q, size_t n2, double a,
                                                 double b) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        dbl2 rv = ((const dbl2*)r)[i], qv = ((const dbl2*)q)[i];
        dbl2 pn = b * qv + rv, rn = rv - a * pn;
        ((dbl2*)r)[i] = rn;
        ((dbl2*)q)[i] = pn;
    }
}

// the same stream with write-through (sc1) stores: no dirty L2 lines at the kernel boundary
__global__ __launch_bounds__(256) void stream_rq_wt(double* __restrict__ r, double* __restrict__ q, size_t n2, double a,
                                                    double b) {
    const __amdgpu_buffer_rsrc_t rr = wt_rsrc(r), rq = wt_rsrc(q);
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        dbl2 rv = ((const dbl2*)r)[i], qv = ((const dbl2*)q)[i];
        dbl2 pn = b * qv + rv, rn = rv - a * pn;
        st_wt16(rr, (int)(i * 16), rn);
        st_wt16(rq, (int)(i * 16), pn);
    }
}


// Kernel-boundary cost: npass ring passes in ONE launch (each block keeps its tiles and its
// LDS tables across passes), optionally with a grid-wide arrival counter between passes (the
// synchronisation a persistent solve needs for its moments).  The spin is bounded by the
// 100 MHz wall clock, so a non-resident grid cannot hang the box.
__device__ int lab_err;
template <int D>
__global__ __launch_bounds__(S2_NTH) __attribute__((amdgpu_waves_per_eu(S2_WPE))) void k_lab_multi(
        SpecTab T, double* __restrict__ rh, double* __restrict__ ph, const double* __restrict__ bh, const SStep* Sg,
        double* out, unsigned* ctr, int npass, int gsync) {
    __shared__ __attribute__((aligned(16))) double ring[RING_NW * D * RING_SLOT + RING_TAB];
    __shared__ double wred[RING_NW * NACC];
    __shared__ double tot[NACC];
    const SStep S0 = *Sg;
    double* tab = ring + RING_NW * D * RING_SLOT;
    const RingWave w = ring_wave(T, ring, D);
    ring_stage_tables(T, tab);
    __syncthreads();
    for (int p = 0; p < npass; ++p) {
        double acc[NACC];
#pragma unroll
        for (int m = 0; m < NACC; ++m) acc[m] = 0.0;
        ring_pass<D, false>(T, w, lds_u32(tab), S0, rh, ph, bh, acc, 0, true);
        blk_sum_rs<NACC, S2_NTH>(acc, wred, tot);
        if (threadIdx.x < NACC)
            __hip_atomic_store(&out[(int64_t)threadIdx.x * gridDim.x + blockIdx.x], tot[threadIdx.x], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifndef LAB_NOFENCE
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
        if (gsync) {
            __syncthreads();
            if (threadIdx.x == 0) {
                __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const unsigned target = (unsigned)(p + 1) * gridDim.x;
                const long long t0 = wall_clock64();
                while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (wall_clock64() - t0 > 100000000LL) { lab_err = 1; break; }   // 1 s
                }
            }
            __syncthreads();
        }
#ifndef LAB_NOFENCE
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
    }
}

int main(int argc, char** argv) {
    const int Nt = argc > 1 ? atoi(argv[1]) : 32, Ny = 480, Nx = 640;   // Nt sweep: fixed cost per pass
    const size_t n = (size_t)Nt * Ny * Nx;
    std::vector<double> mt(Nt), my(Ny), mx(Nx);
    for (int k = 0; k < Nt; ++k) mt[k] = 2 - 2 * cos(M_PI * k / Nt);
    for (int k = 0; k < Ny; ++k) my[k] = 2 - 2 * cos(M_PI * k / Ny);
    for (int k = 0; k < Nx; ++k) mx[k] = 2 - 2 * cos(M_PI * k / Nx);
    double *r, *p, *b, *r2, *p2, *dmt, *dmy, *dmx, *part, *gath, *gath2;
    unsigned* ticket;
    SStep *Sg, *Sg2;
    if (hipMalloc(&r, n * 8) || hipMalloc(&p, n * 8) || hipMalloc(&r2, n * 8) || hipMalloc(&p2, n * 8) ||
        hipMalloc(&b, n * 8) || hipMalloc(&dmt, 8 * Nt) || hipMalloc(&dmy, 8 * Ny) || hipMalloc(&dmx, 8 * Nx) ||
        hipMalloc(&part, 8 * (size_t)NACC * 8192) || hipMalloc(&gath, 8 * 256) || hipMalloc(&gath2, 8 * 256) ||
        hipMalloc(&ticket, 256) || hipMalloc(&Sg, sizeof(SStep)) || hipMalloc(&Sg2, sizeof(SStep)))
        return 1;
    std::vector<double> h(n), hq(n);
    for (size_t i = 0; i < n; ++i) {
        h[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5;
        hq[i] = 1e-3 * (double)((i * 40503u + 7) % 1000) - 0.5;
    }
    (void)hipMemcpy(dmt, mt.data(), 8 * Nt, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmy, my.data(), 8 * Ny, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmx, mx.data(), 8 * Nx, hipMemcpyHostToDevice);
    (void)hipMemcpy(b, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemset(ticket, 0, 256);
    SpecTab T{dmt, dmy, dmx, 1.0, 1e-2, Nt, Ny, Nx, 0, Ny};
    SStep S0{};
    S0.k = 10;
    S0.nsteps = SMAX;
    for (int i = 0; i < SMAX; ++i) { S0.a[i] = 0.05 + 0.01 * i; S0.b[i] = 0.3 + 0.02 * i; }
    S0.rho_prev = 1.0; S0.atol = 1e-30; S0.c0 = 6.0; S0.c1 = 6.0;
    RedBuf rb{part, ticket, NACC * 8192};
    auto reset = [&] {
        (void)hipMemcpy(r, h.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(p, hq.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(r2, h.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(p2, hq.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(Sg, &S0, sizeof(SStep), hipMemcpyHostToDevice);
        (void)hipMemcpy(Sg2, &S0, sizeof(SStep), hipMemcpyHostToDevice);
    };
    printf("SMAX=%d S2_NTH=%d ring D=%d pass sc1 stores %d grid %dx%dx%d\n", SMAX, S2_NTH, FOTO_RING_D, FOTO_PASS_WT, Nx, Ny, Nt);
    // correctness: one pass each from the same state, moments to gath (no fused plan)
    reset();
    const int G = 256;
    k_spec_s2<true, false, false><<<G, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0);
    if (launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, false, 0) != hipSuccess) {
        printf("ring launch failed\n");
        return 3;
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("fault\n"); return 2; }
    {
        std::vector<double> a1(n), a2(n), q1(n), q2(n), m1(NACC), m2(NACC);
        (void)hipMemcpy(a1.data(), r, n * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(a2.data(), r2, n * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(q1.data(), p, n * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(q2.data(), p2, n * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(m1.data(), gath, 8 * NACC, hipMemcpyDeviceToHost);
        (void)hipMemcpy(m2.data(), gath2, 8 * NACC, hipMemcpyDeviceToHost);
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += (a1[i] != a2[i]) + (q1[i] != q2[i]);
        double md = 0;
        for (int m = 0; m < NACC; ++m) md = fmax(md, fabs(m1[m] - m2[m]) / fmax(fabs(m1[m]), 1e-300));
        printf("ring vs product: %zu differing r/q elements, max moment rel diff %.3e (M0 %.17g / %.17g)\n", bad, md,
               m1[0], m2[0]);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    // back-to-back launches (as in a solve): moments to gath, no plan (S stays valid)
    auto timeit = [&](const char* name, auto launch) {
        (void)hipMemcpy(Sg, &S0, sizeof(SStep), hipMemcpyHostToDevice);
        (void)hipMemcpy(Sg2, &S0, sizeof(SStep), hipMemcpyHostToDevice);
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipEventRecord(e0);
            for (int i = 0; i < 20; ++i) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (t < best) best = t;
        }
        printf("%-44s %6.1f us per launch (20 back to back)\n", name, best * 1e3 / 20);
    };
    timeit("pure stream r,q (1024 x 256)", [&] { stream_rq<<<1024, 256>>>(r, p, n / 2, 1e-9, 1e-9); });
    timeit("pure stream r,q (2048 x 256)", [&] { stream_rq<<<2048, 256>>>(r, p, n / 2, 1e-9, 1e-9); });
    timeit("pure stream r,q, sc1 stores (1024 x 256)", [&] { stream_rq_wt<<<1024, 256>>>(r, p, n / 2, 1e-9, 1e-9); });
    timeit("pure stream r,q, sc1 stores (2048 x 256)", [&] { stream_rq_wt<<<2048, 256>>>(r, p, n / 2, 1e-9, 1e-9); });
    timeit("product k_spec_s2, moments only", [&] { k_spec_s2<true, false, false><<<256, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0); });
    for (int d : {2, 4, FOTO_RING_D}) {
        char nm[64];
        snprintf(nm, sizeof nm, "ring D=%d, moments only", d);
        timeit(nm, [&] { (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, false, d); });
    }
    timeit("ring INIT, moments only", [&] { (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, true, false, 0); });
    timeit("product INIT, moments only", [&] { k_spec_s2<true, true, false><<<256, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0); });

    {   // one launch, 20 passes: no grid sync / with the arrival counter
        for (int np : {1, 2, 4}) {
            float best = 1e9;
            for (int rep = 0; rep < 5; ++rep) {
                (void)hipEventRecord(e0);
                k_lab_multi<FOTO_RING_D><<<256, S2_NTH>>>(T, r2, p2, b, Sg2, part, ticket, np, 0);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float t;
                (void)hipEventElapsedTime(&t, e0, e1);
                if (t < best) best = t;
            }
            printf("persistent ring, %d passes, no grid sync     %6.1f us per pass\n", np, best * 1e3 / np);
        }
        for (int gs = 0; gs < 2; ++gs) {
            float best = 1e9;
            for (int rep = 0; rep < 5; ++rep) {
                (void)hipMemset(ticket, 0, 256);
                (void)hipEventRecord(e0);
                k_lab_multi<FOTO_RING_D><<<256, S2_NTH>>>(T, r2, p2, b, Sg2, part, ticket, 20, gs);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float t;
                (void)hipEventElapsedTime(&t, e0, e1);
                if (t < best) best = t;
            }
            int herr = 0;
            (void)hipMemcpyFromSymbol(&herr, HIP_SYMBOL(lab_err), sizeof herr);
            printf("%-44s %6.1f us per pass (one launch of 20%s)\n", gs ? "persistent ring, grid counter" : "persistent ring, no grid sync",
                   best * 1e3 / 20, herr ? ", SPIN TIMEOUT" : "");
        }
        (void)hipMemset(ticket, 0, 256);
    }
    auto single = [&](const char* name, auto launch) {
        float best = 1e9;
        for (int rep = 0; rep < 20; ++rep) {
            (void)hipMemcpy(Sg2, &S0, sizeof(SStep), hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (t < best) best = t;
        }
        printf("%-44s %6.1f us (single launch)\n", name, best * 1e3);
    };
    single("ring D=4 moments only", [&] { (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, false, 0); });
    single("plan kernel alone (8 steps)", [&] { k_spec_s2_plan<<<1, 64>>>(Sg2, gath2, 1, 0, 1e-6, 1000); });
    single("plan kernel alone (maxiter 0)", [&] { k_spec_s2_plan<<<1, 64>>>(Sg2, gath2, 1, 0, 1e-6, 0); });
    {
        SStep hS;
        (void)hipMemcpy(Sg2, &S0, sizeof(SStep), hipMemcpyHostToDevice);
        k_spec_s2_plan<<<1, 64>>>(Sg2, gath2, 1, 0, 1e-6, 1000);
        (void)hipMemcpy(&hS, Sg2, sizeof(SStep), hipMemcpyDeviceToHost);
        printf("   (plan from these moments: %d steps)\n", hS.nsteps);
    }
    // one fused pass timed alone: the plan made at its start from the moments in gath2
    // (S.pend = 1, as in a solve), the pass, the moments and state published in its tail
    {
        std::vector<double> gsave(NACC);
        (void)hipMemcpy(gsave.data(), gath2, 8 * NACC, hipMemcpyDeviceToHost);
        SStep Sl = S0;
        Sl.pend = 1;
        Sl.fin = 0;
        float best = 1e9;
        for (int rep = 0; rep < 20; ++rep) {
            (void)hipMemcpy(Sg2, &Sl, sizeof(SStep), hipMemcpyHostToDevice);
            (void)hipMemcpy(gath2, gsave.data(), 8 * NACC, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, true, 0);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (t < best) best = t;
        }
        SStep hS;
        (void)hipMemcpy(&hS, Sg2, sizeof(SStep), hipMemcpyDeviceToHost);
        printf("%-44s %6.1f us (single launch; %d steps, pend %d)\n", "ring D=4 fused plan (at start)", best * 1e3,
               hS.nsteps, hS.pend);
#ifdef FOTO_PLAN_CLOCK
        long long ck[8];
        (void)hipMemcpyFromSymbol(ck, HIP_SYMBOL(foto_plan_clock), sizeof ck);
        printf("   block 0 wave 0: moments load + plan %.2f us, then barrier %.2f us\n", (ck[1] - ck[0]) * 0.01,
               (ck[2] - ck[1]) * 0.01);
        printf("   plan: to Gram rows %.2f us, steps %.2f us, interval %.2f us, stores %.2f us\n",
               (ck[3] - ck[0]) * 0.01, (ck[4] - ck[3]) * 0.01, (ck[5] - ck[4]) * 0.01, (ck[1] - ck[5]) * 0.01);
#endif
    }
    // the first pass of a solve: the plan from the INIT moments of r_0 = b (q = 0, k = 0), as in
    // a real solve a well-conditioned measure -> an 8-step plan (the state above is random r, q
    // with made-up scalars, which plans 1 step)
    {
        SStep Si = S0;
        Si.k = 0; Si.nsteps = 0; Si.fin = 0; Si.done = 0; Si.pend = 0; Si.rho_prev = 0.0; Si.atol = 1e-30;
        Si.c0 = Si.gc0 = Si.ic0 = 6.005; Si.c1 = Si.gc1 = Si.ic1 = 5.995;
        (void)hipMemcpy(Sg2, &Si, sizeof(SStep), hipMemcpyHostToDevice);
        (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, true, false, 0);   // INIT moments -> gath2
        if (hipDeviceSynchronize() != hipSuccess) { printf("fault\n"); return 2; }
        std::vector<double> gsave(NACC);
        (void)hipMemcpy(gsave.data(), gath2, 8 * NACC, hipMemcpyDeviceToHost);
        Si.pend = 1;
        float best = 1e9;
        for (int rep = 0; rep < 20; ++rep) {
            (void)hipMemcpy(Sg2, &Si, sizeof(SStep), hipMemcpyHostToDevice);
            (void)hipMemcpy(gath2, gsave.data(), 8 * NACC, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, true, 0);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (t < best) best = t;
        }
        SStep hS;
        (void)hipMemcpy(&hS, Sg2, sizeof(SStep), hipMemcpyDeviceToHost);
        printf("%-44s %6.1f us (single launch; %d steps, pend %d)\n", "ring D=4 first pass, plan from INIT moments",
               best * 1e3, hS.nsteps, hS.pend);
        // a solve's pass sequence: from the INIT state, 16 late-planning passes back to back (each
        // plans from the moments the previous one left), as the solver enqueues them
        float bseq = 1e9;
        int kdone = 0, npass = 0;
        for (int rep = 0; rep < 5; ++rep) {
            (void)hipMemcpy(Sg2, &Si, sizeof(SStep), hipMemcpyHostToDevice);
            (void)hipMemcpy(gath2, gsave.data(), 8 * NACC, hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            for (int i = 0; i < 16; ++i) (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, true, 0);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (t < bseq) bseq = t;
            (void)hipMemcpy(&hS, Sg2, sizeof(SStep), hipMemcpyDeviceToHost);
            kdone = hS.k + hS.nsteps;
            npass = hS.passes;
        }
        printf("%-44s %6.1f us per pass (16 back to back; %d plans, %d CG iterations planned)\n",
               "ring D=4 solve sequence from INIT", bseq * 1e3 / 16, npass, kdone);
#ifdef FOTO_PLAN_CLOCK
        long long ck[8];
        (void)hipMemcpyFromSymbol(ck, HIP_SYMBOL(foto_plan_clock), sizeof ck);
        printf("   block 0 wave 0: moments load + plan %.2f us, then barrier %.2f us\n", (ck[1] - ck[0]) * 0.01,
               (ck[2] - ck[1]) * 0.01);
        printf("   plan: to Gram rows %.2f us, steps %.2f us, interval %.2f us, stores %.2f us\n",
               (ck[3] - ck[0]) * 0.01, (ck[4] - ck[3]) * 0.01, (ck[5] - ck[4]) * 0.01, (ck[1] - ck[5]) * 0.01);
#endif
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}
