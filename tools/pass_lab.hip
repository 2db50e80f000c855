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

int main() {
    const int Nt = 32, Ny = 480, Nx = 640;
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
    printf("SMAX=%d S2_NTH=%d ring D=%d\n", SMAX, S2_NTH, FOTO_RING_D);
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
    timeit("product k_spec_s2, moments only", [&] { k_spec_s2<true, false, false><<<256, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0); });
    for (int d : {2, 4, FOTO_RING_D}) {
        char nm[64];
        snprintf(nm, sizeof nm, "ring D=%d, moments only", d);
        timeit(nm, [&] { (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, false, false, d); });
    }
    timeit("ring INIT, moments only", [&] { (void)launch_s2_ring(T, r2, p2, b, Sg2, rb, 1e-6, 1000, gath2, 0, true, false, 0); });
    timeit("product INIT, moments only", [&] { k_spec_s2<true, true, false><<<256, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0); });
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
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}
