// Times the real spectral s-step pass (k_spec_s2, compiled from the product source) at the
// bench grid in isolation: with / without the fused plan, over grid sizes, against a pure
// streaming pass of the same access pattern (read r, q; write r, q; non-zero data -- zero
// data streams faster on this part).  Build with -DFOTO_SMAX=<s> to compare pass widths.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//       -I../optical-flow-optimal-transport_amd/csrc s2_ablation.hip -o s2_ablation
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
    double *r, *p, *b, *dmt, *dmy, *dmx, *part, *gath;
    unsigned* ticket;
    SStep* Sg;
    if (hipMalloc(&r, n * 8) || hipMalloc(&p, n * 8) || hipMalloc(&b, n * 8) || hipMalloc(&dmt, 8 * Nt) ||
        hipMalloc(&dmy, 8 * Ny) || hipMalloc(&dmx, 8 * Nx) || hipMalloc(&part, 8 * (size_t)NACC * 8192) ||
        hipMalloc(&gath, 8 * 256) || hipMalloc(&ticket, 256) || hipMalloc(&Sg, sizeof(SStep)))
        return 1;
    std::vector<double> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5;
    (void)hipMemcpy(r, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(p, h.data(), n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmt, mt.data(), 8 * Nt, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmy, my.data(), 8 * Ny, hipMemcpyHostToDevice);
    (void)hipMemcpy(dmx, mx.data(), 8 * Nx, hipMemcpyHostToDevice);
    (void)hipMemset(ticket, 0, 256);
    SpecTab T{dmt, dmy, dmx, 1.0, 1e-2, Nt, Ny, Nx, 0, Ny};
    SStep S0{};
    S0.k = 10;
    S0.nsteps = SMAX;
    for (int i = 0; i < SMAX; ++i) { S0.a[i] = 1e-9; S0.b[i] = 1e-9; }
    S0.rho_prev = 1.0; S0.atol = 1e-30; S0.c0 = 6.0; S0.c1 = 6.0;
    RedBuf rb{part, ticket, NACC * 8192};
    int per_cu = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_spec_s2<true, false, true>, S2_NTH, 0);
    printf("SMAX=%d NACC=%d blocks/CU=%d\n", SMAX, NACC, per_cu);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto timeit = [&](auto launch, bool reset) {
        float best = 1e9;
        for (int rep = 0; rep < 30; ++rep) {
            if (reset) (void)hipMemcpy(Sg, &S0, sizeof(SStep), hipMemcpyHostToDevice);
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float t;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (t < best) best = t;
        }
        return best * 1e3;
    };
    printf("pure stream r,q (1024 blocks): %6.1f us\n",
           timeit([&] { stream_rq<<<1024, 256>>>(r, p, n / 2, 1e-9, 1e-9); }, false));
    const int grids[6] = {256, 512, 768, 1024, 1536, 2048};
    for (int gi = 0; gi < 6; ++gi) {
        const int G = grids[gi];
        const double tf = timeit([&] { k_spec_s2<true, false, true><<<G, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, nullptr, 0); }, true);
        const double tg = timeit([&] { k_spec_s2<true, false, false><<<G, S2_NTH>>>(T, r, p, b, Sg, rb, 1e-6, 1000, gath, 0); }, true);
        printf("k_spec_s2 grid=%5d  fused plan %6.1f us   moments only %6.1f us\n", G, tf, tg);
    }
    {   // the planning step alone (moments from the last moments-only run in gath)
        const double tp = timeit([&] { k_spec_s2_plan<<<1, 64>>>(Sg, gath, 1, 0, 1e-6, 1000); }, true);
        const double tz = timeit([&] { k_spec_s2_plan<<<1, 64>>>(Sg, gath, 1, 0, 1e-6, 0); }, true);
        SStep h;
        (void)hipMemcpy(Sg, &S0, sizeof(SStep), hipMemcpyHostToDevice);
        k_spec_s2_plan<<<1, 64>>>(Sg, gath, 1, 0, 1e-6, 1000);
        (void)hipMemcpy(&h, Sg, sizeof(SStep), hipMemcpyDeviceToHost);
        printf("plan kernel: %6.1f us (maxiter 0: %6.1f us), planned steps %d\n", tp, tz, h.nsteps);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    return 0;
}
