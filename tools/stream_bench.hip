// Micro-benchmark of the spectral CG pass access pattern on gfx950: read r, p (2 x N fp64),
// write r, p back in place, N = 640*480*32.  Variants: load/store width, non-temporal
// hints, working-set size (fits / exceeds the 256 MiB Infinity Cache), and a read-only and
// write-only reference.  Prints GB/s per variant (best of 20).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double dbl2 __attribute__((ext_vector_type(2)));

template <int V>
__global__ __launch_bounds__(256) void k(double* __restrict__ r, double* __restrict__ p, size_t n, double a,
                                         double b) {
    const size_t n2 = n / 2;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        if (V == 0) {   // 16-B loads, 16-B stores
            dbl2 rv = ((const dbl2*)r)[i], pv = ((const dbl2*)p)[i];
            dbl2 pn = b * pv + rv, rn = rv - a * pn;
            ((dbl2*)r)[i] = rn;
            ((dbl2*)p)[i] = pn;
        } else if (V == 1) {   // 16-B loads, 8-B stores
            dbl2 rv = ((const dbl2*)r)[i], pv = ((const dbl2*)p)[i];
            dbl2 pn = b * pv + rv, rn = rv - a * pn;
            r[2 * i] = rn[0]; r[2 * i + 1] = rn[1];
            p[2 * i] = pn[0]; p[2 * i + 1] = pn[1];
        } else if (V == 2) {   // 16-B loads, non-temporal 16-B stores
            dbl2 rv = ((const dbl2*)r)[i], pv = ((const dbl2*)p)[i];
            dbl2 pn = b * pv + rv, rn = rv - a * pn;
            __builtin_nontemporal_store(rn, (dbl2*)r + i);
            __builtin_nontemporal_store(pn, (dbl2*)p + i);
        } else if (V == 3) {   // non-temporal loads and stores
            dbl2 rv = __builtin_nontemporal_load((const dbl2*)r + i), pv = __builtin_nontemporal_load((const dbl2*)p + i);
            dbl2 pn = b * pv + rv, rn = rv - a * pn;
            __builtin_nontemporal_store(rn, (dbl2*)r + i);
            __builtin_nontemporal_store(pn, (dbl2*)p + i);
        } else if (V == 4) {   // 8-B loads and stores (scalar per element, 2 per lane)
            double r0 = r[2 * i], r1 = r[2 * i + 1], p0 = p[2 * i], p1 = p[2 * i + 1];
            double q0 = b * p0 + r0, q1 = b * p1 + r1;
            r[2 * i] = r0 - a * q0; r[2 * i + 1] = r1 - a * q1;
            p[2 * i] = q0; p[2 * i + 1] = q1;
        }
    }
}

__global__ void rdonly(const dbl2* __restrict__ r, const dbl2* __restrict__ p, size_t n2, double* o) {
    double s = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) {
        dbl2 a = r[i], b = p[i];
        s += a[0] + a[1] + b[0] + b[1];
    }
    if (s == 1.2345) o[0] = s;
}

int main() {
    const size_t N = 640ull * 480 * 32;
    const size_t sizes[2] = {N, 4 * N};
    for (size_t n : sizes) {
        double *r, *p, *o;
        if (hipMalloc(&r, n * 8) || hipMalloc(&p, n * 8) || hipMalloc(&o, 64)) return 1;
        (void)hipMemset(r, 0, n * 8);
        (void)hipMemset(p, 0, n * 8);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        const int grids[3] = {1024, 2048, 8192};
        for (int gi = 0; gi < 3; ++gi) {
            const int G = grids[gi];
            auto run = [&](const char* name, auto launch, double bytes) {
                float best = 1e9;
                for (int rep = 0; rep < 20; ++rep) {
                    (void)hipEventRecord(e0);
                    launch();
                    (void)hipEventRecord(e1);
                    (void)hipEventSynchronize(e1);
                    float t;
                    (void)hipEventElapsedTime(&t, e0, e1);
                    if (t < best) best = t;
                }
                printf("n=%zu MB/array grid=%d %-28s %8.1f us  %7.1f GB/s\n", n * 8 >> 20, G, name, best * 1e3,
                       bytes / best / 1e6);
            };
            const double rw = 4.0 * n * 8;
            run("16B ld / 16B st", [&] { k<0><<<G, 256>>>(r, p, n, 0.5, 0.25); }, rw);
            run("16B ld / 8B st", [&] { k<1><<<G, 256>>>(r, p, n, 0.5, 0.25); }, rw);
            run("16B ld / nt 16B st", [&] { k<2><<<G, 256>>>(r, p, n, 0.5, 0.25); }, rw);
            run("nt ld / nt st", [&] { k<3><<<G, 256>>>(r, p, n, 0.5, 0.25); }, rw);
            run("8B ld / 8B st", [&] { k<4><<<G, 256>>>(r, p, n, 0.5, 0.25); }, rw);
            run("read only 16B", [&] { rdonly<<<G, 256>>>((const dbl2*)r, (const dbl2*)p, n / 2, o); }, 2.0 * n * 8);
        }
        (void)hipFree(r);
        (void)hipFree(p);
        (void)hipFree(o);
    }
    return 0;
}
