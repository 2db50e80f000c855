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


// ---- ablation of the spectral s-step pass: tile loop (4 rows x 128 cols, 2 elements per
// lane), lam from three small tables, two CG steps, optional 12 Chebyshev moments.
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
    {   // spectral pass ablation at the bench grid
        const int Nt = 32, Ny = 480, Nx = 640;
        const size_t n = (size_t)Nt * Ny * Nx;
        double *r, *p, *o, *mt, *my, *mx;
        if (hipMalloc(&r, n * 8) || hipMalloc(&p, n * 8) || hipMalloc(&o, 64) || hipMalloc(&mt, 8 * Nt) ||
            hipMalloc(&my, 8 * Ny) || hipMalloc(&mx, 8 * Nx)) return 1;
        (void)hipMemset(r, 0, n * 8); (void)hipMemset(p, 0, n * 8);
        (void)hipMemset(mt, 0, 8 * Nt); (void)hipMemset(my, 0, 8 * Ny); (void)hipMemset(mx, 0, 8 * Nx);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        const int grids[4] = {512, 1024, 2048, 4096};
        for (int gi = 0; gi < 4; ++gi) {
            for (int mom = 0; mom < 2; ++mom) {
                float best = 1e9;
                for (int rep = 0; rep < 20; ++rep) {
                    (void)hipEventRecord(e0);
                    if (mom) spass<1><<<grids[gi], 256>>>(r, p, mt, my, mx, Nt, Ny, Nx, 0.1, 0.2, 0.3, 0.4, o);
                    else spass<0><<<grids[gi], 256>>>(r, p, mt, my, mx, Nt, Ny, Nx, 0.1, 0.2, 0.3, 0.4, o);
                    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
                    float t; (void)hipEventElapsedTime(&t, e0, e1);
                    if (t < best) best = t;
                }
                printf("spass grid=%d moments=%d %8.1f us  %7.1f GB/s\n", grids[gi], mom, best * 1e3, 4.0 * n * 8 / best / 1e6);
            }
        }
    }
    return 0;
}
