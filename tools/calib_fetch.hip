// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access widths libfoto uses:
// streams a 2 GiB buffer (far beyond the 256 MiB Infinity Cache) with 8-B and 16-B loads
// per lane, and writes 1 GiB with 8-B and 16-B stores.  Known byte counts; compare with
// rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE to get the per-width correction factor.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl2 __attribute__((ext_vector_type(2)));
__global__ void rd8(const double* a, size_t n, double* o) {
    double s = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    if (s == 12345.678) o[0] = s;
}
__global__ void rd16(const dbl2* a, size_t n2, double* o) {
    double s = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) { dbl2 v = a[i]; s += v[0] + v[1]; }
    if (s == 12345.678) o[0] = s;
}
__global__ void wr8(double* a, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (double)i;
}
__global__ void wr16(dbl2* a, size_t n2) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n2; i += (size_t)gridDim.x * 256) a[i] = dbl2{(double)i, 1.0};
}
int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 8;
    double *a, *o;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    hipMemset(a, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
        float t;
        hipEventRecord(e0); rd8<<<4096, 256>>>(a, n, o); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&t, e0, e1); printf("rd8  %zu MiB  %.3f ms  %.1f GB/s\n", bytes >> 20, t, bytes / t / 1e6);
        hipEventRecord(e0); rd16<<<4096, 256>>>((const dbl2*)a, n / 2, o); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&t, e0, e1); printf("rd16 %zu MiB  %.3f ms  %.1f GB/s\n", bytes >> 20, t, bytes / t / 1e6);
        hipEventRecord(e0); wr8<<<4096, 256>>>(a, n / 2); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&t, e0, e1); printf("wr8  %zu MiB  %.3f ms  %.1f GB/s\n", bytes >> 21, t, bytes / 2 / t / 1e6);
        hipEventRecord(e0); wr16<<<4096, 256>>>((dbl2*)a, n / 4); hipEventRecord(e1); hipEventSynchronize(e1);
        hipEventElapsedTime(&t, e0, e1); printf("wr16 %zu MiB  %.3f ms  %.1f GB/s\n", bytes >> 21, t, bytes / 2 / t / 1e6);
    }
    hipDeviceSynchronize();
    return 0;
}
