// Probe of gfx950's v_permlane16_swap / v_permlane32_swap as xor-16 / xor-32 lane exchanges
// (the builtins return {vdst, src0} after the swap): prints, for a few lanes, the value the
// exchange delivers and the lane it should come from.
//   hipcc --offload-arch=gfx950 -O3 permlane_probe.hip -o permlane_probe
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
    const unsigned l = threadIdx.x;
    const unsigned x = 1000 + l;
    auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    out[l] = (l & 16) ? a[0] : a[1];
    out[64 + l] = (l & 32) ? b[0] : b[1];
}
int main() {
    unsigned* d;
    unsigned h[128];
    if (hipMalloc(&d, sizeof h) != hipSuccess) return 1;
    k<<<1, 64>>>(d);
    if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        bad += h[l] != 1000u + (l ^ 16);
        bad += h[64 + l] != 1000u + (l ^ 32);
    }
    printf("lane 5: x16 %u x32 %u; lane 50: x16 %u x32 %u; mismatches %d\n", h[5], h[64 + 5], h[50], h[64 + 50], bad);
    return bad ? 3 : 0;
}
