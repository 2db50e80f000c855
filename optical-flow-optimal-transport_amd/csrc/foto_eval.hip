// Evaluation kernels: the backward warp utils.apply_opticalflow
// (utils.py:186-248) and the flow / intensity error metrics utils.EE / AE / IE
// (utils.py:294-354), behind the C ABI (include/foto.h).
//
// The warp is per pixel in the reference's operation order (built with -ffp-contract=off):
// bit-identical to the reference.  The metrics are two-pass masked sums (mean, then the
// squared deviations) with fixed-order tree reductions: deterministic, and equal to the
// reference's np.sum up to summation order (~1e-16 relative).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <vector>

#include "foto_internal.h"


namespace foto {

constexpr int EV_NT = 256;
constexpr int EV_Q = 6;   // quantities per block partial

__global__ __launch_bounds__(EV_NT) void k_warp(const double* __restrict__ f1, const double* __restrict__ m,
                                                const double* __restrict__ u, const double* __restrict__ v, int w,
                                                int h, double* __restrict__ out) {
    const int64_t n = (int64_t)w * h;
    for (int64_t p = (int64_t)blockIdx.x * EV_NT + threadIdx.x; p < n; p += (int64_t)gridDim.x * EV_NT) {
        const int i = (int)(p / w), j = (int)(p - (p / w) * w);   // row, column
        double ti = (double)i - v[p], tj = (double)j - u[p];
        const double dI = ti - trunc(ti), dJ = tj - trunc(tj);
        const double w1 = (1 - dI) * (1 - dJ), w2 = dJ * (1 - dI), w3 = dI * dJ, w4 = (1 - dJ) * dI;
        if (ti >= h) ti = h - 1;
        if (tj >= w) tj = w - 1;
        if (ti < 0) ti = 0;
        if (tj < 0) tj = 0;
        const int64_t a = (int64_t)ti, b = (int64_t)tj;
        const int64_t a1 = (a < h - 1) ? a + 1 : a, b1 = (b < w - 1) ? b + 1 : b;
        auto F = [&](int64_t q) { return m ? (1 + m[q]) * f1[q] : f1[q]; };   // (1 + m) f1
        double x = w1 * F(a * w + b);
        x = x + w2 * F(a * w + b1);
        x = x + w3 * F(a1 * w + b1);
        x = x + w4 * F(a1 * w + b);
        out[p] = x;
    }
}

__device__ __forceinline__ void ev_block_sum(double (&v)[EV_Q], double* sh /* EV_Q * EV_NT */) {
#pragma unroll
    for (int q = 0; q < EV_Q; ++q) sh[q * EV_NT + threadIdx.x] = v[q];
    __syncthreads();
    for (int st = EV_NT / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st)
#pragma unroll
            for (int q = 0; q < EV_Q; ++q) sh[q * EV_NT + threadIdx.x] += sh[q * EV_NT + threadIdx.x + st];
        __syncthreads();
    }
}

// pass 0: (sum EE | EE <= 50, count, sum AE | AE not NaN, count, sum (255 I - 255 IGT)^2, 0)
// pass 1: (sum (EE - mean_EE)^2 | kept, 0, sum (AE - mean_AE)^2 | kept, 0, 0, 0)
__global__ __launch_bounds__(EV_NT) void k_err_partial(int64_t n, const double* __restrict__ u,
                                                       const double* __restrict__ v, const double* __restrict__ uG,
                                                       const double* __restrict__ vG, const double* __restrict__ I,
                                                       const double* __restrict__ IG, int pass, double mee,
                                                       double mae, double* __restrict__ part) {
    __shared__ double sh[EV_Q * EV_NT];
    double acc[EV_Q] = {0, 0, 0, 0, 0, 0};
    for (int64_t p = (int64_t)blockIdx.x * EV_NT + threadIdx.x; p < n; p += (int64_t)gridDim.x * EV_NT) {
        if (u) {
            const double du = u[p] - uG[p], dv = v[p] - vG[p];
            const double e = sqrt(du * du + dv * dv);
            if (e <= 50) {
                if (pass == 0) { acc[0] += e; acc[1] += 1.0; }
                else acc[0] += (e - mee) * (e - mee);
            }
            const double a = acos((1.0 + u[p] * uG[p] + v[p] * vG[p]) /
                                  (sqrt(1.0 + u[p] * u[p] + v[p] * v[p]) * sqrt(1.0 + uG[p] * uG[p] + vG[p] * vG[p])));
            if (!isnan(a)) {
                if (pass == 0) { acc[2] += a; acc[3] += 1.0; }
                else acc[2] += (a - mae) * (a - mae);
            }
        }
        if (I && pass == 0) {
            const double d = 255 * I[p] - 255 * IG[p];
            acc[4] += d * d;
        }
    }
    ev_block_sum(acc, sh);
    if (threadIdx.x < EV_Q) part[(int64_t)blockIdx.x * EV_Q + threadIdx.x] = sh[threadIdx.x * EV_NT];
}

// sum of nb block partials per quantity (one block, fixed tree)
__global__ __launch_bounds__(EV_NT) void k_err_final(int nb, const double* __restrict__ part,
                                                     double* __restrict__ tot) {
    __shared__ double sh[EV_Q * EV_NT];
    double acc[EV_Q] = {0, 0, 0, 0, 0, 0};
    for (int b = threadIdx.x; b < nb; b += EV_NT)
#pragma unroll
        for (int q = 0; q < EV_Q; ++q) acc[q] += part[(int64_t)b * EV_Q + q];
    ev_block_sum(acc, sh);
    if (threadIdx.x < EV_Q) tot[threadIdx.x] = sh[threadIdx.x * EV_NT];
}

namespace {

// Device buffers of the evaluation calls: grow-only slots kept for the process (a batch worker
// evaluates every solve at one frame size; hipMalloc / hipFree per call synchronise the device
// and cost more than the kernels).  One call at a time holds them.
constexpr int EV_SLOTS = 8;
struct EvSlots {
    void* p[EV_SLOTS] = {};
    size_t cap[EV_SLOTS] = {};
};
std::mutex ev_mu;
std::vector<EvSlots> ev_dev;   // per device (a slot is only valid on the device it was made on)

struct EvScope {
    hipStream_t s = nullptr;
    std::unique_lock<std::mutex> lk{ev_mu};
    EvSlots* sl = nullptr;
    int used = 0;
    int init() {
        FOTO_TRY(stream_acquire(&s));
        const int dev = stream_device(s);
        if (dev < 0) {
            set_error("evaluation: stream without a device");
            return FOTO_ERR_STATE;
        }
        if ((int)ev_dev.size() <= dev) ev_dev.resize(dev + 1);
        sl = &ev_dev[dev];
        return 0;
    }
    int slot(size_t n, double** d) {
        const size_t bytes = std::max<size_t>(n, 1) * sizeof(double);
        if (used >= EV_SLOTS) {
            set_error("evaluation: out of scratch slots");
            return FOTO_ERR_STATE;
        }
        if (sl->cap[used] < bytes) {
            if (sl->p[used]) {
                FOTO_HIP_CHECK(hipStreamSynchronize(s));
                FOTO_HIP_CHECK(hipFree(sl->p[used]));
                sl->p[used] = nullptr;
                sl->cap[used] = 0;
            }
            FOTO_HIP_CHECK(hipMalloc(&sl->p[used], bytes));
            sl->cap[used] = bytes;
        }
        *d = (double*)sl->p[used++];
        return 0;
    }
    int up(const double* h, size_t n, double** d) {
        if (!h) { *d = nullptr; return 0; }
        FOTO_TRY(slot(n, d));
        FOTO_HIP_CHECK(hipMemcpyAsync(*d, h, n * sizeof(double), hipMemcpyHostToDevice, s));
        return 0;
    }
    int dev(size_t n, double** d) { return slot(n, d); }
    ~EvScope() {
        if (s) (void)hipStreamSynchronize(s);
        stream_release(s);
    }
};

int ev_blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + EV_NT - 1) / EV_NT, 2048)); }

// the two passes; out: mean EE, std EE, mean AE, std AE, IE (any of the inputs may be absent)
int ev_errors(const double* u, const double* v, const double* uG, const double* vG, const double* I,
              const double* IG, int w, int h, double* out5) {
    if (w < 1 || h < 1) {
        set_error("flow errors: w, h must be >= 1");
        return FOTO_ERR_ARG;
    }
    const int64_t n = (int64_t)w * h;
    EvScope S;
    FOTO_TRY(S.init());
    double *du, *dv, *duG, *dvG, *dI, *dIG, *part, *tot;
    FOTO_TRY(S.up(u, n, &du));
    FOTO_TRY(S.up(v, n, &dv));
    FOTO_TRY(S.up(uG, n, &duG));
    FOTO_TRY(S.up(vG, n, &dvG));
    FOTO_TRY(S.up(I, n, &dI));
    FOTO_TRY(S.up(IG, n, &dIG));
    const int nb = ev_blocks(n);
    FOTO_TRY(S.dev((size_t)nb * EV_Q, &part));
    FOTO_TRY(S.dev(EV_Q, &tot));
    double h0[EV_Q], h1[EV_Q];
    k_err_partial<<<nb, EV_NT, 0, S.s>>>(n, du, dv, duG, dvG, dI, dIG, 0, 0.0, 0.0, part);
    k_err_final<<<1, EV_NT, 0, S.s>>>(nb, part, tot);
    FOTO_HIP_CHECK(hipGetLastError());
    FOTO_HIP_CHECK(hipMemcpyAsync(h0, tot, sizeof(h0), hipMemcpyDeviceToHost, S.s));
    FOTO_HIP_CHECK(hipStreamSynchronize(S.s));
    const double mee = h0[0] / h0[1], mae = h0[2] / h0[3];
    if (du) {
        k_err_partial<<<nb, EV_NT, 0, S.s>>>(n, du, dv, duG, dvG, nullptr, nullptr, 1, mee, mae, part);
        k_err_final<<<1, EV_NT, 0, S.s>>>(nb, part, tot);
        FOTO_HIP_CHECK(hipGetLastError());
        FOTO_HIP_CHECK(hipMemcpyAsync(h1, tot, sizeof(h1), hipMemcpyDeviceToHost, S.s));
        FOTO_HIP_CHECK(hipStreamSynchronize(S.s));
        out5[0] = mee;
        out5[1] = sqrt(h1[0] / h0[1]);
        out5[2] = mae;
        out5[3] = sqrt(h1[2] / h0[3]);
    }
    if (dI) out5[4] = sqrt(h0[4] / ((double)w * h));
    return 0;
}

}  // namespace
}  // namespace foto

using namespace foto;

extern "C" {

int foto_warp(const double* f1, const double* u, const double* v, const double* m, int w, int h, double* out) {
    if (!f1 || !u || !v || !out || w < 1 || h < 1) {
        set_error("foto_warp: null buffer or w, h < 1");
        return FOTO_ERR_ARG;
    }
    const int64_t n = (int64_t)w * h;
    EvScope S;
    FOTO_TRY(S.init());
    double *df, *dm, *du, *dv, *dout;
    FOTO_TRY(S.up(f1, n, &df));
    FOTO_TRY(S.up(m, n, &dm));
    FOTO_TRY(S.up(u, n, &du));
    FOTO_TRY(S.up(v, n, &dv));
    FOTO_TRY(S.dev(n, &dout));
    k_warp<<<ev_blocks(n), EV_NT, 0, S.s>>>(df, dm, du, dv, w, h, dout);
    FOTO_HIP_CHECK(hipGetLastError());
    FOTO_HIP_CHECK(hipMemcpyAsync(out, dout, n * sizeof(double), hipMemcpyDeviceToHost, S.s));
    FOTO_HIP_CHECK(hipStreamSynchronize(S.s));
    return 0;
}

int foto_flow_errors(const double* u, const double* v, const double* uGT, const double* vGT, int w, int h,
                     double* out4) {
    if (!u || !v || !uGT || !vGT || !out4) {
        set_error("foto_flow_errors: null buffer");
        return FOTO_ERR_ARG;
    }
    double r[5];
    FOTO_TRY(ev_errors(u, v, uGT, vGT, nullptr, nullptr, w, h, r));
    for (int k = 0; k < 4; ++k) out4[k] = r[k];
    return 0;
}

int foto_intensity_error(const double* I, const double* IGT, int w, int h, double* ie) {
    if (!I || !IGT || !ie) {
        set_error("foto_intensity_error: null buffer");
        return FOTO_ERR_ARG;
    }
    double r[5];
    FOTO_TRY(ev_errors(nullptr, nullptr, nullptr, nullptr, I, IGT, w, h, r));
    *ie = r[4];
    return 0;
}

}  // extern "C"
