// libfoto C ABI: per-operator entry points (operators.py matvecs, stepB, RHS, flow
// extraction) and the GN solver (classical.GLLOpticalFlow.process).  Every call copies
// the caller's host buffers to the current device, runs the kernels on a private stream
// and copies the result back; device scratch lives only for the call.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>

#include "foto_internal.h"

using namespace foto;

namespace {

struct Scope {   // one call's stream + device allocations
    hipStream_t s = nullptr;
    std::vector<void*> bufs;
    int init() { return stream_acquire(&s); }
    int dev(size_t n_doubles, double** out) {
        void* p = nullptr;
        FOTO_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n_doubles, 1) * sizeof(double)));
        bufs.push_back(p);
        *out = (double*)p;
        return 0;
    }
    int up(const double* h, size_t n, double** out) {
        FOTO_TRY(dev(n, out));
        FOTO_HIP_CHECK(hipMemcpyAsync(*out, h, n * sizeof(double), hipMemcpyHostToDevice, s));
        return 0;
    }
    int down(double* h, const double* d, size_t n) {
        FOTO_HIP_CHECK(hipMemcpyAsync(h, d, n * sizeof(double), hipMemcpyDeviceToHost, s));
        return 0;
    }
    int sync() {
        FOTO_HIP_CHECK(hipStreamSynchronize(s));
        return 0;
    }
    ~Scope() {
        if (s) (void)hipStreamSynchronize(s);
        for (void* p : bufs) (void)hipFree(p);
        stream_release(s);
    }
};

Geo make_geo(int Nt, int Nx, int Ny) {
    Geo g;
    g.Nt = Nt; g.Ny = Ny; g.Nx = Nx; g.t0 = 0; g.nloc = Nt; g.nxy = (int64_t)Nx * Ny;
    return g;
}

int check3(int Nt, int Nx, int Ny) {
    if (Nt < 2 || Nx < 2 || Ny < 2) {
        set_error("grid (Nt=%d, Nx=%d, Ny=%d): every axis needs >= 2 points (reference raises IndexError)", Nt, Nx, Ny);
        return FOTO_ERR_ARG;
    }
    return 0;
}

int check2(int Nx, int Ny) {
    if (Nx < 2 || Ny < 2) {
        set_error("image %dx%d: every axis needs >= 2 points", Nx, Ny);
        return FOTO_ERR_ARG;
    }
    if ((int64_t)Nx * Ny >= ((int64_t)1 << 31)) {   // pixel indices are 32-bit in the kernels
        set_error("image %dx%d: more than 2^31 pixels", Nx, Ny);
        return FOTO_ERR_ARG;
    }
    return 0;
}

int bc_flag(char bc, int* bcD) {
    if (bc == 'N' || bc == 'n') { *bcD = 0; return 0; }
    if (bc == 'D' || bc == 'd') { *bcD = 1; return 0; }
    set_error("These boundary conditions are not implemented");   // operators.py:6-7
    return FOTO_ERR_BC;
}

}  // namespace

extern "C" {

int foto_grad_st(const double* phi, int Nt, int Nx, int Ny, double* out3) {
    FOTO_TRY(check3(Nt, Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const Geo g = make_geo(Nt, Nx, Ny);
    const size_t N = (size_t)Nt * g.nxy;
    double *d, *o;
    FOTO_TRY(S.up(phi, N, &d));
    FOTO_TRY(S.dev(3 * N, &o));
    FOTO_HIP_CHECK(launch_grad_st(g, d, o, o + N, o + 2 * N, S.s));
    FOTO_TRY(S.down(out3, o, 3 * N));
    return S.sync();
}

int foto_div_st(const double* w3, int Nt, int Nx, int Ny, double* out) {
    FOTO_TRY(check3(Nt, Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const Geo g = make_geo(Nt, Nx, Ny);
    const size_t N = (size_t)Nt * g.nxy;
    double *d, *o;
    FOTO_TRY(S.up(w3, 3 * N, &d));
    FOTO_TRY(S.dev(N, &o));
    FOTO_HIP_CHECK(launch_div_st(g, d, d + N, d + 2 * N, o, S.s));
    FOTO_TRY(S.down(out, o, N));
    return S.sync();
}

static int apply_common(const double* p, int Nt, int Nx, int Ny, double r, double eps, int lap, double* out) {
    FOTO_TRY(check3(Nt, Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const Geo g = make_geo(Nt, Nx, Ny);
    const size_t N = (size_t)Nt * g.nxy;
    double *d, *o;
    FOTO_TRY(S.up(p, N, &d));
    FOTO_TRY(S.dev(N, &o));
    FOTO_HIP_CHECK(launch_apply_A(g, d, o, r, eps, lap, S.s));
    FOTO_TRY(S.down(out, o, N));
    return S.sync();
}

int foto_laplacian_st(const double* p, int Nt, int Nx, int Ny, double* out) {
    return apply_common(p, Nt, Nx, Ny, 1.0, 0.0, 1, out);
}

int foto_apply_A(const double* p, int Nt, int Nx, int Ny, double r, double eps, double* out) {
    return apply_common(p, Nt, Nx, Ny, r, eps, 0, out);
}

int foto_grad2(const double* f, int Nx, int Ny, char bc, double* out2) {
    int bcD;
    FOTO_TRY(bc_flag(bc, &bcD));
    FOTO_TRY(check2(Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const size_t n = (size_t)Nx * Ny;
    double *d, *o;
    FOTO_TRY(S.up(f, n, &d));
    FOTO_TRY(S.dev(2 * n, &o));
    FOTO_HIP_CHECK(launch_grad2(Nx, Ny, d, o, o + n, bcD, S.s));
    FOTO_TRY(S.down(out2, o, 2 * n));
    return S.sync();
}

int foto_div2(const double* uv, int Nx, int Ny, char bc, double* out) {
    int bcD;
    FOTO_TRY(bc_flag(bc, &bcD));
    FOTO_TRY(check2(Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const size_t n = (size_t)Nx * Ny;
    double *d, *o;
    FOTO_TRY(S.up(uv, 2 * n, &d));
    FOTO_TRY(S.dev(n, &o));
    FOTO_HIP_CHECK(launch_div2(Nx, Ny, d, d + n, o, bcD, 1.0, S.s));
    FOTO_TRY(S.down(out, o, n));
    return S.sync();
}

int foto_grad2_forward(const double* f, int Nx, int Ny, double* out2) {
    FOTO_TRY(check2(Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const size_t n = (size_t)Nx * Ny;
    double *d, *o;
    FOTO_TRY(S.up(f, n, &d));
    FOTO_TRY(S.dev(2 * n, &o));
    FOTO_HIP_CHECK(launch_grad2_forward(Nx, Ny, d, o, o + n, S.s));
    FOTO_TRY(S.down(out2, o, 2 * n));
    return S.sync();
}

int foto_stepB(const double* p3, int64_t M, double* q3) {
    if (M < 0 || !p3 || !q3) { set_error("bad stepB arguments"); return FOTO_ERR_ARG; }
    if (M == 0) return 0;
    Scope S;
    FOTO_TRY(S.init());
    double *d, *o;
    FOTO_TRY(S.up(p3, 3 * (size_t)M, &d));
    FOTO_TRY(S.dev(3 * (size_t)M, &o));
    FOTO_HIP_CHECK(launch_stepB(M, d, d + M, d + 2 * M, o, o + M, o + 2 * M, S.s));
    FOTO_TRY(S.down(q3, o, 3 * (size_t)M));
    return S.sync();
}

int foto_bb_rhs(const double* mu3, const double* q3, const double* rho0, const double* rhoT, int Nt, int Nx, int Ny,
                double r, double* F) {
    FOTO_TRY(check3(Nt, Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const Geo g = make_geo(Nt, Nx, Ny);
    const size_t N = (size_t)Nt * g.nxy;
    double *mu, *q, *r0, *rT, *o, *part, *gath;
    FOTO_TRY(S.up(mu3, 3 * N, &mu));
    FOTO_TRY(S.up(q3, 3 * N, &q));
    FOTO_TRY(S.up(rho0, g.nxy, &r0));
    FOTO_TRY(S.up(rhoT, g.nxy, &rT));
    FOTO_TRY(S.dev(N, &o));
    const int nb = flat_blocks((int64_t)N);
    FOTO_TRY(S.dev(nb + 8, &part));
    FOTO_TRY(S.dev(8, &gath));
    FOTO_HIP_CHECK(hipMemsetAsync(part + nb, 0, 8 * sizeof(double), S.s));
    RedBuf rb{part, (unsigned*)(part + nb), nb};
    FOTO_HIP_CHECK(launch_rhs(g, mu, mu + N, mu + 2 * N, q, q + N, q + 2 * N, r0, rT, r, o, rb, gath, 0, S.s));
    FOTO_TRY(S.down(F, o, N));
    return S.sync();
}

int foto_flow_from_phi(const double* phi, int Nt, int Nx, int Ny, double* u, double* v, double* m) {
    FOTO_TRY(check3(Nt, Nx, Ny));
    Scope S;
    FOTO_TRY(S.init());
    const Geo g = make_geo(Nt, Nx, Ny);
    const size_t N = (size_t)Nt * g.nxy, n = (size_t)g.nxy;
    double *d, *px, *py, *du, *dv, *dm;
    FOTO_TRY(S.up(phi, N, &d));
    FOTO_TRY(S.dev(n, &px));
    FOTO_TRY(S.dev(n, &py));
    FOTO_TRY(S.dev(n, &du));
    FOTO_TRY(S.dev(n, &dv));
    FOTO_TRY(S.dev(n, &dm));
    FOTO_HIP_CHECK(launch_traj(g, d, 0, Nt - 1, px, py, 1, S.s));
    FOTO_HIP_CHECK(launch_flow_finish(Nx, Ny, px, py, du, dv, dm, S.s));
    FOTO_TRY(S.down(u, du, n));
    FOTO_TRY(S.down(v, dv, n));
    FOTO_TRY(S.down(m, dm, n));
    return S.sync();
}

// ----------------------------------------------------------------------------- GN

int foto_gn_apply(const double* f1, const double* f2, int w, int h, double alpha, double lam, const double* x3,
                  double* y3) {
    FOTO_TRY(check2(w, h));
    Scope S;
    FOTO_TRY(S.init());
    const size_t n = (size_t)w * h;
    double *d1, *d2, *fx, *fy, *ft, *x, *y;
    FOTO_TRY(S.up(f1, n, &d1));
    FOTO_TRY(S.up(f2, n, &d2));
    FOTO_TRY(S.up(x3, 3 * n, &x));
    FOTO_TRY(S.dev(n, &fx));
    FOTO_TRY(S.dev(n, &fy));
    FOTO_TRY(S.dev(n, &ft));
    FOTO_TRY(S.dev(3 * n, &y));
    FOTO_HIP_CHECK(launch_gn_coeffs(w, h, d1, d2, fx, fy, ft, S.s));
    FOTO_HIP_CHECK(launch_gn_apply(w, h, fx, fy, d2, alpha, lam, x, y, S.s));
    FOTO_TRY(S.down(y3, y, 3 * n));
    return S.sync();
}

int foto_gn_rhs(const double* f1, const double* f2, int w, int h, double* b3) {
    FOTO_TRY(check2(w, h));
    Scope S;
    FOTO_TRY(S.init());
    const size_t n = (size_t)w * h;
    double *d1, *d2, *fx, *fy, *ft, *b;
    FOTO_TRY(S.up(f1, n, &d1));
    FOTO_TRY(S.up(f2, n, &d2));
    FOTO_TRY(S.dev(n, &fx));
    FOTO_TRY(S.dev(n, &fy));
    FOTO_TRY(S.dev(n, &ft));
    FOTO_TRY(S.dev(3 * n, &b));
    FOTO_HIP_CHECK(launch_gn_coeffs(w, h, d1, d2, fx, fy, ft, S.s));
    FOTO_HIP_CHECK(launch_gn_rhs(w, h, fx, fy, d2, ft, b, S.s));
    FOTO_TRY(S.down(b3, b, 3 * n));
    return S.sync();
}

// classical.GLLOpticalFlow.process: PCG to rtol on the assembled-equivalent operator.
// Device-resident loop; the host polls the done flag between chunks of iterations.
static int gn_solve_impl(const double* f1, const double* f2, int w, int h, double alpha, double lam, double rtol,
                         int maxiter, double* u, double* v, double* m, int* iterations, foto_gn_stats* st);

int foto_gn_solve(const double* f1, const double* f2, int w, int h, double alpha, double lam, double rtol,
                  int maxiter, double* u, double* v, double* m, int* iterations) {
    return gn_solve_impl(f1, f2, w, h, alpha, lam, rtol, maxiter, u, v, m, iterations, nullptr);
}

// Algorithmic HBM bytes of one MG-PCG iteration (bench.py gn_bytes_per_iteration):
// k_gnp_dir 12 n, k_gnp_upd 18 n, per level k_mg_down2 18 n_l + 3 n_l+1 and k_mg_up2 21 n_l + 3 n_l+1
// (level 0: 9 n_0 and 12 n_0, its B and D^-1 formed from fx, fy, f2; FOTO_GN_RECOMP=0 loads them
// and moves more than this counts), the coarsest level 18 n_c fp64 values; levels halve (rounding
// up) until <= 1024 cells.
static double gn_alg_bytes(int w, int h, int* levels) {
    std::vector<double> ns{(double)w * h};
    while ((double)w * h > 1024) {
        w = (w + 1) / 2;
        h = (h + 1) / 2;
        ns.push_back((double)w * h);
    }
    double v = 30.0 * ns[0];
    for (size_t l = 0; l + 1 < ns.size(); ++l) v += (l == 0 ? 21.0 : 39.0) * ns[l] + 6.0 * ns[l + 1];
    v += 18.0 * ns.back();
    if (levels) *levels = (int)ns.size();
    return 8.0 * v;
}

int foto_gn_solve_ex(const double* f1, const double* f2, int w, int h, double alpha, double lam, double rtol,
                     int maxiter, double* u, double* v, double* m, foto_gn_stats* st) {
    int its = 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (st) memset(st, 0, sizeof(*st));
    const int rc = gn_solve_impl(f1, f2, w, h, alpha, lam, rtol, maxiter, u, v, m, &its, st);
    if (rc >= 0 && st) {
        st->iterations = its;
        st->info = rc;
        st->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return rc;
}

static int gn_solve_impl(const double* f1, const double* f2, int w, int h, double alpha, double lam, double rtol,
                         int maxiter, double* u, double* v, double* m, int* iterations, foto_gn_stats* st) {
    FOTO_TRY(check2(w, h));
    if (!(alpha > 0) || !(lam > 0)) {
        set_error("GN needs alpha > 0 and lambda > 0 (the block-Jacobi preconditioner divides by them)");
        return FOTO_ERR_ARG;
    }
    if (maxiter < 0) { set_error("maxiter < 0"); return FOTO_ERR_ARG; }
    const char* emg = getenv("FOTO_GN_MG");   // 0: 3x3 block-Jacobi preconditioner (A/B runs)
    if (!(emg && atoi(emg) == 0)) {
        // multigrid-preconditioned CG through a plan (foto_gn.hip), cached per process like an
        // FFT plan: a call with the same (w, h, alpha, lambda, rtol, maxiter) as the previous
        // one reuses its buffers and graph (FOTO_GN_PLAN_CACHE=0: make and destroy a plan per call)
        const char* ec = getenv("FOTO_GN_PLAN_CACHE");
        const bool cache = !(ec && atoi(ec) == 0);
        // (the cached plan is never destroyed at process exit: the HIP runtime may be gone by then)
        static std::mutex mu;
        static foto_gn_plan* cached = nullptr;
        static double key[6] = {0, 0, 0, 0, 0, 0};
        const double k6[6] = {(double)w, (double)h, alpha, lam, rtol, (double)maxiter};
        std::lock_guard<std::mutex> lk(mu);
        int dev = 0;
        FOTO_HIP_CHECK(hipGetDevice(&dev));
        const bool reused = !(!cache || !cached || memcmp(key, k6, sizeof(k6)) != 0 || foto_gn_plan_device(cached) != dev);
        if (!reused) {
            foto_gn_plan_destroy(cached);
            cached = nullptr;
            FOTO_TRY(foto_gn_plan_create(w, h, alpha, lam, rtol, maxiter, &cached));
            memcpy(key, k6, sizeof(k6));
        }
        const int rc = foto_gn_plan_solve(cached, f1, f2, u, v, m, iterations);
        if (st && rc >= 0) {
            // (no early return here: the plan below must still be destroyed when caching is off,
            // and a timing readback cannot turn a finished solve into an error)
            double t4[4] = {0, 0, 0, 0};
            if (foto_gn_plan_timing(cached, t4) < 0) t4[0] = t4[1] = -1.0;
            st->ms_setup = t4[0];
            st->ms_pcg = t4[1];
            st->plan_reused = reused ? 1 : 0;
            st->alg_bytes_per_iter = gn_alg_bytes(w, h, &st->levels);
        }
        if (!cache || rc < 0) {
            foto_gn_plan_destroy(cached);
            cached = nullptr;
        }
        return rc;
    }
    // 3x3 block-Jacobi PCG (the first GPU version; kept for A/B runs)
    Scope S;
    FOTO_TRY(S.init());
    const size_t n = (size_t)w * h;
    double *d1, *d2, *fx, *fy, *ft, *b, *x, *r, *z, *p0, *p1, *part, *gath, *scal;
    const int nb = flat_blocks((int64_t)n);
    {   // one allocation (a solve is ~15 ms; per-buffer hipMalloc/hipFree added up to ~1 ms)
        const size_t nscal = sizeof(CGScal) / sizeof(double) + 1;
        double* base;
        FOTO_TRY(S.dev(23 * n + 2 * (size_t)nb + 8 + 8 + nscal, &base));
        d1 = base; fx = base + 2 * n; fy = fx + n; ft = fy + n;
        d2 = base + n;
        b = ft + n; x = b + 3 * n; r = x + 3 * n; z = r + 3 * n; p0 = z + 3 * n; p1 = p0 + 3 * n;
        part = p1 + 3 * n; gath = part + 2 * (size_t)nb + 8; scal = gath + 8;
        FOTO_HIP_CHECK(hipMemcpyAsync(d1, f1, n * sizeof(double), hipMemcpyHostToDevice, S.s));
        FOTO_HIP_CHECK(hipMemcpyAsync(d2, f2, n * sizeof(double), hipMemcpyHostToDevice, S.s));
    }
    CGScal* dS = (CGScal*)scal;
    FOTO_HIP_CHECK(hipMemsetAsync(part + 2 * nb, 0, 8 * sizeof(double), S.s));
    FOTO_HIP_CHECK(hipMemsetAsync(dS, 0, sizeof(CGScal), S.s));
    FOTO_HIP_CHECK(hipMemsetAsync(x, 0, 3 * n * sizeof(double), S.s));
    RedBuf rb{part, (unsigned*)(part + 2 * nb), 2 * nb};
    double* g_rz = gath;       // {r.r, r.z}
    double* g_pq = gath + 2;   // {p.q}
    FOTO_HIP_CHECK(launch_gn_coeffs(w, h, d1, d2, fx, fy, ft, S.s));
    FOTO_HIP_CHECK(launch_gn_rhs(w, h, fx, fy, d2, ft, b, S.s));
    FOTO_HIP_CHECK(launch_gn_pcg_init(w, h, fx, fy, d2, alpha, lam, b, r, z, rb, g_rz, S.s));
    CGScal* hS = nullptr;
    FOTO_HIP_CHECK(hipHostMalloc((void**)&hS, sizeof(CGScal)));
    std::unique_ptr<CGScal, void (*)(CGScal*)> hguard(hS, [](CGScal* p) { (void)hipHostFree(p); });
    int k = 0;
    bool done = false;
    {
        while (k < maxiter) {
            const int chunk = std::min(k == 0 ? 64 : 32, maxiter - k);
            for (int j = 0; j < chunk; ++j, ++k) {
                double* po = (k & 1) ? p1 : p0;
                double* pn = (k & 1) ? p0 : p1;
                FOTO_HIP_CHECK(launch_gn_pcg_dir(w, h, k, fx, fy, d2, alpha, lam, z, po, pn, dS, rb, g_rz, g_pq, rtol,
                                                 S.s));
                FOTO_HIP_CHECK(launch_gn_pcg_upd(w, h, k, fx, fy, d2, alpha, lam, pn, x, r, z, dS, rb, g_pq, g_rz,
                                                 S.s));
            }
            FOTO_HIP_CHECK(hipMemcpyAsync(hS, dS, sizeof(CGScal), hipMemcpyDeviceToHost, S.s));
            FOTO_TRY(S.sync());
            if (hS->done) { done = true; break; }
        }
    }
    FOTO_TRY(S.down(u, x, n));
    FOTO_TRY(S.down(v, x + n, n));
    FOTO_TRY(S.down(m, x + 2 * n, n));
    FOTO_TRY(S.sync());
    if (iterations) *iterations = done ? hS->iters : maxiter;
    if (st) {   // (no plan, no multigrid: 3 fields of 10 + 3 coefficient + 6 block-inverse values)
        st->levels = 0;
        st->alg_bytes_per_iter = 8.0 * (double)n * (3 * 10 + 3 + 6);
    }
    return done ? 0 : maxiter;
}

}  // extern "C"
