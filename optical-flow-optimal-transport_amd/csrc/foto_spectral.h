// Spectral (DCT-II basis) CG for A = -r L_st + r eps I.  See foto_spectral.hip.
#pragma once
#include "foto_internal.h"

namespace foto {

struct KTimer;

struct SpectralPlan {
    int init(const Geo& g, int world, double r, double eps, int sstep, hipStream_t s);
    // b (physical, overwritten as scratch) -> x (physical); scipy stopping rule.
    int solve(double* b, double* x, double rtol, int maxiter, int predicted, int* iters, int* info, KTimer* kt,
              hipStream_t s);
    ~SpectralPlan();
    void* impl = nullptr;
};

}  // namespace foto
