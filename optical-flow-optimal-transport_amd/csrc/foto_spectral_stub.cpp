#include "foto_spectral.h"
namespace foto {
int SpectralPlan::init(const Geo&, int, double, double, hipStream_t) {
    set_error("spectral CG not built");
    return FOTO_ERR_ARG;
}
int SpectralPlan::solve(double*, double*, double, int, int, int*, int*, KTimer*, hipStream_t) { return FOTO_ERR_ARG; }
SpectralPlan::~SpectralPlan() {}
}  // namespace foto
