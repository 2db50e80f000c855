"""foto -- MI355X-native FOTO hot path (Benamou-Brenier optical flow + GN baseline).

Python host code over libfoto.so (hand-written HIP for gfx950, RCCL for time-slab
sharding) through a C ABI (include/foto.h).  No PyTorch on the product path.
"""
from ._lib import FotoError, lib, device_count  # noqa: F401
from . import ops, bb, gn, synthetic  # noqa: F401
from .bb import BBSolver, solve, CG_STENCIL, CG_SPECTRAL, CG_SSTEP, CG_GAUSS  # noqa: F401

__all__ = ["FotoError", "lib", "device_count", "ops", "bb", "gn", "synthetic", "BBSolver", "solve",
           "CG_STENCIL", "CG_SPECTRAL", "CG_SSTEP", "CG_GAUSS"]
