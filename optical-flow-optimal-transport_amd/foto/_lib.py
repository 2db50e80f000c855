"""ctypes binding of libfoto.so (the C ABI declared in include/foto.h).

This is the only place Python touches the native library.  There is no fallback: if
libfoto.so is missing or cannot be loaded, ``lib()`` raises, and every compute call that
fails on the device raises ``FotoError`` with the library's message.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FOTO_LIB", os.path.join(HERE, "libfoto.so"))

FOTO_ERR_ARG = -1
FOTO_ERR_HIP = -2
FOTO_ERR_COMM = -3
FOTO_ERR_STATE = -4
FOTO_ERR_BC = -5

K_CG_DIR, K_CG_UPD, K_RHS, K_PROX, K_SPEC, K_DCT, K_FLOW, K_SLAB = range(8)
K_OTHER = K_SLAB
# dct_slab: the sharded path's slab-side x / y DCTs (foto.h FOTO_K_SLAB), apart from "dct" (the
# box-side t axis, x^) so the scaling proxy sees what the pipelined all-to-alls overlap
K_NAMES = ["cg_dir", "cg_upd", "rhs", "prox", "spec_cg", "dct", "flow", "dct_slab"]


class FotoError(RuntimeError):
    pass


class BBOpts(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int),
        ("cg_maxiter", ctypes.c_int),
        ("cg_rtol", ctypes.c_double),
        ("cg_mode", ctypes.c_int),
        ("rank", ctypes.c_int),
        ("world", ctypes.c_int),
        ("nccl_id", ctypes.c_void_p),
        ("virtual_ranks", ctypes.c_int),
        ("timing", ctypes.c_int),
    ]


class BBStats(ctypes.Structure):
    _fields_ = [
        ("outer_iters", ctypes.c_int),
        ("cg_iters_total", ctypes.c_int64),
        ("last_crit", ctypes.c_double),
        ("ms_rhs", ctypes.c_double),
        ("ms_cg", ctypes.c_double),
        ("ms_prox", ctypes.c_double),
        ("ms_flow", ctypes.c_double),
        ("n_k", ctypes.c_int64 * 8),
        ("ms_k", ctypes.c_double * 8),
        ("bytes_k", ctypes.c_double * 8),
        ("cg_redo", ctypes.c_int),
    ]


class BBSolveStats(ctypes.Structure):
    """foto_bb_solve_stats (include/foto.h): the caller sizes crit / cg_its / cg_info by cap."""
    _fields_ = [
        ("cap", ctypes.c_int),
        ("crit", ctypes.POINTER(ctypes.c_double)),
        ("cg_its", ctypes.POINTER(ctypes.c_int)),
        ("cg_info", ctypes.POINTER(ctypes.c_int)),
        ("outer_iters", ctypes.c_int),
        ("stopped", ctypes.c_int),
        ("phi_t0", ctypes.c_int),
        ("phi_nloc", ctypes.c_int),
        ("ms_create", ctypes.c_double),
        ("ms_loop", ctypes.c_double),
        ("ms_flow", ctypes.c_double),
        ("alg_bytes_per_iter", ctypes.c_double),
        ("bb", BBStats),
    ]


class GNStats(ctypes.Structure):
    """foto_gn_stats (include/foto.h)."""
    _fields_ = [
        ("iterations", ctypes.c_int),
        ("info", ctypes.c_int),
        ("plan_reused", ctypes.c_int),
        ("levels", ctypes.c_int),
        ("ms_setup", ctypes.c_double),
        ("ms_pcg", ctypes.c_double),
        ("ms_total", ctypes.c_double),
        ("alg_bytes_per_iter", ctypes.c_double),
    ]


ITER_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int)

_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.c_int
_Dbl = ctypes.c_double
_P = ctypes.c_void_p

# name -> (restype, argtypes)
SIGNATURES = {
    "foto_last_error": (ctypes.c_char_p, []),
    "foto_version": (_I, []),
    "foto_device_count": (_I, [ctypes.POINTER(_I)]),
    "foto_grad_st": (_I, [_D, _I, _I, _I, _D]),
    "foto_div_st": (_I, [_D, _I, _I, _I, _D]),
    "foto_laplacian_st": (_I, [_D, _I, _I, _I, _D]),
    "foto_apply_A": (_I, [_D, _I, _I, _I, _Dbl, _Dbl, _D]),
    "foto_grad2": (_I, [_D, _I, _I, ctypes.c_char, _D]),
    "foto_div2": (_I, [_D, _I, _I, ctypes.c_char, _D]),
    "foto_grad2_forward": (_I, [_D, _I, _I, _D]),
    "foto_stepB": (_I, [_D, ctypes.c_int64, _D]),
    "foto_bb_rhs": (_I, [_D, _D, _D, _D, _I, _I, _I, _Dbl, _D]),
    "foto_cg": (_I, [_D, _I, _I, _I, _Dbl, _Dbl, _Dbl, _I, _I, _D, ctypes.POINTER(_I)]),
    "foto_flow_from_phi": (_I, [_D, _I, _I, _I, _D, _D, _D]),
    "foto_bb_opts_default": (_I, [ctypes.POINTER(BBOpts)]),
    "foto_bb_create": (_I, [_D, _D, _I, _I, _I, _Dbl, _Dbl, ctypes.POINTER(BBOpts), ctypes.POINTER(_P)]),
    "foto_bb_iterate": (_I, [_P, _I, _Dbl, _I, ITER_CB, _P, ctypes.POINTER(_I)]),
    "foto_bb_flow": (_I, [_P, _D, _D, _D]),
    "foto_bb_reset": (_I, [_P, _D, _D]),
    "foto_bb_get_phi": (_I, [_P, _D]),
    "foto_bb_get_state": (_I, [_P, _D, _D]),
    "foto_bb_shard": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "foto_bb_comm_size": (_I, [_P, ctypes.POINTER(_I)]),
    "foto_bb_stats_get": (_I, [_P, ctypes.POINTER(BBStats)]),
    "foto_bb_stats_reset": (_I, [_P]),
    "foto_bb_set_timing": (_I, [_P, _I]),
    "foto_bb_sync": (_I, [_P]),
    "foto_bb_destroy": (None, [_P]),
    "foto_bb_solve": (_I, [_D, _D, _I, _I, _I, _Dbl, _Dbl, _Dbl, _I, ITER_CB, _P, _D, _D, _D]),
    "foto_bb_solve_ex": (_I, [_D, _D, _I, _I, _I, _Dbl, _Dbl, _Dbl, _I, ctypes.POINTER(BBOpts), _D, _D, _D, _D,
                              ctypes.POINTER(BBSolveStats)]),
    "foto_nccl_unique_id": (_I, [_P]),
    "foto_xfer_calls": (_I, [_I, _I, _I, _I, _I, _I, _I, ctypes.POINTER(ctypes.c_int64), _I, ctypes.POINTER(_I)]),
    "foto_dct": (_I, [_D, _I, _I, _I, _I, _I, _D]),
    "foto_stream_probe": (_I, [ctypes.c_int64, _I, _D]),
    "foto_stream_probe4": (_I, [ctypes.c_int64, _I, _D]),
    "foto_gn_apply": (_I, [_D, _D, _I, _I, _Dbl, _Dbl, _D, _D]),
    "foto_gn_rhs": (_I, [_D, _D, _I, _I, _D]),
    "foto_gn_solve": (_I, [_D, _D, _I, _I, _Dbl, _Dbl, _Dbl, _I, _D, _D, _D, ctypes.POINTER(_I)]),
    "foto_gn_solve_ex": (_I, [_D, _D, _I, _I, _Dbl, _Dbl, _Dbl, _I, _D, _D, _D, ctypes.POINTER(GNStats)]),
    "foto_gn_plan_create": (_I, [_I, _I, _Dbl, _Dbl, _Dbl, _I, ctypes.POINTER(_P)]),
    "foto_gn_plan_solve": (_I, [_P, _D, _D, _D, _D, _D, ctypes.POINTER(_I)]),
    "foto_gn_plan_timing": (_I, [_P, _D]),
    "foto_gn_plan_device": (_I, [_P]),
    "foto_gn_plan_destroy": (None, [_P]),
    "foto_warp": (_I, [_D, _D, _D, _D, _I, _I, _D]),
    "foto_flow_errors": (_I, [_D, _D, _D, _D, _I, _I, _D]),
    "foto_intensity_error": (_I, [_D, _D, _I, _I, _D]),
}

_lib = None


def load(path):
    """A libfoto build at `path` with every signature of include/foto.h set (lib() is the
    product library; tests load libfoto_mockrccl.so, the in-process RCCL transport, this way)."""
    if not os.path.exists(path):
        raise FotoError(f"libfoto.so not found at {path}; build it with "
                        "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C csrc`")
    L = ctypes.CDLL(path)
    lax = os.environ.get("FOTO_LIB_LAX") == "1"   # A/B runs against older builds (tools/ab_lib.sh)
    for name, (res, args) in SIGNATURES.items():
        if lax and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def lib():
    """Load libfoto.so (once).  Raises if it is missing: there is no CPU fallback."""
    global _lib
    if _lib is None:
        _lib = load(LIB_PATH)
    return _lib


def check(rc, L=None):
    if rc < 0:
        msg = (L or lib()).foto_last_error().decode(errors="replace")
        if rc == FOTO_ERR_BC:
            raise NotImplementedError("These boundary conditions are not implemented")
        raise FotoError(f"libfoto error {rc}: {msg}")
    return rc


def dptr(a):
    return a.ctypes.data_as(_D)


def f64(a, n=None, name="array"):
    """C-contiguous float64 copy-free view (or copy) with an optional length check."""
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64).ravel())
    if n is not None and a.size != n:
        raise ValueError(f"{name}: expected {n} values, got {a.size}")
    return a


def device_count():
    n = ctypes.c_int(0)
    check(lib().foto_device_count(ctypes.byref(n)))
    return n.value
