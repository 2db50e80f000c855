"""CPU checks of the boundary: libfoto.so loads and exports every symbol include/foto.h
declares, the ctypes signatures cover exactly that set, and compute calls fail loudly
(no silent CPU fallback) when no device is present."""
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "foto.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(foto_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_parses():
    names = header_functions()
    for must in ("foto_bb_create", "foto_bb_iterate", "foto_cg", "foto_stepB", "foto_gn_solve", "foto_apply_A"):
        assert must in names
    assert "foto_bb_iter_cb" not in names


def test_library_exports_header():
    from foto import _lib
    L = _lib.lib()
    missing = [n for n in header_functions() if not hasattr(L, n)]
    assert not missing, missing


def test_ctypes_signatures_match_header():
    from foto import _lib
    assert set(_lib.SIGNATURES) == set(header_functions())


def test_error_string_and_version():
    from foto import _lib
    assert _lib.lib().foto_version() >= 1
    assert isinstance(_lib.lib().foto_last_error(), bytes)


def test_no_silent_fallback_without_gpu():
    from foto import _lib, ops
    n = 0
    try:
        n = _lib.device_count()
    except _lib.FotoError:
        n = 0
    if n > 0:
        pytest.skip("a GPU is visible; covered by the gpu tests")
    with pytest.raises(_lib.FotoError):
        ops.apply_A(np.zeros(2 * 3 * 4), 2, 4, 3, 1.0, 1e-2)


def test_struct_layouts():
    import ctypes
    from foto import _lib
    # foto_bb_opts: int,int,double,int,int,int,(pad),void*,int,int
    assert ctypes.sizeof(_lib.BBOpts) == 48
    assert _lib.BBStats.n_k.offset == 56
    assert ctypes.sizeof(_lib.BBStats) == 256
    # foto_bb_solve_stats: int cap, 3 pointers, 4 ints, 4 doubles, then foto_bb_stats
    assert _lib.BBSolveStats.ms_create.offset == 48 and _lib.BBSolveStats.bb.offset == 80
    assert ctypes.sizeof(_lib.BBSolveStats) == 336
    assert ctypes.sizeof(_lib.GNStats) == 48 and _lib.GNStats.ms_setup.offset == 16


def test_solve_ex_argument_errors_without_gpu():
    """foto_bb_solve_ex keeps the reference's max_it = 0 failure (benamou_brenier.py:271: phi is
    unbound) as FOTO_ERR_STATE before touching a device, and Nt < 2 as FOTO_ERR_ARG."""
    from foto import _lib
    L = _lib.lib()
    z = np.zeros(12)
    st = _lib.BBSolveStats()
    null = _lib._D()
    rc = L.foto_bb_solve_ex(_lib.dptr(z), _lib.dptr(z), 4, 4, 3, 1.0, 0.3, 1e-3, 0, None, null, null, null, null,
                            st)
    assert rc == _lib.FOTO_ERR_STATE
    rc = L.foto_bb_solve_ex(_lib.dptr(z), _lib.dptr(z), 1, 4, 3, 1.0, 0.3, 1e-3, 5, None, null, null, null, null,
                            st)
    assert rc == _lib.FOTO_ERR_ARG
