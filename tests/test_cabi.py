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
