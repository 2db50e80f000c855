"""The RCCL code path of the time-sharded solve, run on one GPU.

bench.py --gpus N and the 8-GPU configs (BASELINE configs 4 and 5) shard the outer loop of
benamou_brenier.py:204-258 over time slabs with one process per GPU; every exchange then goes
through foto_bb.cpp's RCCL branches (grouped ncclSend / ncclRecv, the in-place ncclAllGather of
the s-step moments).  Real RCCL refuses two ranks on one device and the test boxes have one GPU,
so libfoto_mockrccl.so -- the same objects linked to an in-process transport with NCCL's
matching rules (csrc/foto_mockrccl.cpp) -- runs W ranks as W threads on one device.

The virtual-rank path (all shards in one context, the same transfer lists executed as device
copies) is already checked against the single-GPU solve (test_gpu_parity.py).  Here each rank
is its own context, exactly as in a multi-process run, and its results must be BIT-identical to
the virtual ranks': the same kernels on the same slabs and boxes, the same moment sums in rank
order, only the transport differs.
"""
import os
import threading

import numpy as np
import pytest

from conftest import PKG

MOCK = os.path.join(PKG, "foto", "libfoto_mockrccl.so")

pytestmark = pytest.mark.gpu


def _mock():
    from foto import _lib
    return _lib.load(MOCK)


def run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters, cg_mode=2, eps=1e-2):
    """W threads, one BBSolver (one RCCL-mode context) each; returns per-rank results."""
    import ctypes
    from foto import _lib
    from foto.bb import BBSolver
    buf = ctypes.create_string_buffer(128)
    _lib.check(L.foto_nccl_unique_id(buf), L)
    nid = bytes(buf.raw)
    out = [None] * W
    errs = []

    def rank(g):
        try:
            with BBSolver(rho0, rhoT, Nt, Nx, Ny, r=1.0, reg_epsilon=eps, device=0, cg_mode=cg_mode, rank=g,
                          world=W, nccl_id=nid, library=L) as s:
                s.iterate(iters, 0.0, stop_rules=False)
                fl = s.flow()
                out[g] = {"crit": list(s.crit), "cg": list(s.cg_its), "flow": fl, "phi": s.phi(),
                          "shard": s.shard(), "redo": s.stats()["cg_redo"]}
        except BaseException as e:  # noqa: BLE001 -- reported by the main thread
            errs.append((g, e))

    th = [threading.Thread(target=rank, args=(g,)) for g in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in th), "a rank hung (mock RCCL waits are bounded: see the log)"
    assert not errs, errs
    return out


def run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters, cg_mode=2, eps=1e-2):
    from foto.bb import BBSolver
    with BBSolver(rho0, rhoT, Nt, Nx, Ny, r=1.0, reg_epsilon=eps, device=0, cg_mode=cg_mode, virtual_ranks=W,
                  library=L) as s:
        s.iterate(iters, 0.0, stop_rules=False)
        return {"crit": list(s.crit), "cg": list(s.cg_its), "flow": s.flow(), "phi": s.phi()}


def compare(ranks, virt, Nt, Nx, Ny, W):
    nxy = Nx * Ny
    for g, res in enumerate(ranks):
        assert res["crit"] == virt["crit"], (g, res["crit"][:3], virt["crit"][:3])
        assert res["cg"] == virt["cg"], (g, res["cg"], virt["cg"])
        t0, nl = res["shard"]
        np.testing.assert_array_equal(res["phi"], virt["phi"][t0 * nxy:(t0 + nl) * nxy])
    for a, b in zip(ranks[0]["flow"], virt["flow"]):
        np.testing.assert_array_equal(a, b)
    for g in range(1, W):
        assert ranks[g]["flow"] is None


@pytest.mark.parametrize("cg_mode", [2, 3])
@pytest.mark.parametrize("W", [2, 3, 4, 5, 8])
def test_rccl_path_bit_identical_to_virtual_ranks(W, cg_mode):
    """cg_mode 2: one moment all-gather per s-step pass; cg_mode 3: one histogram all-gather
    (4096 doubles) per CG solve."""
    from foto.synthetic import translating_gaussian
    Nt, Nx, Ny = 16, 64, 48
    rho0, rhoT = translating_gaussian(Nx, Ny)
    L = _mock()
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=6, cg_mode=cg_mode)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=6, cg_mode=cg_mode)
    compare(ranks, virt, Nt, Nx, Ny, W)


def test_rccl_path_gauss_redo(monkeypatch):
    """A failed Gauss solve on every rank (FOTO_GQ_KLIM=1: status 2 everywhere, from the same
    gathered histograms) is redone by every rank with the s-step CG at the crit sync: the
    collective sequences stay paired and the results equal the virtual ranks' bit for bit."""
    from foto.synthetic import translating_gaussian
    monkeypatch.setenv("FOTO_GQ_KLIM", "1")
    Nt, Nx, Ny, W = 16, 64, 48, 3
    rho0, rhoT = translating_gaussian(Nx, Ny)
    L = _mock()
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    compare(ranks, virt, Nt, Nx, Ny, W)
    assert all(r["redo"] == 4 for r in ranks)


def test_rccl_path_stencil_cg():
    """cg_mode 0: a halo exchange of p and two scalar all-gathers per CG iteration."""
    from foto.synthetic import translating_gaussian
    Nt, Nx, Ny, W = 9, 40, 30, 3
    rho0, rhoT = translating_gaussian(Nx, Ny)
    L = _mock()
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=3, cg_mode=0)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=3, cg_mode=0)
    compare(ranks, virt, Nt, Nx, Ny, W)


@pytest.mark.parametrize("cg_mode", [2, 3])
def test_rccl_path_bench_grid_w8(cg_mode):
    """The driver's 8-GPU scaling run: the bench grid 640x480x32 over 8 ranks (4 planes and 60
    rows each), three outer iterations, against the same decomposition as virtual ranks and,
    within the spectral path's bar, against one shard."""
    from foto.synthetic import translating_gaussian
    Nt, Nx, Ny, W = 32, 640, 480, 8
    rho0, rhoT = translating_gaussian(Nx, Ny)
    L = _mock()
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=3, cg_mode=cg_mode)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=3, cg_mode=cg_mode)
    compare(ranks, virt, Nt, Nx, Ny, W)
    one = run_virtual(L, 1, rho0, rhoT, Nt, Nx, Ny, iters=3, cg_mode=cg_mode)
    assert all(abs(a - b) <= 1 for a, b in zip(ranks[0]["cg"], one["cg"]))
    np.testing.assert_allclose(ranks[0]["crit"], one["crit"], rtol=1e-7)


def test_rccl_path_c4_w8():
    """BASELINE config 4 (1024 x 1024 x 64, time-sharded over 8 GPUs) through the RCCL branches:
    8 planes and 128 rows per rank, the default Gauss CG (one histogram all-gather per solve),
    the fused prox + RHS with its two-plane phi / one-plane mu halos.  Bit-identical to the same
    decomposition as virtual ranks; CG counts within one of a single shard's."""
    from foto.synthetic import translating_gaussian
    Nt, Nx, Ny, W = 64, 1024, 1024, 8
    rho0, rhoT = translating_gaussian(Nx, Ny)
    L = _mock()
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=2, cg_mode=3)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=2, cg_mode=3)
    compare(ranks, virt, Nt, Nx, Ny, W)
    one = run_virtual(L, 1, rho0, rhoT, Nt, Nx, Ny, iters=2, cg_mode=3)
    assert all(abs(a - b) <= 1 for a, b in zip(ranks[0]["cg"], one["cg"]))
    np.testing.assert_allclose(ranks[0]["crit"], one["crit"], rtol=1e-7)
    assert all(r["redo"] == 0 for r in ranks)


def test_rccl_path_c4_w4():
    """The driver's N = 4 scaling run of config 4: 16 planes and 256 rows per rank, the default
    pipelined all-to-alls with the phi halo inside the backward one (planes of 2^20 voxels) --
    bit-identical to the same decomposition as virtual ranks."""
    from foto.synthetic import translating_gaussian
    Nt, Nx, Ny, W = 64, 1024, 1024, 4
    rho0, rhoT = translating_gaussian(Nx, Ny)
    L = _mock()
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=2, cg_mode=3)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=2, cg_mode=3)
    compare(ranks, virt, Nt, Nx, Ny, W)
    assert all(r["redo"] == 0 for r in ranks)


@pytest.mark.parametrize("W", [2, 3, 5])
def test_rccl_comm_stream_pipelined_alltoall_and_phi_halo(monkeypatch, W):
    """The communication stream and the pipelined all-to-alls (foto_bb.cpp comm_fork / comm_join,
    sharded_fwd / sharded_inv: 1, 2 or 3 parts per direction; phi's halo planes delivered by the
    backward all-to-all, FOTO_A2A_HALO) change only where and when data travels: every variant,
    over the mock RCCL and as virtual ranks, equals the plain sequence (one part, the separate
    phi halo exchange, every call on the compute stream) bit for bit.  Nt = 7: slabs of one to
    four planes, so some ranks have empty parts; the textured pair gives the flow something to
    carry."""
    from foto.synthetic import textured_pair
    Nt, Nx, Ny = 7, 48, 40
    rho0, rhoT = textured_pair(Nx, Ny, seed=5, dx=1.0, dy=0.5)
    L = _mock()
    for k in ("FOTO_A2A_PARTS", "FOTO_A2A_HALO", "FOTO_COMM_STREAM", "FOTO_WT_OVERLAP"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("FOTO_A2A_PARTS", "1")
    monkeypatch.setenv("FOTO_A2A_HALO", "0")
    monkeypatch.setenv("FOTO_COMM_STREAM", "0")
    plain = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    # (at 48 x 40 the halo delivery is off by default -- a2a_big_planes -- so it is forced on here:
    # alltoall_part_xfers with halo = 1, the inverse DCTs on nloc + 2 planes, prox without its
    # own phi halo exchange)
    for env in ({}, {"FOTO_A2A_PARTS": "3"}, {"FOTO_A2A_HALO": "0"}, {"FOTO_COMM_STREAM": "0"},
                {"FOTO_A2A_HALO": "1"}, {"FOTO_A2A_PARTS": "3", "FOTO_A2A_HALO": "1"},
                {"FOTO_A2A_PARTS": "2", "FOTO_A2A_HALO": "1", "FOTO_COMM_STREAM": "0"}):
        for k in ("FOTO_A2A_PARTS", "FOTO_A2A_HALO", "FOTO_COMM_STREAM", "FOTO_WT_OVERLAP"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
        virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
        compare(ranks, virt, Nt, Nx, Ny, W)
        for a, b in zip(ranks, plain):
            assert a["crit"] == b["crit"] and a["cg"] == b["cg"], env
            np.testing.assert_array_equal(a["phi"], b["phi"])
        for a, b in zip(ranks[0]["flow"], plain[0]["flow"]):
            np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("W,parts", [(2, 1), (3, 2), (3, 3)])
def test_rccl_wt_exchange_overlapped_with_interior_planes(monkeypatch, W, parts):
    """The deferred slab edges' w_t computed first (k_wt_pre) and exchanged on the communication
    stream while k_prox_rhs runs, the edges' F finished by the next forward (foto_bb.cpp
    wt_overlap / prox_rhs / sharded_fwd), equals the prox-then-exchange order (FOTO_WT_OVERLAP=0)
    bit for bit, and the virtual ranks with and without k_wt_pre.  Nt = 10: slabs of three and
    four planes (the overlap needs >= 3 on every rank)."""
    from foto.synthetic import textured_pair
    Nt, Nx, Ny = 10, 48, 40
    rho0, rhoT = textured_pair(Nx, Ny, seed=7, dx=0.5, dy=1.0)
    L = _mock()
    for k in ("FOTO_A2A_HALO", "FOTO_COMM_STREAM"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("FOTO_A2A_PARTS", str(parts))
    monkeypatch.setenv("FOTO_WT_OVERLAP", "0")
    seq = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    monkeypatch.setenv("FOTO_WT_OVERLAP", "1")
    ranks = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    virt = run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    compare(ranks, virt, Nt, Nx, Ny, W)
    monkeypatch.setenv("FOTO_WT_PRE", "1")   # virtual ranks with k_wt_pre (tools/proxy_scaling.py)
    compare(ranks, run_virtual(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3), Nt, Nx, Ny, W)
    monkeypatch.delenv("FOTO_WT_PRE")
    # k_wt_pre reads the phi halo plane: with the halo delivered inside the backward all-to-all too
    monkeypatch.setenv("FOTO_A2A_HALO", "1")
    halo = run_ranks(L, W, rho0, rhoT, Nt, Nx, Ny, iters=4, cg_mode=3)
    for got in (ranks, halo):
        for a, b in zip(got, seq):
            assert a["crit"] == b["crit"] and a["cg"] == b["cg"]
            np.testing.assert_array_equal(a["phi"], b["phi"])
        for a, b in zip(got[0]["flow"], seq[0]["flow"]):
            np.testing.assert_array_equal(a, b)
