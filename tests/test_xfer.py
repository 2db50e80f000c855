"""CPU checks of the multi-GPU exchange layer before it ever runs over RCCL.

The time-sharded solve (the outer loop of benamou_brenier.py:204-258 split
into contiguous time slabs, the spectral CG on row boxes) moves data only through the
transfer lists of csrc/foto_xfer.h.  Over RCCL each rank issues, for one list, a grouped
sequence of ncclSend / ncclRecv calls followed by local copies.  NCCL pairs the k-th send from
rank a to rank b with the k-th receive posted by b from a, so the sequences must agree call
for call across ranks, or the 8-GPU run hangs or corrupts data.

These tests take the call sequences from the library itself (foto_xfer_calls, the exact code
path foto_bb.cpp executes) for W = 2 .. 8 at the bench grid, the Dimetrodon size and C4's
1024x1024x64, and check: sends pair with receives (same peers, order and counts), nothing goes
through RCCL to itself, every offset stays inside its buffer, the received regions tile the
destination exactly, and -- by replaying the calls on numpy arrays -- that the slab <-> row-box
all-to-all, the halos, the trajectory relay and the flow delivery move the right elements.
"""
import ctypes

import numpy as np
import pytest

XFER_HALO, XFER_SLAB_TO_BOX, XFER_BOX_TO_SLAB, XFER_RELAY, XFER_DELIVER, XFER_HALO2 = range(6)
XFER_SLAB_TO_BOX_PART, XFER_BOX_TO_SLAB_PART = 6, 7
SEND, RECV, COPY = range(3)

GRIDS = [(32, 480, 640), (32, 388, 584), (64, 1024, 1024)]   # (Nt, Ny, Nx)


def split(n, W, h):
    base, extra = divmod(n, W)
    return h * base + min(h, extra), base + (1 if h < extra else 0)


def calls(kind, Nt, Ny, Nx, W, rank, arg=0):
    from foto import _lib
    cap = 4 * W * (Nt + W + 2) + 8   # (the all-to-all: one transfer per plane and peer)
    out = (ctypes.c_int64 * (5 * cap))()
    cnt = ctypes.c_int(0)
    _lib.check(_lib.lib().foto_xfer_calls(kind, Nt, Ny, Nx, W, rank, arg, out, cap, ctypes.byref(cnt)))
    a = np.frombuffer(out, dtype=np.int64, count=5 * cnt.value).reshape(cnt.value, 5)
    return [tuple(int(v) for v in row) for row in a]


def all_calls(kind, Nt, Ny, Nx, W, arg=0):
    return [calls(kind, Nt, Ny, Nx, W, g, arg) for g in range(W)]


def src_extent(kind, Nt, Ny, Nx, W, g):
    """[lo, hi) in doubles of the buffer a send / copy of rank g reads."""
    nxy = Nx * Ny
    _, nl = split(Nt, W, g)
    _, nyl = split(Ny, W, g)
    if kind == XFER_HALO:
        return -nxy, (nl + 1) * nxy
    if kind == XFER_HALO2:
        return 0, nl * nxy                      # own planes only (halos come from their owners)
    if kind in (XFER_SLAB_TO_BOX, XFER_SLAB_TO_BOX_PART):
        return 0, nl * nxy                      # the slab [tl][y][x] (the rank's RHS buffer)
    if kind in (XFER_BOX_TO_SLAB, XFER_BOX_TO_SLAB_PART):
        return 0, Nt * nyl * Nx                 # box_out: [t][own rows][x]
    return 0, nxy                               # px / py / fu, fv, fm


def dst_extent(kind, Nt, Ny, Nx, W, g):
    nxy = Nx * Ny
    _, nl = split(Nt, W, g)
    _, nyl = split(Ny, W, g)
    if kind == XFER_HALO:
        return -nxy, (nl + 1) * nxy
    if kind == XFER_HALO2:
        return -2 * nxy, (nl + 2) * nxy
    if kind in (XFER_SLAB_TO_BOX, XFER_SLAB_TO_BOX_PART):
        return 0, max(Nt * nyl * Nx, nl * nxy)   # box_in (the spectral tmp buffer)
    if kind == XFER_BOX_TO_SLAB:
        return 0, nl * nxy                       # the slab [tl][y][x]
    if kind == XFER_BOX_TO_SLAB_PART:
        return -nxy, (nl + 1) * nxy              # the slab with one halo plane per side
    return 0, nxy


def check_pairing(cs, W):
    """sends of a to b == receives at b from a, in order and count; no RCCL self-transfers"""
    for a in range(W):
        for op, peer, off, n, doff in cs[a]:
            assert n > 0
            if op in (SEND, RECV):
                assert peer != a, f"rank {a}: {('send', 'recv')[op]} to itself through RCCL"
            else:
                assert op == COPY and peer == a
        ops = [c[0] for c in cs[a]]
        # the group (sends / receives) comes first, copies after it
        assert ops == sorted(ops, key=lambda o: o == COPY), ops
    for a in range(W):
        for b in range(W):
            if a == b:
                continue
            sends = [c[3] for c in cs[a] if c[0] == SEND and c[1] == b]
            recvs = [c[3] for c in cs[b] if c[0] == RECV and c[1] == a]
            assert sends == recvs, f"{a}->{b}: sends {sends} vs receives {recvs}"


def check_bounds_and_tiling(kind, cs, Nt, Ny, Nx, W, expect_full):
    for g in range(W):
        slo, shi = src_extent(kind, Nt, Ny, Nx, W, g)
        dlo, dhi = dst_extent(kind, Nt, Ny, Nx, W, g)
        got = []
        for op, peer, off, n, doff in cs[g]:
            if op in (SEND, COPY):
                assert slo <= off and off + n <= shi, (g, op, off, n, slo, shi)
            if op == RECV:
                assert dlo <= off and off + n <= dhi, (g, off, n, dlo, dhi)
                got.append((off, off + n))
            if op == COPY:
                assert dlo <= doff and doff + n <= dhi, (g, doff, n, dlo, dhi)
                got.append((doff, doff + n))
        got.sort()
        for (a0, a1), (b0, b1) in zip(got, got[1:]):
            assert a1 <= b0, f"rank {g}: overlapping destination regions {a0, a1} {b0, b1}"
        if expect_full is not None:
            lo, hi = expect_full(g)
            assert got and got[0][0] == lo and got[-1][1] == hi, (g, got[:2], got[-2:], lo, hi)
            assert all(a1 == b0 for (_, a1), (b0, _) in zip(got, got[1:])), f"rank {g}: gaps"


@pytest.mark.parametrize("grid", GRIDS, ids=lambda g: "x".join(map(str, g[::-1])))
@pytest.mark.parametrize("W", range(2, 9))
def test_rccl_call_sequences_pair(grid, W):
    Nt, Ny, Nx = grid
    nxy = Nx * Ny
    for kind in (XFER_HALO, XFER_HALO2, XFER_SLAB_TO_BOX, XFER_BOX_TO_SLAB, XFER_DELIVER):
        cs = all_calls(kind, Nt, Ny, Nx, W)
        check_pairing(cs, W)
        if kind == XFER_SLAB_TO_BOX:
            full = lambda g: (0, Nt * split(Ny, W, g)[1] * Nx)
        elif kind == XFER_BOX_TO_SLAB:
            full = lambda g: (0, split(Nt, W, g)[1] * nxy)
        else:
            full = None
        check_bounds_and_tiling(kind, cs, Nt, Ny, Nx, W, full)
    # halo: rank g receives exactly its two neighbour planes
    cs = all_calls(XFER_HALO, Nt, Ny, Nx, W)
    for g in range(W):
        _, nl = split(Nt, W, g)
        recv = sorted((c[1], c[2], c[3]) for c in cs[g] if c[0] == RECV)
        want = sorted(([(g - 1, -nxy, nxy)] if g > 0 else []) + ([(g + 1, nl * nxy, nxy)] if g + 1 < W else []))
        assert recv == want
    # two-plane halo (phi of the fused prox + RHS): each halo plane from the rank owning it
    cs = all_calls(XFER_HALO2, Nt, Ny, Nx, W)
    owner = [g for g in range(W) for _ in range(split(Nt, W, g)[1])]
    for g in range(W):
        t0, nl = split(Nt, W, g)
        got = sorted([(c[1], c[2]) for c in cs[g] if c[0] == RECV] + [(g, c[4]) for c in cs[g] if c[0] == COPY])
        want = sorted((owner[t0 + h], h * nxy) for h in (-2, -1, nl, nl + 1) if 0 <= t0 + h < Nt)
        assert got == want
    # relay: only ranks j and j + 1 take part, one plane of positions
    for j in range(W - 1):
        cs = all_calls(XFER_RELAY, Nt, Ny, Nx, W, j)
        check_pairing(cs, W)
        for g in range(W):
            want = [(SEND, j + 1, 0, nxy, 0)] if g == j else [(RECV, j, 0, nxy, 0)] if g == j + 1 else []
            assert cs[g] == want


def replay(kind, Nt, Ny, Nx, W, src, dst, arg=0):
    """Execute every rank's calls on numpy buffers, pairing the k-th send a->b with the k-th
    receive at b from a (NCCL's matching rule); buffers are dicts rank -> (array, origin)."""
    cs = all_calls(kind, Nt, Ny, Nx, W, arg)
    check_pairing(cs, W)
    queues = {}
    for a in range(W):
        for op, peer, off, n, doff in cs[a]:
            if op == SEND:
                buf, o = src[a]
                queues.setdefault((a, peer), []).append(buf[o + off:o + off + n].copy())
    for b in range(W):
        taken = {}
        for op, peer, off, n, doff in cs[b]:
            buf, o = dst[b]
            if op == RECV:
                k = taken.get(peer, 0)
                taken[peer] = k + 1
                data = queues[(peer, b)][k]
                assert data.size == n
                buf[o + off:o + off + n] = data
            elif op == COPY:
                sbuf, so = src[b]
                buf[o + doff:o + doff + n] = sbuf[so + off:so + off + n]


@pytest.mark.parametrize("shape", [(9, 7, 5), (16, 12, 10), (32, 48, 64)], ids=lambda s: "x".join(map(str, s[::-1])))
@pytest.mark.parametrize("W", range(2, 9))
def test_replayed_exchanges_move_the_right_elements(shape, W):
    Nt, Ny, Nx = shape
    if W > Nt or W > Ny:
        pytest.skip("each rank needs a time plane and a row")
    rng = np.random.default_rng(W)
    G = rng.standard_normal((Nt, Ny, Nx))
    nxy = Nx * Ny
    slabs = [split(Nt, W, g) for g in range(W)]
    boxes = [split(Ny, W, g) for g in range(W)]

    # slab -> box: straight from each rank's planes in their natural layout (one transfer per plane
    # and destination box)
    stage = {g: (G[t0:t0 + nl].ravel().copy(), 0) for g, (t0, nl) in enumerate(slabs)}
    box_in = {g: (np.full(max(Nt * boxes[g][1] * Nx, slabs[g][1] * nxy), np.nan), 0) for g in range(W)}
    replay(XFER_SLAB_TO_BOX, Nt, Ny, Nx, W, stage, box_in)
    for g, (y0, nyl) in enumerate(boxes):
        np.testing.assert_array_equal(box_in[g][0][:Nt * nyl * Nx].reshape(Nt, nyl, Nx), G[:, y0:y0 + nyl, :])

    # box -> slab: the inverse (box_out = own rows of every plane) lands in the natural layout
    box_out = {g: (G[:, y0:y0 + nyl, :].ravel().copy(), 0) for g, (y0, nyl) in enumerate(boxes)}
    stage2 = {g: (np.full(slabs[g][1] * nxy, np.nan), 0) for g in range(W)}
    replay(XFER_BOX_TO_SLAB, Nt, Ny, Nx, W, box_out, stage2)
    for g, (t0, nl) in enumerate(slabs):
        np.testing.assert_array_equal(stage2[g][0].reshape(nl, Ny, Nx), G[t0:t0 + nl])

    # halos: planes -1 and nloc of every rank's padded field hold the neighbours' planes
    fields = {}
    for g, (t0, nl) in enumerate(slabs):
        f = np.full((nl + 2) * nxy, np.nan)
        f[nxy:(nl + 1) * nxy] = G[t0:t0 + nl].ravel()
        fields[g] = (f, nxy)   # origin: local plane 0
    replay(XFER_HALO, Nt, Ny, Nx, W, fields, fields)
    for g, (t0, nl) in enumerate(slabs):
        f = fields[g][0].reshape(nl + 2, nxy)
        np.testing.assert_array_equal(f[1:nl + 1], G[t0:t0 + nl].reshape(nl, nxy))
        if g > 0:
            np.testing.assert_array_equal(f[0], G[t0 - 1].ravel())
        if g + 1 < W:
            np.testing.assert_array_equal(f[nl + 1], G[t0 + nl].ravel())

    # two-plane halos (planes -2, -1, nloc, nloc + 1), from two ranks away when a slab is one plane
    fields2 = {}
    for g, (t0, nl) in enumerate(slabs):
        f = np.full((nl + 4) * nxy, np.nan)
        f[2 * nxy:(nl + 2) * nxy] = G[t0:t0 + nl].ravel()
        fields2[g] = (f, 2 * nxy)
    replay(XFER_HALO2, Nt, Ny, Nx, W, fields2, fields2)
    for g, (t0, nl) in enumerate(slabs):
        f = fields2[g][0].reshape(nl + 4, nxy)
        for h in (-2, -1, nl, nl + 1):
            if 0 <= t0 + h < Nt:
                np.testing.assert_array_equal(f[h + 2], G[t0 + h].ravel())
            else:
                assert np.all(np.isnan(f[h + 2]))

    # trajectory relay j -> j + 1 and the flow delivery W - 1 -> 0
    pos = {g: (np.full(nxy, float(g)), 0) for g in range(W)}
    for j in range(W - 1):
        replay(XFER_RELAY, Nt, Ny, Nx, W, pos, pos, j)
        assert np.all(pos[j + 1][0] == 0.0)   # rank 0's positions travelled all the way
    flow = {g: (np.full(nxy, float(g)), 0) for g in range(W)}
    replay(XFER_DELIVER, Nt, Ny, Nx, W, flow, flow)
    assert np.all(flow[0][0] == W - 1)


def test_bad_arguments_rejected():
    from foto import _lib
    cnt = ctypes.c_int(0)
    out = (ctypes.c_int64 * 5)()
    L = _lib.lib()
    assert L.foto_xfer_calls(XFER_HALO, 4, 8, 8, 5, 0, 0, out, 1, ctypes.byref(cnt)) == _lib.FOTO_ERR_ARG   # Nt < W
    assert L.foto_xfer_calls(9, 8, 8, 8, 2, 0, 0, out, 1, ctypes.byref(cnt)) == _lib.FOTO_ERR_ARG          # kind
    assert L.foto_xfer_calls(XFER_RELAY, 8, 8, 8, 2, 0, 1, out, 1, ctypes.byref(cnt)) == _lib.FOTO_ERR_ARG  # step
    assert L.foto_xfer_calls(XFER_SLAB_TO_BOX, 8, 8, 8, 4, 0, 0, out, 1, ctypes.byref(cnt)) == _lib.FOTO_ERR_ARG  # cap


def part_arg(part, parts, halo=0):
    return part | (parts << 8) | (halo << 16)


def part_planes(Nt, W, g, part, parts, halo):
    """foto_xfer.h alltoall_part_planes: the local planes a backward part delivers to rank g."""
    t0, nl = split(Nt, W, g)
    lo, hi = part * nl // parts, (part + 1) * nl // parts
    if halo and part == 0 and t0 > 0:
        lo -= 1
    if halo and part == parts - 1 and t0 + nl < Nt:
        hi += 1
    return lo, hi


@pytest.mark.parametrize("grid", GRIDS, ids=lambda g: "x".join(map(str, g[::-1])))
@pytest.mark.parametrize("W", [2, 3, 5, 8])
def test_pipelined_alltoall_parts_pair_and_cover(grid, W):
    """The pipelined all-to-alls (foto_bb.cpp sharded_fwd / sharded_inv): every part pairs on its
    own (each part is one RCCL group), the forward parts together are the plain forward list,
    and the backward parts deliver exactly the planes alltoall_part_planes says -- the own
    planes tiled once, plus phi's halo planes (t0 - 1, t0 + nloc where they exist) with halo = 1."""
    Nt, Ny, Nx = grid
    nxy = Nx * Ny
    full_fwd = [sorted(c) for c in all_calls(XFER_SLAB_TO_BOX, Nt, Ny, Nx, W)]
    full_bwd = [sorted(c) for c in all_calls(XFER_BOX_TO_SLAB, Nt, Ny, Nx, W)]
    for parts in (1, 2, 3):
        got_fwd = [[] for _ in range(W)]
        for halo in (0, 1):
            got_bwd = [[] for _ in range(W)]
            for part in range(parts):
                cf = all_calls(XFER_SLAB_TO_BOX_PART, Nt, Ny, Nx, W, part_arg(part, parts))
                check_pairing(cf, W)
                check_bounds_and_tiling(XFER_SLAB_TO_BOX_PART, cf, Nt, Ny, Nx, W, None)
                if halo == 0:
                    for g in range(W):
                        got_fwd[g] += cf[g]
                cb = all_calls(XFER_BOX_TO_SLAB_PART, Nt, Ny, Nx, W, part_arg(part, parts, halo))
                check_pairing(cb, W)
                check_bounds_and_tiling(XFER_BOX_TO_SLAB_PART, cb, Nt, Ny, Nx, W, None)
                for g in range(W):
                    got_bwd[g] += cb[g]
                    lo, hi = part_planes(Nt, W, g, part, parts, halo)
                    landed = sorted({(c[2] if c[0] == RECV else c[4]) // nxy for c in cb[g] if c[0] in (RECV, COPY)})
                    assert landed == list(range(lo, hi)), (parts, part, halo, g, landed, lo, hi)
            for g in range(W):
                if halo == 0:
                    assert sorted(got_bwd[g]) == full_bwd[g]
        for g in range(W):
            assert sorted(got_fwd[g]) == full_fwd[g]


@pytest.mark.parametrize("W", [2, 3, 5])
def test_replayed_backward_alltoall_delivers_phi_halo(W):
    """Replaying the backward parts with halo = 1 on numpy buffers: every rank's slab planes and
    its two halo planes (where they exist) hold the right rows of the global volume, planes
    outside [0, Nt) stay untouched."""
    Nt, Ny, Nx = 9, 7, 5
    rng = np.random.default_rng(W)
    G = rng.standard_normal((Nt, Ny, Nx))
    nxy = Nx * Ny
    slabs = [split(Nt, W, g) for g in range(W)]
    boxes = [split(Ny, W, g) for g in range(W)]
    box_out = {g: (G[:, y0:y0 + nyl, :].ravel().copy(), 0) for g, (y0, nyl) in enumerate(boxes)}
    dst = {g: (np.full((nl + 2) * nxy, np.nan), nxy) for g, (t0, nl) in enumerate(slabs)}
    for parts in (2, 3):
        for g in dst:
            dst[g][0][:] = np.nan
        for part in range(parts):
            replay(XFER_BOX_TO_SLAB_PART, Nt, Ny, Nx, W, box_out, dst, part_arg(part, parts, 1))
        for g, (t0, nl) in enumerate(slabs):
            f = dst[g][0].reshape(nl + 2, Ny, Nx)
            for h in range(-1, nl + 1):
                if 0 <= t0 + h < Nt:
                    np.testing.assert_array_equal(f[h + 1], G[t0 + h])
                else:
                    assert np.all(np.isnan(f[h + 1]))

