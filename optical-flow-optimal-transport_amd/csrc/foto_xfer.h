// Transfer lists of the time-sharded Benamou-Brenier solve (host-only C++, no HIP).
//
// Every exchange between the shards of the 8-GPU decomposition (contiguous
// time slabs, benamou_brenier.py:204-258 sharded on t) is a list of point-to-point transfers
// {src rank, dst rank, src offset, dst offset, count}, built by the same code on every rank.
// foto_bb.cpp executes a list either as device copies (virtual ranks, one process) or as one
// RCCL group (ncclSend for each transfer from this rank, ncclRecv for each transfer to it,
// in list order; a transfer to itself is a device copy).  rccl_calls() is that issue order,
// and the test entry foto_xfer_calls (foto_bb.cpp) exposes it so a CPU test can check that
// every rank's sends pair with its peers' receives for W = 2 .. 8 without a GPU.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace foto {

// balanced split of n items over W ranks: rank gets [*t0, *t0 + *nloc)
inline int split_planes(int n, int W, int rank, int* t0, int* nloc) {
    const int base = n / W, extra = n % W;
    *nloc = base + (rank < extra ? 1 : 0);
    *t0 = rank * base + std::min(rank, extra);
    return *nloc >= 1 ? 0 : -1;
}

struct Xfer {
    int src, dst;
    int64_t soff, doff, n;   // doubles, relative to the picked buffer of each shard
};

// halo planes of a halo-padded field (pointer at local plane 0): plane -1 <- the previous
// rank's last plane, plane nloc <- the next rank's first plane
inline std::vector<Xfer> halo_xfers(int Nt, int64_t nxy, int W) {
    std::vector<Xfer> xs;
    for (int j = 0; j + 1 < W; ++j) {
        int t0, nl;
        split_planes(Nt, W, j, &t0, &nl);
        xs.push_back({j, j + 1, (int64_t)(nl - 1) * nxy, -nxy, nxy});   // up: last plane -> halo below
        xs.push_back({j + 1, j, 0, (int64_t)nl * nxy, nxy});             // down: first plane -> halo above
    }
    return xs;
}

// `depth` halo planes on each side (planes -depth .. -1 and nloc .. nloc + depth - 1 of every
// rank), each from the rank that owns that global plane (a rank with fewer planes than depth
// gets some of its halo from two ranks away); planes outside [0, Nt) are not sent.  depth 1
// is halo_xfers' list in a different order; the fused prox + RHS reads phi two planes deep.
inline std::vector<Xfer> halo_depth_xfers(int Nt, int64_t nxy, int W, int depth) {
    std::vector<int> t0(W), nl(W), owner(Nt);
    for (int g = 0; g < W; ++g) {
        split_planes(Nt, W, g, &t0[g], &nl[g]);
        for (int t = t0[g]; t < t0[g] + nl[g]; ++t) owner[t] = g;
    }
    std::vector<Xfer> xs;
    for (int b = 0; b < W; ++b)
        for (int k = 0; k < 2 * depth; ++k) {
            const int h = (k < depth) ? k - depth : nl[b] + (k - depth);   // local halo plane of rank b
            const int t = t0[b] + h;
            if (t < 0 || t >= Nt) continue;
            const int a = owner[t];
            xs.push_back({a, b, (int64_t)(t - t0[a]) * nxy, (int64_t)h * nxy, nxy});
        }
    return xs;
}

// all-to-all between the physical slabs and the spectral row boxes (SpectralPlan), one transfer
// per (source, destination, plane) straight between the natural layouts -- no packing pass:
//   forward : rank a's slab [tl][y][x], rows [y0_b, + nyl_b) of its plane tl -> box_in_b[t0_a + tl][.][.]
//   backward: rank a's box_out [t][y - y0_a][x], plane t0_b + tl             -> slab_b[tl][y0_a ..][.]
// (a plane's rows of one box are contiguous on both sides: nyl * Nx doubles per transfer)
inline std::vector<Xfer> alltoall_xfers(int Nt, int Ny, int Nx, int W, bool forward) {
    std::vector<Xfer> xs;
    const int64_t nxy = (int64_t)Nx * Ny;
    for (int a = 0; a < W; ++a)
        for (int b = 0; b < W; ++b) {
            int ta, na, tb, nb, ya, nya, yb, nyb;
            split_planes(Nt, W, a, &ta, &na);
            split_planes(Nt, W, b, &tb, &nb);
            split_planes(Ny, W, a, &ya, &nya);
            split_planes(Ny, W, b, &yb, &nyb);
            if (forward) {
                for (int tl = 0; tl < na; ++tl)
                    if (nyb > 0)
                        xs.push_back({a, b, tl * nxy + (int64_t)yb * Nx, (int64_t)(ta + tl) * nyb * Nx,
                                      (int64_t)nyb * Nx});
            } else {
                for (int tl = 0; tl < nb; ++tl)
                    if (nya > 0)
                        xs.push_back({a, b, (int64_t)(tb + tl) * nya * Nx, tl * nxy + (int64_t)ya * Nx,
                                      (int64_t)nya * Nx});
            }
        }
    return xs;
}

// part `part` of `parts` of n items: [part n / parts, (part + 1) n / parts)
inline void split_part(int n, int parts, int part, int* lo, int* hi) {
    *lo = (int)((int64_t)part * n / parts);
    *hi = (int)((int64_t)(part + 1) * n / parts);
}

// The pipelined all-to-alls (foto_bb.cpp sharded_fwd / sharded_inv): the same transfers as
// alltoall_xfers, issued in `parts` groups so a group travels on the communication stream while
// the compute stream transforms the next one.
//   forward, part p: the planes of part p of every SOURCE slab (sent once their x / y DCTs ran);
//   backward, part p: the planes of part p of every DESTINATION slab (transformed back once they
//   arrived), with `halo` (0 or 1) extra planes per side -- the lower halo plane (t0 - 1) with
//   the first part, the upper one (t0 + nloc) with the last, landing in the slab's halo planes
//   (local -1, nloc); planes outside [0, Nt) are not sent.  The inverse x / y DCTs then run on
//   nloc + 2 planes and phi arrives with the halo plane the fused prox + RHS reads: rows of it
//   from every box owner, over all links, instead of a whole plane from one neighbour over one.
// parts = 1, halo = 0: alltoall_xfers' lists, in the same order.
inline std::vector<Xfer> alltoall_part_xfers(int Nt, int Ny, int Nx, int W, bool forward, int part, int parts,
                                             int halo) {
    std::vector<Xfer> xs;
    const int64_t nxy = (int64_t)Nx * Ny;
    for (int a = 0; a < W; ++a)
        for (int b = 0; b < W; ++b) {
            int ta, na, tb, nb, ya, nya, yb, nyb;
            split_planes(Nt, W, a, &ta, &na);
            split_planes(Nt, W, b, &tb, &nb);
            split_planes(Ny, W, a, &ya, &nya);
            split_planes(Ny, W, b, &yb, &nyb);
            if (forward) {
                int lo, hi;
                split_part(na, parts, part, &lo, &hi);
                for (int tl = lo; tl < hi; ++tl)
                    if (nyb > 0)
                        xs.push_back({a, b, tl * nxy + (int64_t)yb * Nx, (int64_t)(ta + tl) * nyb * Nx,
                                      (int64_t)nyb * Nx});
            } else {
                int lo, hi;
                split_part(nb, parts, part, &lo, &hi);
                if (halo && part == 0 && tb > 0) lo -= 1;
                if (halo && part == parts - 1 && tb + nb < Nt) hi += 1;
                for (int tl = lo; tl < hi; ++tl)
                    if (nya > 0)
                        xs.push_back({a, b, (int64_t)(tb + tl) * nya * Nx, tl * nxy + (int64_t)ya * Nx,
                                      (int64_t)nya * Nx});
            }
        }
    return xs;
}

// the local planes [lo, hi) a backward part delivers to rank g (halo planes included)
inline void alltoall_part_planes(int Nt, int W, int g, int part, int parts, int halo, int* lo, int* hi) {
    int t0, nl;
    split_planes(Nt, W, g, &t0, &nl);
    split_part(nl, parts, part, lo, hi);
    if (halo && part == 0 && t0 > 0) *lo -= 1;
    if (halo && part == parts - 1 && t0 + nl < Nt) *hi += 1;
}

// trajectory positions after rank j's planes -> rank j + 1 (one list per field, px and py)
inline std::vector<Xfer> relay_xfers(int64_t nxy, int j) { return {{j, j + 1, 0, 0, nxy}}; }

// the last rank's (u, v, m) -> rank 0 (one list per field)
inline std::vector<Xfer> deliver_xfers(int64_t nxy, int W) { return {{W - 1, 0, 0, 0, nxy}}; }

// in-place all-gather of `cnt` doubles per rank, as device copies (virtual ranks; RCCL runs
// one ncclAllGather instead)
inline std::vector<Xfer> allgather_xfers(int W, int cnt) {
    std::vector<Xfer> xs;
    for (int g = 0; g < W; ++g)
        for (int h = 0; h < W; ++h)
            if (g != h) xs.push_back({g, h, (int64_t)g * cnt, (int64_t)g * cnt, cnt});
    return xs;
}

// What rank `me` issues for a list over RCCL, in issue order: inside one group (when any
// transfer crosses ranks) a send for each transfer from `me` to a peer and a receive for each
// transfer from a peer to `me`, in list order; after the group, each transfer to itself as a
// device copy.
enum CallOp { CALL_SEND = 0, CALL_RECV = 1, CALL_COPY = 2 };
struct Call {
    int op, peer;
    int64_t off, n, doff;   // send / copy: source offset; recv: destination offset; copy: doff too
};

inline bool crosses_ranks(const std::vector<Xfer>& xs, int me) {
    for (const Xfer& x : xs)
        if ((x.src == me) != (x.dst == me)) return true;
    return false;
}

inline std::vector<Call> rccl_calls(const std::vector<Xfer>& xs, int me) {
    std::vector<Call> cs;
    if (crosses_ranks(xs, me))
        for (const Xfer& x : xs) {
            if (x.src == me && x.dst != me) cs.push_back({CALL_SEND, x.dst, x.soff, x.n, 0});
            if (x.dst == me && x.src != me) cs.push_back({CALL_RECV, x.src, x.doff, x.n, 0});
        }
    for (const Xfer& x : xs)
        if (x.src == me && x.dst == me) cs.push_back({CALL_COPY, me, x.soff, x.n, x.doff});
    return cs;
}

}  // namespace foto
