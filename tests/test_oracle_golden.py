"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.npz,
produced by tests/golden/make_golden.py from /root/reference).  CPU only."""
import io
import contextlib

import numpy as np
import pytest

from oracle import foto_oracle as O


def _grids(d):
    k = 0
    while f"g{k}_shape" in d:
        yield k, tuple(int(s) for s in d[f"g{k}_shape"])
        k += 1


def test_ops_space_time(gold):
    d = gold("ops.npz")
    n = 0
    for k, (Nt, Ny, Nx) in _grids(d):
        phi, w = d[f"g{k}_phi"], d[f"g{k}_w"]
        np.testing.assert_allclose(O.grad_st(phi, Nt, Ny, Nx), d[f"g{k}_grad_st"], rtol=0, atol=1e-13)
        np.testing.assert_allclose(O.div_st(w, Nt, Ny, Nx), d[f"g{k}_div_st"], rtol=0, atol=1e-13)
        np.testing.assert_allclose(O.apply_laplacian_st(phi, Nt, Ny, Nx), d[f"g{k}_lap_st"], rtol=0, atol=1e-13)
        for r, eps in [(1.0, 1e-2), (1.7, 1e-3)]:
            np.testing.assert_allclose(O.apply_A(phi, r, eps, Nt, Ny, Nx), d[f"g{k}_A_{r}_{eps}"], rtol=0, atol=1e-12)
            A = O.assemble_A(r, eps, Nt, Ny, Nx)
            np.testing.assert_allclose(A @ phi, d[f"g{k}_A_{r}_{eps}"], rtol=0, atol=1e-12)
        n += 1
    assert n == 4


def test_ops_2d(gold):
    d = gold("ops.npz")
    for k, (Nt, Ny, Nx) in _grids(d):
        f = d[f"g{k}_phi"][: Nx * Ny]
        uv = d[f"g{k}_w"][: 2 * Nx * Ny]
        np.testing.assert_allclose(O.grad2_central(f, Nx, Ny, "N"), d[f"g{k}_grad2_N"], atol=1e-14, rtol=0)
        np.testing.assert_allclose(O.grad2_central(f, Nx, Ny, "D"), d[f"g{k}_grad2_D"], atol=1e-14, rtol=0)
        np.testing.assert_allclose(O.div2_central(uv, Nx, Ny, "D"), d[f"g{k}_div2_D"], atol=1e-14, rtol=0)
        np.testing.assert_allclose(O.div2_central(uv, Nx, Ny, "N"), d[f"g{k}_div2_N"], atol=1e-14, rtol=0)
        np.testing.assert_allclose(O.grad2_forward(f, Nx, Ny), d[f"g{k}_gradf_N"], atol=1e-14, rtol=0)


def test_ops_1d_dense(gold):
    d = gold("ops.npz")
    for n in (2, 3, 5):
        for h in (1.0, 0.5):
            eye = np.eye(n)
            cw = np.stack([O.d1_central_weird(eye[:, j], 0, h) for j in range(n)], axis=1)
            np.testing.assert_array_equal(cw, d[f"d1_cw_{n}_{h}"])
            for bc in ("N", "D"):
                c = np.stack([O.d1_central(eye[:, j], 0, bc, h) for j in range(n)], axis=1)
                np.testing.assert_array_equal(c, d[f"d1_c_{bc}_{n}_{h}"])
            lap = np.stack([O.d1_lap(eye[:, j], 0, h) for j in range(n)], axis=1)
            np.testing.assert_array_equal(lap, d[f"d1_lap_N_{n}_{h}"])


def test_bc_errors():
    with pytest.raises(NotImplementedError):
        O.d1_central(np.zeros(4), 0, "X")


def test_stepb(gold):
    d = gold("stepb.npz")
    M = int(d["M"])
    q = O.stepB(d["p"], M)
    np.testing.assert_allclose(q, d["q"], rtol=0, atol=1e-12)


def test_stepb_is_projection(gold):
    d = gold("stepb.npz")
    M = int(d["M"])
    q = O.stepB(d["p"], M)
    a, b1, b2 = q[:M], q[M:2 * M], q[2 * M:]
    assert np.all(a + 0.5 * (b1 ** 2 + b2 ** 2) <= 1e-12)
    # idempotence: projecting a projected point is the identity (up to the boundary rounding)
    q2 = O.stepB(q, M)
    np.testing.assert_allclose(q2, q, atol=1e-10, rtol=0)


def test_cg(gold):
    d = gold("cg.npz")
    for c in range(3):
        Nt, Ny, Nx = (int(s) for s in d[f"c{c}_shape"])
        r, eps = d[f"c{c}_r_eps"]
        A = O.assemble_A(r, eps, Nt, Ny, Nx)
        x, info, its = O.cg(A.dot, d[f"c{c}_b"], rtol=1e-6, maxiter=1000)
        assert info == int(d[f"c{c}_info"])
        assert its == int(d[f"c{c}_its"])
        np.testing.assert_allclose(x, d[f"c{c}_x"], rtol=0, atol=1e-12)
        # matrix-free matvec: same iterates up to rounding; CG amplifies a last-bit change
        # in the matvec to ~1e-9 relative in x (kappa ~ 12/eps), so the bar is 1e-8 * max|x|
        x2, info2, its2 = O.cg(lambda p: O.apply_A(p, r, eps, Nt, Ny, Nx), d[f"c{c}_b"])
        assert its2 == its
        np.testing.assert_allclose(x2, d[f"c{c}_x"], rtol=0, atol=1e-8 * np.abs(d[f"c{c}_x"]).max())
        x5, info5, its5 = O.cg(A.dot, d[f"c{c}_b"], rtol=1e-6, maxiter=5)
        assert info5 == int(d[f"c{c}_info_max5"]) == 5
        np.testing.assert_allclose(x5, d[f"c{c}_x_max5"], rtol=0, atol=1e-12)


def test_bb_step(gold):
    d = gold("bbstep.npz")
    Nt, Ny, Nx = (int(s) for s in d["shape"])
    r, eps = d["r_eps"]
    F = O.bb_rhs(d["mu"], d["q"], d["rho0"], d["rhoT"], r, Nt, Ny, Nx)
    np.testing.assert_allclose(F, d["F"], rtol=0, atol=1e-13)
    A = O.assemble_A(r, eps, Nt, Ny, Nx)
    phi, info, its = O.solve_step(d["mu"], d["q"], d["rho0"], d["rhoT"], r, A.dot, Nt, Ny, Nx)
    np.testing.assert_allclose(phi, d["phi"], rtol=0, atol=1e-10)


def test_flow(gold):
    d = gold("flow.npz")
    for f in range(4):
        Nt, Ny, Nx = (int(s) for s in d[f"f{f}_shape"])
        u, v, m = O.flow_from_phi(d[f"f{f}_phi"], Nt, Nx, Ny)
        np.testing.assert_array_equal(u, d[f"f{f}_u"])
        np.testing.assert_array_equal(v, d[f"f{f}_v"])
        np.testing.assert_allclose(m, d[f"f{f}_m"], rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize("name", ["bb_small.npz", "bb_tex.npz"])
def test_bb_solve_small(gold, name):
    d = gold(name)
    Nt, Ny, Nx = (int(s) for s in d["shape"])
    r, tol, eps, max_it = d["params"]
    buf = io.StringIO()
    stats = {}
    with contextlib.redirect_stdout(buf):
        u, v, m = O.solve(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, convergence_tol=tol, reg_epsilon=eps,
                          max_it=int(max_it), stats=stats)
    assert list(stats["cg_its"]) == list(d["cg_its"])
    np.testing.assert_allclose(stats["crit"], d["crit"], rtol=1e-9, atol=0)
    np.testing.assert_allclose(stats["phi"], d["phi"], rtol=0, atol=1e-9)
    for a, b in ((u, d["u"]), (v, d["v"]), (m, d["m"])):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-9)
    # stdout lines have the reference format
    lines = buf.getvalue().splitlines()
    assert len(lines) == len(d["crit"])
    assert lines[0].endswith(f"(1/{int(max_it)})")


@pytest.mark.slow
def test_bb_solve_c1(gold):
    d = gold("bb_c1.npz")
    Nt, Ny, Nx = (int(s) for s in d["shape"])
    r, tol, eps, max_it = d["params"]
    stats = {}
    u, v, m = O.solve(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, convergence_tol=tol, reg_epsilon=eps,
                      max_it=int(max_it), stats=stats, log=lambda s: None)
    assert len(stats["crit"]) == len(d["crit"]) == 46
    assert np.max(np.abs(np.array(stats["cg_its"]) - d["cg_its"])) <= 1
    np.testing.assert_allclose(stats["crit"], d["crit"], rtol=1e-7, atol=0)
    for a, b in ((u, d["u"]), (v, d["v"]), (m, d["m"])):
        np.testing.assert_allclose(a, b, rtol=0, atol=1e-7)


def test_gn(gold):
    d = gold("gn.npz")
    for g in range(2):
        w, h = (int(s) for s in d[f"n{g}_wh"])
        alpha, lam = d[f"n{g}_alpha_lambda"]
        f1, f2 = d[f"n{g}_f1"], d[f"n{g}_f2"]
        A, b = O.gn_assemble(f1, f2, w, h, alpha, lam)
        np.testing.assert_allclose(A @ d[f"n{g}_x"], d[f"n{g}_Ax"], rtol=0, atol=1e-13)
        np.testing.assert_allclose(O.gn_apply(d[f"n{g}_x"], f1, f2, w, h, alpha, lam), d[f"n{g}_Ax"],
                                   rtol=0, atol=1e-13)
        np.testing.assert_allclose(b, d[f"n{g}_b"], rtol=0, atol=0)
        u, v, m = O.gn_solve(f1, f2, w, h, alpha, lam)
        for a, ref in ((u, d[f"n{g}_u"]), (v, d[f"n{g}_v"]), (m, d[f"n{g}_m"])):
            np.testing.assert_allclose(a, ref, rtol=0, atol=1e-8)


@pytest.mark.slow
def test_reference_rounding_sensitivity(gold):
    """Documents the parity bar of the full solve: changing only the rounding of A p
    (matrix-free stencil instead of scipy CSR) moves CG counts by one and crit by ~1e-6
    relative in the reference algorithm itself."""
    d = gold("bb_c1.npz")
    Nt, Ny, Nx = (int(s) for s in d["shape"])
    r, tol, eps, max_it = d["params"]
    st = {}
    u, v, m = O.solve(d["rho0"], d["rhoT"], Nt, Nx, Ny, r=r, convergence_tol=tol, reg_epsilon=eps,
                      max_it=int(max_it), stats=st, log=lambda s: None, assembled=False)
    dk = np.abs(np.array(st["cg_its"]) - d["cg_its"])
    rel = np.max(np.abs(st["crit"] / d["crit"] - 1))
    assert dk.max() <= 1 and 1e-7 < rel < 1e-5
    assert np.abs(u - d["u"]).max() < 1e-5
