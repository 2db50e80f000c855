"""Generate the golden vectors that pin the oracle (and through it the HIP path).

Run ONCE in the build container, where the reference is mounted read-only at
/root/reference and importable (importing it works, no
permission denial).  It never runs on the GPU box and nothing under tests/
imports it; the committed output is data only (inputs + the reference's
outputs), written to tests/golden/*.npz.

    python tests/golden/make_golden.py [--ref /root/reference] [--skip-c1]

Cases (SURVEY.md §8(c) "Golden vectors to generate"):
  ops.npz        A1-A5, A12, grad_forward applied to seeded fields on several
                 small grids (incl. the minimum sizes 2 and odd sizes)
  stepb.npz      A8 stepB on crafted branch points + random N(0, 3^2) points
  cg.npz         A6/A7: scipy cg on A = -r L + r eps I (x, info, iteration count)
  bbstep.npz     A6 solve_benamou_brenier_step for a random (mu, q) state
  flow.npz       A13/A14 opticalflow_from_benamoubrenier for given phi fields
  bb_small.npz   full solve() on 20x16x4 (stdout crit lines, cg counts, phi, u, v, m)
  bb_c1.npz      full solve() on C1 64x64x8, run.sh params (r=1, tol=0.01,
                 eps=1e-2, max_it=100) -- 46 outer iterations, ~25 s
  gn.npz         GLLOpticalFlow assemble A@x, b, process() u, v, m on 40x30 and 17x13
  io.npz         saveFlo bytes, openFlo round trip, EE/AE/IE, apply_opticalflow
  cli.npz        main.py's pipeline on a 36x28 PNG pair (FOTO Nt=4, 8 its; GN): flows, IE, .flo bytes
  bb_metric.npz  the bench grid 640x480x32 (SURVEY.md §8(d) S-metric), run.sh params, max_it=2
                 (~5 min): crit lines, CG counts, strided subsamples of phi after each
                 outer iteration and of the final u, v, m
  bb_c2s.npz     a Dimetrodon-shaped small grid 146x194x4 whose DCT half-lengths carry the
                 prime factors 73 and 97 of the C2 grid 584x388 (textured pair, 10 its;
                 phi, u, v, m every 5th value)
  gn_c3.npz      GN at the C3 size 640x480 (sinusoid pair; SuperLU ~75 s): u, v, m subsample
  bin.npz        the dataset-prep scripts bin/normalize_image.py, create_lum_dataset.py and
                 data_diff.py run on a 48x40 PNG pair (decoded output pixels), and bash's
                 RANDOM sequence after RANDOM=12345 (run.sh:33 seeds create_lum_dataset)
"""
import argparse
import contextlib
import io
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "optical-flow-optimal-transport_amd"))
from foto.synthetic import translating_gaussian, sinusoid_pair, textured_pair  # noqa: E402


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


def gen_ops(operators, rng):
    out = {}
    grids = [(5, 6, 7), (2, 3, 2), (3, 2, 5), (4, 9, 8)]
    for gi, (Nt, Ny, Nx) in enumerate(grids):
        N = Nt * Nx * Ny
        phi = rng.standard_normal(N)
        w = rng.standard_normal(3 * N)
        G = operators.grad_st(Nt, Nx, Ny, 1, 1, 1, bc="N")
        D = operators.div_st(Nt, Nx, Ny, 1, 1, 1, bc="N")
        L = operators.laplacian_st(Nt, Nx, Ny, 1, 1, 1, bc="N")
        out[f"g{gi}_shape"] = np.array([Nt, Ny, Nx])
        out[f"g{gi}_phi"] = phi
        out[f"g{gi}_w"] = w
        out[f"g{gi}_grad_st"] = G @ phi
        out[f"g{gi}_div_st"] = D @ w
        out[f"g{gi}_lap_st"] = L @ phi
        for r, eps in [(1.0, 1e-2), (1.7, 1e-3)]:
            A = -r * L + r * eps * __import__("scipy").sparse.eye(N)
            out[f"g{gi}_A_{r}_{eps}"] = A @ phi
        # 2-D operators on the first slab (Nx*Ny)
        f = phi[: Nx * Ny]
        uv = w[: 2 * Nx * Ny]
        out[f"g{gi}_grad2_N"] = operators.grad(Nx, Ny, 1, 1, bc="N") @ f
        out[f"g{gi}_grad2_D"] = operators.grad(Nx, Ny, 1, 1, bc="D") @ f
        out[f"g{gi}_div2_D"] = operators.div(Nx, Ny, 1, 1, bc="D") @ uv
        out[f"g{gi}_div2_N"] = operators.div(Nx, Ny, 1, 1, bc="N") @ uv
        out[f"g{gi}_gradf_N"] = operators.grad_forward(Nx, Ny, 1, 1) @ f
    # 1-D building blocks as dense matrices (small)
    for n in (2, 3, 5):
        for h in (1.0, 0.5):
            out[f"d1_cw_{n}_{h}"] = operators.grad_1d_central_weird(n, h, "N").toarray()
            out[f"d1_c_N_{n}_{h}"] = operators.grad_1d_central(n, h, "N").toarray()
            out[f"d1_c_D_{n}_{h}"] = operators.grad_1d_central(n, h, "D").toarray()
            out[f"d1_f_N_{n}_{h}"] = operators.grad_1d_forward(n, h, "N").toarray()
            out[f"d1_lap_N_{n}_{h}"] = operators.lap1d(n, h, "N").toarray()
            out[f"d1_lap_D_{n}_{h}"] = operators.lap1d(n, h, "D").toarray()
    save("ops.npz", **out)


def gen_stepb(bb, rng):
    crafted = [
        # inside K: 2a + |b|^2 <= 0
        (-1.0, 0.1, 0.2), (-5.0, 1.0, -2.0), (0.0, 0.0, 0.0), (-0.5, 1.0, 0.0),  # last: boundary 2a+|b|^2 = 0
        # Cardano branch (outside, -32(a+1)^3 - 108 rho^2 < 0)
        (1.0, 0.0, 0.0), (0.5, 1.0, 1.0), (3.0, -2.0, 0.5), (-0.9, 2.0, 0.0), (10.0, 0.0, 3.0),
        (0.0, 1e-8, 0.0), (2.0, 0.0, -0.0), (-0.2, 0.0, 1.0),
        # trigonometric branch (outside, a < -1, small rho)
        (-1.5, 1.2, 0.0), (-3.0, 1.0, 2.3), (-2.0, -1.9, 0.5), (-1.1, 0.0, 0.47), (-8.0, 3.9, 0.1),
    ]
    pts = np.array(crafted, dtype=np.float64)
    rnd = 3.0 * rng.standard_normal((1500, 3))
    pts = np.concatenate([pts, rnd], axis=0)
    M = pts.shape[0]
    p = np.concatenate([pts[:, 0], pts[:, 1], pts[:, 2]])
    # stepB(p, Nt, Nx, Ny) only uses Nt*Nx*Ny = M
    q = bb.stepB(p, 1, M, 1)
    save("stepb.npz", p=p, q=q, M=np.array(M))


def count_cg(spla):
    """Wrap scipy cg to record (x, info, iterations) for each call."""
    calls = []
    real = spla.cg

    def cg(A, b, **kw):
        n = [0]

        def cb(xk):
            n[0] += 1
        x, info = real(A, b, callback=cb, **kw)
        calls.append((int(info), n[0]))
        return x, info
    return cg, calls


def gen_cg(operators, rng):
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    out = {}
    for ci, (Nt, Ny, Nx, r, eps) in enumerate([(5, 6, 7, 1.0, 1e-2), (8, 12, 16, 1.0, 1e-3), (4, 10, 9, 2.5, 1e-2)]):
        N = Nt * Nx * Ny
        L = operators.laplacian_st(Nt, Nx, Ny, 1, 1, 1, bc="N")
        A = -r * L + r * eps * sp.eye(N)
        b = rng.standard_normal(N)
        n = [0]
        x, info = spla.cg(A, b, rtol=1e-6, maxiter=1000, callback=lambda xk: n.__setitem__(0, n[0] + 1))
        out[f"c{ci}_shape"] = np.array([Nt, Ny, Nx])
        out[f"c{ci}_r_eps"] = np.array([r, eps])
        out[f"c{ci}_b"] = b
        out[f"c{ci}_x"] = x
        out[f"c{ci}_info"] = np.array(info)
        out[f"c{ci}_its"] = np.array(n[0])
        # maxiter-limited run (info > 0 path)
        n2 = [0]
        x2, info2 = spla.cg(A, b, rtol=1e-6, maxiter=5, callback=lambda xk: n2.__setitem__(0, n2[0] + 1))
        out[f"c{ci}_x_max5"] = x2
        out[f"c{ci}_info_max5"] = np.array(info2)
    save("cg.npz", **out)


def gen_bbstep(bb, operators, rng):
    import scipy.sparse as sp
    Nt, Ny, Nx = 6, 10, 12
    N = Nt * Nx * Ny
    r, eps = 1.3, 1e-2
    rho0, rhoT = translating_gaussian(Nx, Ny)
    mu = np.abs(rng.standard_normal(3 * N))
    q = rng.standard_normal(3 * N)
    D = operators.div_st(Nt, Nx, Ny, 1, 1, 1, bc="N")
    L = operators.laplacian_st(Nt, Nx, Ny, 1, 1, 1, bc="N")
    A = -r * L + r * eps * sp.eye(N)
    phi = bb.solve_benamou_brenier_step(mu, q, rho0, rhoT, r, A, D, Nt, Nx, Ny, 1, 1, 1)
    # the RHS alone (F = div(mu - r q) + BC correction), restated here only to record it
    F = D @ (mu - r * q)
    nxy = Nx * Ny
    F[:nxy] -= rho0 - mu[:nxy] + r * q[:nxy]
    F[(Nt - 1) * nxy:Nt * nxy] += rhoT - mu[(Nt - 1) * nxy:Nt * nxy] + r * q[(Nt - 1) * nxy:Nt * nxy]
    save("bbstep.npz", shape=np.array([Nt, Ny, Nx]), r_eps=np.array([r, eps]), rho0=rho0, rhoT=rhoT,
         mu=mu, q=q, F=F, phi=phi)


def gen_flow(utils, operators, rng):
    out = {}
    cases = [(4, 10, 12, 1.0), (6, 9, 7, 25.0), (2, 5, 6, 3.0), (5, 16, 20, 60.0)]
    for fi, (Nt, Ny, Nx, scale) in enumerate(cases):
        N = Nt * Nx * Ny
        phi = scale * rng.standard_normal(N)
        grad = operators.grad(Nx, Ny, 1, 1, bc="N")
        div = operators.div(Nx, Ny, 1, 1, bc="D")
        u, v, m = utils.opticalflow_from_benamoubrenier(phi, Nt, Nx, Ny, grad, div)
        out[f"f{fi}_shape"] = np.array([Nt, Ny, Nx])
        out[f"f{fi}_phi"] = phi
        out[f"f{fi}_u"] = np.asarray(u)
        out[f"f{fi}_v"] = np.asarray(v)
        out[f"f{fi}_m"] = np.asarray(m)
    save("flow.npz", **out)


def run_solve(bb, spla_mod, rho0, rhoT, Nt, Nx, Ny, **kw):
    cg_wrapped, calls = count_cg(spla_mod)
    real_cg = bb.cg
    bb.cg = cg_wrapped
    captured = {}
    real_flow = bb.utils.opticalflow_from_benamoubrenier

    def flow(phi, *a):
        captured["phi"] = np.array(phi)
        return real_flow(phi, *a)
    bb.utils.opticalflow_from_benamoubrenier = flow
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            u, v, m = bb.solve(rho0, rhoT, Nt, Nx, Ny, **kw)
    finally:
        bb.cg = real_cg
        bb.utils.opticalflow_from_benamoubrenier = real_flow
    lines = buf.getvalue().splitlines()
    crit = np.array([float(l.split(" ")[0]) for l in lines if l.endswith(")")])
    return dict(u=np.asarray(u), v=np.asarray(v), m=np.asarray(m), phi=captured["phi"],
                crit=crit, stdout=np.array(buf.getvalue()),
                cg_info=np.array([c[0] for c in calls]), cg_its=np.array([c[1] for c in calls]))


def gen_bb(bb, name, Nt, Nx, Ny, pair="gauss", stride=0, **kw):
    """stride > 0: keep every stride-th value of phi, u, v, m and no inputs (large grids; the
    inputs are the deterministic synthetic pair, recorded by their sums)."""
    import scipy.sparse.linalg as spla
    if pair == "gauss":
        rho0, rhoT = translating_gaussian(Nx, Ny)
    else:
        rho0, rhoT = textured_pair(Nx, Ny, seed=3, dx=1.5, dy=0.5)
    res = run_solve(bb, spla, rho0, rhoT, Nt, Nx, Ny, **kw)
    params = np.array([kw.get("r", 1), kw.get("convergence_tol", 0.3), kw.get("reg_epsilon", 1e-3),
                       kw.get("max_it", 100)], dtype=np.float64)
    if stride:
        for k in ("phi", "u", "v", "m"):
            res[k] = res[k][::stride]
        save(name, shape=np.array([Nt, Ny, Nx]), params=params, stride=np.array(stride),
             rho_sum=np.array([rho0.sum(), rhoT.sum()]), **res)
    else:
        save(name, shape=np.array([Nt, Ny, Nx]), params=params, rho0=rho0, rhoT=rhoT, **res)
    print(f"  {name}: {len(res['crit'])} outer its, cg its {res['cg_its'].tolist()}")


# strides of the bench-grid subsamples: primes, so the samples walk every x, y and t phase
METRIC_PHI_STRIDE = 499
METRIC_FLOW_STRIDE = 37


def gen_metric(bb):
    """640x480x32, the bench workload (bench.py): 2 outer iterations."""
    import scipy.sparse.linalg as spla
    Nt, Nx, Ny = 32, 640, 480
    rho0, rhoT = translating_gaussian(Nx, Ny)
    xs = []
    real = spla.cg

    def cg_keep(A, b, **kw):
        x, info = real(A, b, **kw)
        xs.append(np.array(x[::METRIC_PHI_STRIDE]))
        return x, info
    spla_shim = type("S", (), {"cg": staticmethod(cg_keep)})
    res = run_solve(bb, spla_shim, rho0, rhoT, Nt, Nx, Ny, r=1, convergence_tol=0.01, reg_epsilon=1e-2,
                    max_it=2)
    sub = {k: res[k][::METRIC_FLOW_STRIDE] for k in ("u", "v", "m")}
    save("bb_metric.npz", shape=np.array([Nt, Ny, Nx]), params=np.array([1.0, 0.01, 1e-2, 2.0]),
         phi_stride=np.array(METRIC_PHI_STRIDE), flow_stride=np.array(METRIC_FLOW_STRIDE),
         phi_its=np.stack(xs), crit=res["crit"], stdout=res["stdout"], cg_info=res["cg_info"],
         cg_its=res["cg_its"], rho_sum=np.array([rho0.sum(), rhoT.sum()]), **sub)
    print(f"  bb_metric.npz: crit {res['crit'].tolist()}, cg its {res['cg_its'].tolist()}")


def gen_c2s(bb):
    """Half-lengths 73 (Nx = 146) and 97 (Ny = 194): the prime factors of C2's 584x388."""
    gen_bb(bb, "bb_c2s.npz", 4, 146, 194, pair="tex", stride=5, r=1, convergence_tol=0.01, reg_epsilon=1e-2,
           max_it=10)


def gen_gn(classical, rng):
    out = {}
    for gi, (w, h) in enumerate([(40, 30), (17, 13)]):
        if gi == 0:
            f1, f2 = sinusoid_pair(w, h)
        else:
            f1, f2 = textured_pair(w, h, seed=5)
        alpha, lam = 0.1, 0.2
        g = classical.GLLOpticalFlow(w, h)
        g.setAlpha(alpha)
        g.setLambda(lam)
        g.assemble(f1, f2)
        x = rng.standard_normal(3 * w * h)
        u, v, m = g.process()
        out[f"n{gi}_wh"] = np.array([w, h])
        out[f"n{gi}_alpha_lambda"] = np.array([alpha, lam])
        out[f"n{gi}_f1"] = f1
        out[f"n{gi}_f2"] = f2
        out[f"n{gi}_x"] = x
        out[f"n{gi}_Ax"] = g.A @ x
        out[f"n{gi}_b"] = g.b
        out[f"n{gi}_u"] = u
        out[f"n{gi}_v"] = v
        out[f"n{gi}_m"] = m
    save("gn.npz", **out)


def gen_gn_c3(classical):
    """GN at the C3 (Grove2) size 640x480 on the synthetic sinusoid stand-in (SURVEY.md
    §8(d)); SuperLU takes ~75 s.  u, v, m kept every METRIC_FLOW_STRIDE-th pixel."""
    w, h, alpha, lam = 640, 480, 0.1, 0.2
    f1, f2 = sinusoid_pair(w, h)
    g = classical.GLLOpticalFlow(w, h)
    g.setAlpha(alpha)
    g.setLambda(lam)
    g.assemble(f1, f2)
    u, v, m = g.process()
    s = METRIC_FLOW_STRIDE
    save("gn_c3.npz", wh=np.array([w, h]), alpha_lambda=np.array([alpha, lam]), stride=np.array(s),
         u=np.asarray(u)[::s], v=np.asarray(v)[::s], m=np.asarray(m)[::s],
         b_norm=np.array(np.linalg.norm(g.b)))


def gen_io(utils, rng):
    w, h = 7, 5
    u = rng.standard_normal(w * h) * 3
    v = rng.standard_normal(w * h) * 3
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "x.flo")
        utils.saveFlo(w, h, u, v, p)
        flo = np.fromfile(p, dtype=np.uint8)
        w2, h2, u2, v2 = utils.openFlo(p)
    f1 = rng.random(w * h)
    f2 = rng.random(w * h)
    m = 0.1 * rng.standard_normal(w * h)
    uGT = u + 0.3 * rng.standard_normal(w * h)
    vGT = v + 0.3 * rng.standard_normal(w * h)
    uGT[3] = 1e3  # one EE > 50, ignored by EE (utils.py:311)
    ee = np.array(utils.EE(w, h, u, v, uGT, vGT))
    ae = np.array(utils.AE(w, h, u, v, uGT, vGT))
    rec = utils.apply_opticalflow(f1, u, v, w, h, m)
    ie = np.array(utils.IE(w, h, np.clip(rec, 0, 1), f2))
    save("io.npz", wh=np.array([w, h]), u=u, v=v, flo_bytes=flo, u_rt=u2, v_rt=v2, f1=f1, f2=f2, m=m,
         uGT=uGT, vGT=vGT, ee=ee, ae=ae, rec=rec, ie=ie)


def gen_cli(utils, bb, classical):
    """The computation main.py performs (main.py:52-146), reproduced by calling the
    reference functions directly (main.py itself imports cv2, absent here): PNG frames ->
    openGrayscaleImage -> solver -> apply_opticalflow / clip / IE -> saveFlo bytes."""
    from PIL import Image
    w, h = 36, 28
    a, b = textured_pair(w, h, seed=11, dx=1.2, dy=0.6)
    out = {}
    with tempfile.TemporaryDirectory() as d:
        p0, p1 = os.path.join(d, "f0.png"), os.path.join(d, "f1.png")
        Image.fromarray(np.uint8(np.round(255 * a.reshape(h, w))), "L").save(p0)
        Image.fromarray(np.uint8(np.round(255 * b.reshape(h, w))), "L").save(p1)
        out["png0"] = np.fromfile(p0, dtype=np.uint8)
        out["png1"] = np.fromfile(p1, dtype=np.uint8)
        f1, w_, h_ = utils.openGrayscaleImage(p0)
        f2, _, _ = utils.openGrayscaleImage(p1)
        for algo in ("foto", "GN"):
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                if algo == "foto":
                    u, v, m = bb.solve(f1, f2, 4, w_, h_, r=1.0, convergence_tol=0.01, reg_epsilon=1e-2, max_it=8)
                else:
                    g = classical.GLLOpticalFlow(w_, h_)
                    g.setAlpha(0.1)
                    g.setLambda(0.2)
                    u, v, m = g.assemble(f1, f2).process()
            rec = np.clip(utils.apply_opticalflow(f1, u, v, w_, h_, m), 0, 1)
            ie = utils.IE(w_, h_, rec, f2)
            fp = os.path.join(d, algo + ".flo")
            utils.saveFlo(w_, h_, u, v, fp)
            out[f"{algo}_u"], out[f"{algo}_v"], out[f"{algo}_m"] = np.asarray(u), np.asarray(v), np.asarray(m)
            out[f"{algo}_rec"], out[f"{algo}_ie"] = rec, np.array(ie)
            out[f"{algo}_flo"] = np.fromfile(fp, dtype=np.uint8)
            out[f"{algo}_stdout"] = np.array(buf.getvalue())
    out["f1"], out["f2"] = f1, f2
    save("cli.npz", **out)


def gen_bin(ref):
    """run.sh's dataset-prep scripts (bin/*.py), executed as the reference runs them."""
    import subprocess
    from PIL import Image
    yy, xx = np.mgrid[0:40, 0:48].astype(np.float64)
    a = 0.5 + 0.3 * np.sin(xx / 5.0) * np.cos(yy / 7.0) + 0.1 * np.exp(-((xx - 20) ** 2 + (yy - 18) ** 2) / 60.0)
    b = 0.5 + 0.3 * np.sin((xx - 1.5) / 5.0) * np.cos((yy - 0.5) / 7.0) + 0.1 * np.exp(-((xx - 22) ** 2 + (yy - 18) ** 2) / 60.0)
    f1 = np.uint8(np.clip(a, 0, 1) * 255)
    f2 = np.uint8(np.clip(b, 0, 1) * 255)
    out = {"f1": f1, "f2": f2}
    env = dict(os.environ, PYTHONPATH=ref)
    with tempfile.TemporaryDirectory() as td:
        p1, p2 = os.path.join(td, "frame10.png"), os.path.join(td, "frame11.png")
        Image.fromarray(f1, "L").save(p1)
        Image.fromarray(f2, "L").save(p2)

        def run(script, *args):
            subprocess.run([sys.executable, os.path.join(ref, "bin", script), *args], env=env, cwd=td, check=True)

        def load(name):
            return np.asarray(Image.open(os.path.join(td, name)).convert("L"))

        run("normalize_image.py", p1, p2, "n1.png", "n2.png")
        out["norm1"], out["norm2"] = load("n1.png"), load("n2.png")
        run("data_diff.py", p1, p2, "diff.png")
        out["diff"] = load("diff.png")
        seeds = [12345, 7, 31337]
        out["lum_seeds"] = np.array(seeds)
        for sd in seeds:
            run("create_lum_dataset.py", p2, f"lum{sd}.png", str(sd))
            out[f"lum_{sd}"] = load(f"lum{sd}.png")
    r = subprocess.run(["bash", "-c", "RANDOM=12345; for i in 1 2 3 4 5 6 7 8 9 10; do echo $RANDOM; done"],
                       capture_output=True, text=True, check=True)
    out["bash_random_12345"] = np.array([int(x) for x in r.stdout.split()])
    save("bin.npz", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--skip-c1", action="store_true")
    ap.add_argument("--metric", action="store_true", help="also the 640x480x32 bench grid (~5 min)")
    ap.add_argument("--only", help="comma-separated generators to run (e.g. bin)")
    args = ap.parse_args()
    sys.path.insert(0, args.ref)
    import operators  # noqa: F401  (reference modules)
    import utils
    import benamou_brenier as bb
    import classical
    if args.only:
        for name in args.only.split(","):
            {"bin": lambda: gen_bin(args.ref),
             "metric": lambda: gen_metric(bb),
             "c2s": lambda: gen_c2s(bb),
             "gn_c3": lambda: gen_gn_c3(classical)}[name]()
        return

    rng = np.random.default_rng(0)
    gen_ops(operators, rng)
    gen_stepb(bb, rng)
    gen_cg(operators, rng)
    gen_bbstep(bb, operators, rng)
    gen_flow(utils, operators, rng)
    gen_gn(classical, rng)
    gen_io(utils, rng)
    gen_cli(utils, bb, classical)
    gen_bb(bb, "bb_small.npz", 4, 20, 16, r=1, convergence_tol=0.01, reg_epsilon=1e-2, max_it=30)
    gen_bb(bb, "bb_tex.npz", 5, 24, 18, pair="tex", r=1.5, convergence_tol=0.05, reg_epsilon=1e-3, max_it=12)
    gen_bin(args.ref)
    gen_c2s(bb)
    if not args.skip_c1:
        gen_bb(bb, "bb_c1.npz", 8, 64, 64, r=1, convergence_tol=0.01, reg_epsilon=1e-2, max_it=100)
    if args.metric:
        gen_metric(bb)
        gen_gn_c3(classical)


if __name__ == "__main__":
    main()
