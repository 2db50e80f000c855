"""Drop-in for the reference's ``main.py`` CLI (main.py:27-148): same flags, same stdout,
same output files (.flo, benchmark txt, reconstruction / luminosity PNGs).  The solvers run
on the GPU; ``--device`` and ``--cg-mode`` are additions.

    python main.py frame10.png frame11.png --algo=foto --Nt=16 --r=1 \
        --convergence-tol=0.01 --reg-epsilon=1e-2 --max-it=200 --out=foto.flo
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
from PIL import Image  # noqa: E402

import utils  # noqa: E402
import benamou_brenier  # noqa: E402
import classical  # noqa: E402


def build_parser():
    p = argparse.ArgumentParser(description="sample argument parser")
    p.add_argument("f0", help="first frame")
    p.add_argument("f1", help="second frame")
    p.add_argument("--out", nargs="?", help="optical flow output")
    p.add_argument("--ground-truth", nargs="?", help="optical flow ground truth")
    p.add_argument("--save-benchmark", nargs="?", help="file output of benchmark")
    p.add_argument("--save-reconstruction", nargs="?", help="file output of reconstruction")
    p.add_argument("--save-lum", nargs="?", help="file output of luminosity")
    p.add_argument("--algo", nargs="?", help="Algorithm")
    p.add_argument("--Nt", nargs="?", type=int, default=4, help="Discretization in time")
    p.add_argument("--r", nargs="?", type=float, default=1., help="augmented langrangian parameter")
    p.add_argument("--convergence-tol", nargs="?", type=float, default=0.1, help="Stopping threshold")
    p.add_argument("--reg-epsilon", nargs="?", type=float, default=1e-3,
                   help="Regularization for the step 1 of Benamou-Brenier")
    p.add_argument("--max-it", nargs="?", type=int, default=100, help="Maximal number of iteration")
    p.add_argument("--normalize", action=argparse.BooleanOptionalAction, help="normalize the input images if enabled")
    p.add_argument("--alpha", nargs="?", type=float, default=0.1, help="Horn-Schunck alpha")
    p.add_argument("--lambdaa", nargs="?", type=float, default=0.2, help="Horn-Schunck lambda")
    # additions
    p.add_argument("--device", type=int, default=-1, help="HIP device ordinal (default: current)")
    p.add_argument("--cg-mode", type=int, default=None, help="0 stencil, 1 spectral, 2 spectral s-step, 3 Gauss-compressed spectral CG (default)")
    return p


def _save_gray(img, w, h, path):
    Image.fromarray(img.reshape([h, w]), "L").save(path)


def main(argv=None, writer=None):
    """``writer``: an executor (run.py passes a one-thread pool) that takes the output-file
    writes (.flo, PNGs) off this thread, so the encoding overlaps the next solve; the files
    are the same.  None: written here, before main returns, as the reference does."""
    args = build_parser().parse_args(argv)

    def emit(fn, *a):
        if writer is None:
            fn(*a)
        else:
            writer.submit(fn, *a)

    np.random.seed(0)
    f1, w, h = utils.openGrayscaleImage(args.f0)
    f2, w, h = utils.openGrayscaleImage(args.f1)

    print("***********************************")
    print("Input images: ")
    print(" - f0 = " + str(args.f0) + " / total mass = " + str(np.sum(f1)))
    print(" - f1 = " + str(args.f1) + " / total mass = " + str(np.sum(f2)))
    if args.normalize is True:
        print(" - normalize input images")
        rho1 = f1 / (np.sum(f1))
        rho2 = f2 / (np.sum(f2))
    else:
        rho1 = f1
        rho2 = f2

    start_time = time.time()
    if args.algo == "foto":
        print(" - algorithm: FOTO")
        print(f"\t - Nt={args.Nt}")
        print(f"\t - r={args.r}")
        print(f"\t - convergence_tol={args.convergence_tol}")
        print(f"\t - reg_epsilon={args.reg_epsilon}")
        print(f"\t - max_it={args.max_it}")
        opts = {"device": args.device}
        if args.cg_mode is not None:
            opts["cg_mode"] = args.cg_mode
        u, v, m = benamou_brenier.solve(rho1, rho2, args.Nt, w, h, r=args.r, convergence_tol=args.convergence_tol,
                                        reg_epsilon=args.reg_epsilon, max_it=args.max_it, **opts)
    elif args.algo == "GN":
        print(" - algorithm: GN")
        print(f"\t - alpha={args.alpha}")
        print(f"\t - lambda={args.lambdaa}")
        gn = classical.GLLOpticalFlow(w, h)
        gn.setAlpha(args.alpha)
        gn.setLambda(args.lambdaa)
        [u, v, m] = gn.assemble(rho1, rho2).process()
    else:
        # reference: `assert("not implemented")` (always true), then NameError on `u` below
        raise NotImplementedError(f"algorithm {args.algo!r} is not implemented (use --algo=foto or --algo=GN)")
    timer = time.time() - start_time

    print("Benchmark:")
    rec = utils.apply_opticalflow(f1, u, v, w, h, m)
    rec = np.clip(rec, 0, 1)
    IE = utils.IE(w, h, rec, f2)
    print(" - time: " + str(timer) + "s")
    print(" - IE: " + str(IE))

    if args.ground_truth:
        wGT, hGT, uGT, vGT = utils.openFlo(args.ground_truth)
        assert wGT == w and hGT == h
        AEE, SDEE = utils.EE(w, h, u, v, uGT, vGT)
        AAE, SDAE = utils.AE(w, h, u, v, uGT, vGT)
        print(" - EE-mean: " + str(AEE))
        print(" - EE-stddev: " + str(SDEE))
        print(" - AE-mean: " + str(AAE))
        print(" - AE-stddev: " + str(SDAE))

    if args.save_benchmark:
        with open(args.save_benchmark, "w") as f:
            if args.ground_truth:
                f.write("EE-mean: " + str(AEE) + "\n")
                f.write("EE-stddev: " + str(SDEE) + "\n")
                f.write("AE-mean: " + str(AAE) + "\n")
                f.write("AE-stddev: " + str(SDAE) + "\n")
            f.write("IE: " + str(IE) + "\n")
            f.write("time: " + str(timer) + "s")

    if args.out:
        print("saving flo file...")
        emit(utils.saveFlo, w, h, u, v, args.out)

    if args.save_reconstruction:
        print("saving reconstruction...")
        emit(_save_gray, np.uint8(255 * rec), w, h, args.save_reconstruction)

    if args.save_lum:
        print("saving luminosity...")
        emit(_save_gray, np.uint8(255 * np.clip((m + 1) / 2, 0, 1)), w, h, args.save_lum)

    print("***********************************")
    return u, v, m


if __name__ == "__main__":
    main()
