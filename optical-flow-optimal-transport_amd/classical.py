"""Drop-in for the reference's ``classical.py``: the Gennert-Negahdaripour variational
flow with a multiplicative brightness term (classical.py:25-130), solved on the GPU.

``process`` replaces SuperLU's direct solve with conjugate gradients preconditioned by
a multigrid V-cycle (replayed as a hipGraph) in libfoto.so (relative residual 1e-10 by
default; agrees with spsolve to ~1e-8).  ``A`` and ``b`` are still available as attributes, assembled on the host on
first access, for callers that inspect the system.
"""
import sys

import numpy as np

from foto import gn as _gn


class GLLOpticalFlow(object):
    """Gennert and Negahdaripour Optical Flow Estimator."""
    NAME = "GLL"
    LUMINOSITY = True

    def __init__(self, w=0, h=0):
        self.w = w
        self.h = h
        self.alpha = 0.1
        self.rtol = _gn.GN_RTOL
        self.maxiter = _gn.GN_MAXITER
        self.iterations = None

    def setAlpha(self, alpha):
        self.alpha = alpha

    def setLambda(self, lambdap):
        self.lambdap = lambdap

    def assemble(self, f1, f2):
        """Stores the frames (the system is applied matrix-free on the GPU).  Like the
        reference, requires setLambda first (AttributeError otherwise)."""
        self.lambdap = self.lambdap   # reference: AttributeError when setLambda was never called
        n = self.w * self.h
        self.f1 = np.ascontiguousarray(np.asarray(f1, dtype=np.float64).reshape(-1)[:n])
        self.f2 = np.ascontiguousarray(np.asarray(f2, dtype=np.float64).reshape(-1)[:n])
        self._A = None
        return self

    # host-side view of the assembled system (classical.py:88-111)
    def _assemble_host(self):
        # scipy only here: importing it costs ~0.3 s per process, a tenth of a batch worker's run
        from scipy import sparse
        import operators
        w, h = self.w, self.h
        f1, f2 = self.f1, self.f2
        F2 = f2.reshape(h, w)
        fx = np.zeros((h, w))
        fy = np.zeros((h, w))
        fx[:, 1:-1] = 0.5 * (F2[:, 2:] - F2[:, :-2])
        fy[1:-1, :] = 0.5 * (F2[2:, :] - F2[:-2, :])
        fx, fy = fx.ravel(), fy.ravel()
        ft = f2 - f1
        G = operators.grad_forward(w, h, 1, 1)
        lap = (-G.transpose()) @ G
        d = sparse.diags
        self._A = sparse.bmat([[-self.alpha * lap + d(fx ** 2), d(fx * fy), d(-fx * f2)],
                               [d(fy * fx), -self.alpha * lap + d(fy ** 2), d(-fy * f2)],
                               [d(-f2 * fx), d(-f2 * fy), -self.lambdap * lap + d(f2 ** 2)]]).tocsr()
        self._b = np.hstack((-fx * ft, -fy * ft, f2 * ft))

    @property
    def A(self):
        if getattr(self, "_A", None) is None:
            self._assemble_host()
        return self._A

    @property
    def b(self):
        if getattr(self, "_A", None) is None:
            self._assemble_host()
        return self._b

    def process(self):
        """Solve for [u, v, m] on the GPU.  The solver plan (device buffers, multigrid levels,
        the replayed PCG graph) comes from a process-wide cache keyed by (w, h, alpha, lambda,
        rtol, maxiter) (foto.gn.cached_plan), so every instance with the same size and
        parameters -- a batch of frames -- shares one."""
        plan = _gn.cached_plan(self.w, self.h, self.alpha, self.lambdap, self.rtol, self.maxiter)
        u, v, m, info, its = plan.solve(self.f1, self.f2)
        self.iterations = its
        if info > 0:
            # stderr: the reference (spsolve) never prints here, so stdout stays identical
            print(f"WARNING: GN PCG did not converge in {info} iterations.", file=sys.stderr)
        return [u, v, m]
