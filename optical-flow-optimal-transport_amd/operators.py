"""Drop-in for the reference's ``operators.py``: the same builder names and signatures,
returning scipy sparse matrices (host-side API surface; the solvers never build them).

Finite-difference conventions (h = grid step):
  grad_1d_central_weird  interior (z[k+1]-z[k-1])/(2h); bc 'N' end rows z1-z0, z[n-1]-z[n-2]
                          (not scaled by h: the reference assigns them after the /h,
                          operators.py:40-46)
  grad_1d_central        interior central; bc 'N' end rows zero; bc 'D' zero extension
  grad_1d_forward        (z[k+1]-z[k])/h; bc 'N' last row zero
  grad_1d_backward       (z[k]-z[k-1])/h; bc 'N' first row zero
  grad_1d_forward_weird / grad_1d_backward_weird   the reference's unused variants
  lap1d                  3-point Laplacian / h^2; bc 'N' one-sided end rows
  grad_st / div_st / laplacian_st / grad / grad_forward / div  Kronecker compositions,
  voxel k = n*Nx*Ny + j*Nx + i (operators.py:114-191).
The GPU computes the same operators matrix-free (foto.ops, libfoto.so).
"""
import numpy as np
from scipy import sparse


def _check(bc):
    if bc not in ("N", "D"):
        raise NotImplementedError("These boundary conditions are not implemented")


def _csr(n, rows, cols, vals):
    return sparse.csr_matrix((np.asarray(vals, dtype=np.float64), (np.asarray(rows), np.asarray(cols))),
                             shape=(n, n))


def _band(n, lower, upper, h):
    """rows k: lower*z[k-1] + upper*z[k+1], scaled by 1/h (interior pattern)."""
    k = np.arange(n)
    rows = np.concatenate([k[1:], k[:-1]])
    cols = np.concatenate([k[:-1], k[1:]])
    vals = np.concatenate([np.full(n - 1, lower / h), np.full(n - 1, upper / h)])
    return rows, cols, vals


def grad_1d_forward_weird(n, h, bc):
    _check(bc)
    D = sparse.lil_matrix(sparse.diags([-np.ones(n) / h, np.ones(n - 1) / h], [0, 1], shape=(n, n)))
    D[n - 1, n - 1] = 1
    D[n - 1, n - 2] = -1
    return D.tocsr()


def grad_1d_backward_weird(n, h, bc):
    _check(bc)
    D = sparse.lil_matrix(sparse.diags([-np.ones(n - 1) / h, np.ones(n) / h], [-1, 0], shape=(n, n)))
    D[0, 0] = -1
    D[0, 1] = 1
    return D.tocsr()


def grad_1d_central_weird(n, h, bc):
    _check(bc)
    rows, cols, vals = _band(n, -0.5, 0.5, h)
    keep = np.ones(rows.size, dtype=bool)
    if bc == "N":
        keep &= (rows != 0) & (rows != n - 1)
        rows = np.concatenate([rows[keep], [0, 0, n - 1, n - 1]])
        cols = np.concatenate([cols[keep], [0, 1, n - 1, n - 2]])
        vals = np.concatenate([vals[keep], [-1.0, 1.0, 1.0, -1.0]])
    return _csr(n, rows, cols, vals)


def grad_1d_central(n, h, bc):
    _check(bc)
    rows, cols, vals = _band(n, -0.5, 0.5, h)
    if bc == "N":
        keep = (rows != 0) & (rows != n - 1)
        rows, cols, vals = rows[keep], cols[keep], vals[keep]
    return _csr(n, rows, cols, vals)


def grad_1d_forward(n, h, bc):
    _check(bc)
    k = np.arange(n)
    rows = np.concatenate([k, k[:-1]])
    cols = np.concatenate([k, k[:-1] + 1])
    vals = np.concatenate([np.full(n, -1.0 / h), np.full(n - 1, 1.0 / h)])
    if bc == "N":
        keep = ~((rows == n - 1) & (cols == n - 1))
        rows, cols, vals = rows[keep], cols[keep], vals[keep]
    return _csr(n, rows, cols, vals)


def grad_1d_backward(n, h, bc):
    _check(bc)
    k = np.arange(n)
    rows = np.concatenate([k, k[1:]])
    cols = np.concatenate([k, k[1:] - 1])
    vals = np.concatenate([np.full(n, 1.0 / h), np.full(n - 1, -1.0 / h)])
    if bc == "N":
        keep = ~((rows == 0) & (cols == 0))
        rows, cols, vals = rows[keep], cols[keep], vals[keep]
    return _csr(n, rows, cols, vals)


def lap1d(N, dx, bc):
    _check(bc)
    h2 = dx * dx
    rows, cols, vals = _band(N, 1.0, 1.0, h2)
    diag = np.full(N, -2.0 / h2)
    if bc == "N":
        diag[0] = diag[-1] = -1.0 / h2
    k = np.arange(N)
    return _csr(N, np.concatenate([rows, k]), np.concatenate([cols, k]), np.concatenate([vals, diag]))


def _eye(n):
    return sparse.identity(n, format="csr")


def grad_st(Nt, Nx, Ny, dt, dx, dy, bc):
    Dt, Dx, Dy = grad_1d_central_weird(Nt, dt, bc), grad_1d_central_weird(Nx, dx, bc), grad_1d_central_weird(Ny, dy, bc)
    t = sparse.kron(Dt, _eye(Nx * Ny))
    x = sparse.kron(_eye(Nt), sparse.kron(_eye(Ny), Dx))
    y = sparse.kron(_eye(Nt), sparse.kron(Dy, _eye(Nx)))
    return sparse.vstack([t, x, y]).tocsr()


def div_st(Nt, Nx, Ny, dt, dx, dy, bc):
    """Same 1-D operator as grad_st, NOT -grad_st^T (operators.py:129-142)."""
    Dt, Dx, Dy = grad_1d_central_weird(Nt, dt, bc), grad_1d_central_weird(Nx, dx, bc), grad_1d_central_weird(Ny, dy, bc)
    t = sparse.kron(Dt, _eye(Nx * Ny))
    x = sparse.kron(_eye(Nt), sparse.kron(_eye(Ny), Dx))
    y = sparse.kron(_eye(Nt), sparse.kron(Dy, _eye(Nx)))
    return sparse.hstack([t, x, y]).tocsr()


def laplacian_st(Nt, Nx, Ny, dt, dx, dy, bc):
    Lx, Ly, Lt = lap1d(Nx, dx, bc), lap1d(Ny, dy, bc), lap1d(Nt, dt, bc)
    Lspace = sparse.kron(_eye(Ny), Lx) + sparse.kron(Ly, _eye(Nx))
    return (sparse.kron(Lt, _eye(Nx * Ny)) + sparse.kron(_eye(Nt), Lspace)).tocsr()


def grad(Nx, Ny, dx, dy, bc):
    Dx, Dy = grad_1d_central(Nx, dx, bc), grad_1d_central(Ny, dy, bc)
    return sparse.vstack([sparse.kron(_eye(Ny), Dx), sparse.kron(Dy, _eye(Nx))]).tocsr()


def grad_forward(Nx, Ny, dx, dy, bc="N"):
    Dx, Dy = grad_1d_forward(Nx, dx, bc), grad_1d_forward(Ny, dy, bc)
    return sparse.vstack([sparse.kron(_eye(Ny), Dx), sparse.kron(Dy, _eye(Nx))]).tocsr()


def div(Nx, Ny, dx, dy, bc):
    Dx, Dy = grad_1d_central(Nx, dx, bc), grad_1d_central(Ny, dy, bc)
    return sparse.hstack([sparse.kron(_eye(Ny), Dx), sparse.kron(Dy, _eye(Nx))]).tocsr()
