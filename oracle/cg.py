"""numpy restatement of the pathwise-conditioning step after the GRF path.

TEST INFRASTRUCTURE ONLY -- imported by ``tests/`` (the checker) and never by the
product package.

* :func:`linear_cg` restates ``linear_operator.utils.linear_cg.linear_cg`` as the
  reference calls it (``efficient_graph_gp_sparse/models/sparse_grf_model.py:43``):
  no preconditioner, no tridiagonalisation, zero initial guess.  linear_operator
  is a third-party dependency pinned through ``requirements.txt:5``
  (gpytorch==1.11 -> linear_operator 0.5.x) and is NOT installed here, so this
  restatement follows its published algorithm:
    - rhs normalised per column (norms < eps=1e-10 treated as 1 and flagged);
    - per iteration: alpha = r.r / p.Ap (0 when p.Ap < eps or the column has
      converged), r -= alpha Ap, x += alpha p, beta = r'.r' / r.r (0 when the old
      r.r < eps), p = r + beta p;
    - residual norms ||r|| (0 for zero rhs), has_converged = norm < 1e-10;
    - stop after iteration k >= min(10, max_iter - 1) once mean(norm) < tolerance
      (gpytorch.settings.cg_tolerance = 1, max_cg_iterations = 1000 by default);
    - result * rhs_norm.
  Parity of the restatement itself is unpinned (no linear_operator here and no
  fixture in the reference); it is pinned to the exact solve instead
  (tests/test_cg_oracle.py: converged CG == numpy.linalg.solve).
* :func:`pathwise_predict` restates ``SparseGraphGP.predict``
  (``models/sparse_grf_model.py:21-45``) with the random draws passed in.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def linear_cg(matmul, rhs, tolerance=1.0, eps=1e-10, stop_updating_after=1e-10, max_iter=1000, dtype=np.float64):
    """Returns (solution, iterations run)."""
    rhs = np.asarray(rhs, dtype)
    if rhs.ndim == 1:
        x, k = linear_cg(matmul, rhs[:, None], tolerance, eps, stop_updating_after, max_iter, dtype)
        return x[:, 0], k
    rhs_norm = np.linalg.norm(rhs, axis=0, keepdims=True).astype(dtype)
    rhs_is_zero = rhs_norm < eps
    rhs_norm = np.where(rhs_is_zero, dtype(1), rhs_norm)
    rhs = rhs / rhs_norm
    result = np.zeros_like(rhs)
    residual = rhs - matmul(result)
    residual_norm = np.linalg.norm(residual, axis=0, keepdims=True)
    has_converged = residual_norm < stop_updating_after
    n_iter = 0 if has_converged.all() else max_iter
    p = residual.copy()
    rr = np.sum(residual * residual, axis=0, keepdims=True)
    k_done = 0
    for k in range(n_iter):
        mvms = matmul(p)
        pap = np.sum(p * mvms, axis=0, keepdims=True)
        zero = pap < eps
        alpha = np.where(zero, dtype(0), rr / np.where(zero, dtype(1), pap))
        alpha = np.where(has_converged, dtype(0), alpha)
        residual = residual - alpha * mvms
        result = result + alpha * p
        rr_new = np.sum(residual * residual, axis=0, keepdims=True)
        zero = rr < eps
        beta = np.where(zero, dtype(0), rr_new / np.where(zero, dtype(1), rr))
        rr = rr_new
        p = p * beta + residual
        residual_norm = np.linalg.norm(residual, axis=0, keepdims=True)
        residual_norm = np.where(rhs_is_zero, dtype(0), residual_norm)
        has_converged = residual_norm < stop_updating_after
        k_done = k + 1
        if k >= min(10, max_iter - 1) and residual_norm.mean() < tolerance:
            break
    return result * rhs_norm, k_done


def pathwise_predict(phi: sp.csr_matrix, train_idx, test_idx, y_train, noise, eps1, eps2, tolerance=1.0,
                     max_iter=1000):
    """(S x n_test) samples and the CG iteration count; fp64 throughout."""
    phi = sp.csr_matrix(phi, dtype=np.float64)
    p_tr = phi[np.asarray(train_idx)]
    p_te = phi[np.asarray(test_idx)]
    eps1 = np.asarray(eps1, np.float64)
    eps2 = np.asarray(eps2, np.float64)
    f_test = (p_te @ eps1.T).T
    f_train = (p_tr @ eps1.T).T
    b = np.asarray(y_train, np.float64)[None, :] - (f_train + eps2)

    def matmul(v):
        return p_tr @ (p_tr.T @ v) + noise * v

    v, iters = linear_cg(matmul, b.T, tolerance=tolerance, max_iter=max_iter)
    return f_test + (p_te @ (p_tr.T @ v)).T, iters
