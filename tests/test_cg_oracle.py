"""CPU: the numpy restatement of linear_cg / SparseGraphGP.predict (oracle/cg.py).

linear_operator (the reference's CG, via gpytorch==1.11) is absent, so the restatement is
pinned to textbook CG (identical iterates while no eps guard fires) and to the exact solve
(run to its floor it must match numpy.linalg.solve; linear_cg's eps = 1e-10 guards act on
the squared norms r.r and p.Ap, so a normalised column stalls near a relative residual of
1e-5 -- that floor is linear_cg's own); run with gpytorch's default cg_tolerance (1) it must
stop after iteration k = 10 (11 matvecs).
"""
import numpy as np
import scipy.sparse as sp

from oracle import cg as OCG


def _spd(n, seed, noise=0.1):
    r = np.random.default_rng(seed)
    phi = sp.random(n, 3 * n, density=0.05, random_state=seed, format="csr")
    A = (phi @ phi.T).toarray() + noise * np.eye(n)
    return phi, A, r


def _textbook_cg(A, b, iters):
    x = np.zeros_like(b)
    r = b.copy()
    p = r.copy()
    rr = r @ r
    for _ in range(iters):
        ap = A @ p
        a = rr / (p @ ap)
        x = x + a * p
        r = r - a * ap
        rr_new = r @ r
        p = r + (rr_new / rr) * p
        rr = rr_new
    return x


def test_linear_cg_iterates_are_textbook_cg():
    phi, A, r = _spd(50, 4)
    B = r.standard_normal((50, 3))
    X, k = OCG.linear_cg(lambda v: A @ v, B, max_iter=6)
    assert k == 6
    for c in range(3):
        np.testing.assert_allclose(X[:, c], _textbook_cg(A, B[:, c], 6), rtol=1e-10, atol=1e-12)


def test_linear_cg_converges_to_solve():
    phi, A, r = _spd(60, 1)
    B = r.standard_normal((60, 5))
    X, k = OCG.linear_cg(lambda v: A @ v, B, tolerance=1e-12, max_iter=1000)
    want = np.linalg.solve(A, B)
    assert np.linalg.norm(A @ X - B, axis=0).max() <= 1e-4 * np.linalg.norm(B, axis=0).min()
    np.testing.assert_allclose(X, want, rtol=2e-3, atol=1e-4 * np.abs(want).max())
    assert k == 1000                                  # the stall floor (~1e-5) never meets 1e-12


def test_linear_cg_default_tolerance_runs_eleven_iterations():
    phi, A, r = _spd(80, 2)
    B = r.standard_normal((80, 4))
    _, k = OCG.linear_cg(lambda v: A @ v, B)          # cg_tolerance = 1
    assert k == 11
    _, k1 = OCG.linear_cg(lambda v: A @ v, B, max_iter=3)
    assert k1 == 3                                    # min(10, max_iter - 1) = 2 -> stop at k = 2


def test_linear_cg_zero_and_vector_rhs():
    phi, A, r = _spd(40, 3)
    B = r.standard_normal((40, 3))
    B[:, 1] = 0.0
    X, _ = OCG.linear_cg(lambda v: A @ v, B, max_iter=30)
    assert np.all(X[:, 1] == 0.0)
    X2, _ = OCG.linear_cg(lambda v: A @ v, B[:, [0, 2]], max_iter=30)
    np.testing.assert_allclose(X[:, [0, 2]], X2, rtol=1e-12)
    x, _ = OCG.linear_cg(lambda v: A @ v, B[:, 0], max_iter=30)
    assert x.shape == (40,)
    np.testing.assert_allclose(x, X[:, 0], rtol=1e-12)
    Z, k = OCG.linear_cg(lambda v: A @ v, np.zeros((40, 2)))
    assert k == 0 and not Z.any()


def test_pathwise_predict_matches_exact_posterior_sample():
    """Converged pathwise conditioning = f_test + K_te,tr (K_tr,tr + s2 I)^-1 (y - f_train - eps2)."""
    n = 90
    phi = sp.random(n, n, density=0.08, random_state=7, format="csr")
    r = np.random.default_rng(7)
    tr, te = np.arange(0, 60), np.arange(60, 90)
    y = r.standard_normal(60)
    s2 = 0.05
    e1, e2 = r.standard_normal((4, n)), np.sqrt(s2) * r.standard_normal((4, 60))
    out, _ = OCG.pathwise_predict(phi, tr, te, y, s2, e1, e2, tolerance=1e-4)
    P = phi.toarray()
    K = P @ P.T
    f = e1 @ P.T
    want = f[:, te] + (K[np.ix_(te, tr)] @ np.linalg.solve(K[np.ix_(tr, tr)] + s2 * np.eye(60),
                                                          (y[None, :] - f[:, tr] - e2).T)).T
    np.testing.assert_allclose(out, want, rtol=1e-3, atol=1e-4 * np.abs(want).max())
