"""GPU parity of the step after the path: K.v = Phi (Phi^T v), the
CSR transpose it uses, the linear_cg solve and SparseGraphGP.predict
(efficient_graph_gp_sparse/models/sparse_grf_model.py:21-45), against oracle/cg.py.

Tolerances
  * CSR transpose: exact (same entries, ascending rows per column).
  * SpMM (fp32, fixed order) vs fp64: |dY| <= 2e-6 * (|A| |X|) elementwise.
  * CG / predict: linear_cg's trajectory is chaotic in ANY precision once CG loses
    orthogonality -- on these systems a 1e-15 relative change of B moves the fp64 oracle's
    own iterate by 1e-13 after 6 iterations, 1e-7 after 10 and 1e-3 after 11-12
    (measured; tools/cg_diag.py shows the GPU tracking the oracle with the same growth).
    So the algorithm is pinned iterate by iterate where it is still determined by its
    inputs: fp64 vs the fp64 oracle for max_iter = 1..7 to 1e-10 relative (exact
    iteration counts), the reference's fp32 for max_iter = 1..3 to 1e-4; full runs are
    checked through the stopping rule on the solver's own trajectory (mean residual of
    the last iteration < tolerance, of the one before >= tolerance), the true residual
    it reached, zero columns and limits.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import cg as OCG

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from grf_amd.engine import GRFEngine
    return GRFEngine("cuda:0")


def _graph(n, deg, seed):
    r = np.random.default_rng(seed)
    m = int(n * deg / 2)
    u, v = r.integers(0, n, m), r.integers(0, n, m)
    keep = u != v
    A = sp.coo_matrix((np.ones(keep.sum()), (u[keep], v[keep])), shape=(n, n)).tocsr()
    A = (A + A.T).tocsr()
    A.data[:] = 1.0
    return A


@pytest.fixture(scope="module")
def phi(eng):
    A = _graph(3000, 8, 5)
    G = eng.laplacian(A)
    f = [1.0, -0.5, 0.25, -0.125]
    return eng.compact(eng.walk_phi(G, 16, 0.2, 4, f, seed=3))


def _phi32(phi):
    P = phi.to_scipy().astype(np.float64)
    P.data = phi.val32.cpu().numpy().astype(np.float64)
    return P


def test_csr_transpose_exact(eng, phi):
    import torch
    P = _phi32(phi)
    t = eng.csr_transpose(phi)
    want = P.T.tocsr()
    want.sort_indices()
    assert np.array_equal(t.ptr.cpu().numpy(), want.indptr)
    assert np.array_equal(t.idx.cpu().numpy(), want.indices)
    assert np.array_equal(t.val32.cpu().numpy().astype(np.float64), want.data)
    rows = np.random.default_rng(0).permutation(3000)[:1700]
    rows[5] = rows[9]                                   # a repeated row
    t = eng.csr_transpose(phi, torch.from_numpy(rows))
    want = P[rows].T.tocsr()
    want.sort_indices()
    assert np.array_equal(t.ptr.cpu().numpy(), want.indptr)
    assert np.array_equal(t.idx.cpu().numpy(), want.indices)
    assert np.array_equal(t.val32.cpu().numpy().astype(np.float64), want.data)
    e = eng.csr_transpose(phi, torch.empty(0, dtype=torch.int32))
    assert e.nnz == 0 and not e.ptr.cpu().numpy().any()


@pytest.mark.parametrize("S", [1, 2, 3, 7, 12, 33, 64, 100, 130])
@pytest.mark.parametrize("f64", [False, True])
def test_spmm_vs_fp64(eng, phi, S, f64):
    import torch
    P = _phi32(phi)
    r = np.random.default_rng(S)
    X = r.standard_normal((3000, S)).astype(np.float64 if f64 else np.float32)
    rows = r.integers(0, 3000, 777)
    Y = eng.spmm(phi, torch.from_numpy(X).cuda(), torch.from_numpy(rows)).cpu().numpy()
    want = P[rows] @ X.astype(np.float64)
    bound = abs(P[rows]) @ np.abs(X).astype(np.float64)
    assert np.all(np.abs(Y - want) <= (1e-14 if f64 else 2e-6) * bound + 1e-300)
    Y2 = eng.spmm(phi, torch.from_numpy(X).cuda(), torch.from_numpy(rows)).cpu().numpy()
    assert np.array_equal(Y, Y2)                        # fixed summation order


def test_gram_matvec(eng, phi):
    import torch
    P = _phi32(phi)
    r = np.random.default_rng(1)
    V = r.standard_normal((3000, 64)).astype(np.float32)
    Y = eng.gram_matvec(phi, torch.from_numpy(V).cuda(), noise=0.3).cpu().numpy()
    want = P @ (P.T @ V.astype(np.float64)) + 0.3 * V
    assert np.linalg.norm(Y - want) <= 1e-5 * np.linalg.norm(want)


def _system(phi, n_tr, S, seed, noise):
    P = _phi32(phi)
    r = np.random.default_rng(seed)
    tr = np.sort(r.permutation(P.shape[0])[:n_tr])
    B = r.standard_normal((n_tr, S)).astype(np.float32)
    Pt = P[tr]
    return P, tr, B, (lambda v: Pt @ (Pt.T @ v) + noise * v)


@pytest.mark.parametrize("S", [64, 5, 1, 200])
def test_cg_iterates_fp64_vs_oracle(eng, phi, S):
    import torch
    for noise in (0.1, 2.0):
        P, tr, B, mm = _system(phi, 1800, S, S, noise)
        Bd = torch.from_numpy(B.astype(np.float64)).cuda()
        for mi in range(1, 8):
            X, it = eng.cg_solve(phi, Bd, noise, torch.from_numpy(tr), max_iter=mi)
            Xo, ito = OCG.linear_cg(mm, B.astype(np.float64), max_iter=mi)
            assert it == ito == mi
            X = X.cpu().numpy()
            rel = np.linalg.norm(X - Xo) / np.linalg.norm(Xo)
            assert rel <= 1e-10, (noise, mi, rel)
        X2, _ = eng.cg_solve(phi, Bd, noise, torch.from_numpy(tr), max_iter=7)
        assert np.array_equal(X, X2.cpu().numpy())       # deterministic


@pytest.mark.parametrize("S", [64, 3])
def test_cg_iterates_fp32_vs_oracle(eng, phi, S):
    import torch
    P, tr, B, mm = _system(phi, 1800, S, 7, 2.0)
    for mi in range(1, 4):
        X, it = eng.cg_solve(phi, torch.from_numpy(B).cuda(), 2.0, torch.from_numpy(tr), max_iter=mi)
        Xo, ito = OCG.linear_cg(mm, B.astype(np.float64), max_iter=mi)
        assert it == ito == mi and X.dtype == torch.float32
        X = X.cpu().numpy()
        assert np.linalg.norm(X - Xo) <= 1e-4 * np.linalg.norm(Xo)


@pytest.mark.parametrize("dtype,noise,tol", [("f64", 0.1, 1.0), ("f64", 2.0, 1.0), ("f64", 0.5, 0.05),
                                             ("f32", 0.1, 1.0), ("f32", 2.0, 1.0)])
def test_cg_full_run_stopping_rule(eng, phi, dtype, noise, tol):
    """linear_cg's rule on the solver's own trajectory: it stops at the first k >= 10 whose
    mean residual norm is below the tolerance."""
    import torch
    P, tr, B, mm = _system(phi, 1800, 64, 11, noise)
    Bt = torch.from_numpy(B.astype(np.float64) if dtype == "f64" else B).cuda()
    rows = torch.from_numpy(tr)
    X, it, res = eng.cg_solve(phi, Bt, noise, rows, tolerance=tol, return_residuals=True)
    assert 11 <= it < 1000 and res.mean() < tol
    if it > 11:
        _, it_prev, res_prev = eng.cg_solve(phi, Bt, noise, rows, tolerance=tol, max_iter=it - 1,
                                            return_residuals=True)
        assert it_prev == it - 1 and res_prev.mean() >= tol
    # the recursive residual is the true one (up to the recurrence's drift)
    Xh = X.cpu().numpy().astype(np.float64)
    true = np.linalg.norm(mm(Xh) - B, axis=0) / np.linalg.norm(B, axis=0)
    assert np.allclose(true, res, rtol=0.05 if dtype == "f64" else 0.2, atol=1e-3)


def test_cg_zero_rhs_column_and_limits(eng, phi):
    # (iterates compared at max_iter = 5: this small-noise system (noise 0.2, 500 rows) amplifies rounding
    # faster than the 1800-row ones -- with round 6's Philox stream its Phi gives 2.4e-10 relative at
    # iteration 7, the chaotic growth the module docstring describes, not a solver difference)
    import torch
    P, tr, B, mm = _system(phi, 500, 4, 9, 0.2)
    B = B.astype(np.float64)
    B[:, 2] = 0.0
    X, it = eng.cg_solve(phi, torch.from_numpy(B).cuda(), 0.2, torch.from_numpy(tr), max_iter=5)
    Xo, ito = OCG.linear_cg(mm, B, max_iter=5)
    X = X.cpu().numpy()
    assert it == ito and not X[:, 2].any()
    assert np.linalg.norm(X - Xo) <= 1e-10 * np.linalg.norm(Xo)
    X, it = eng.cg_solve(phi, torch.from_numpy(B).cuda(), 0.2, torch.from_numpy(tr))
    assert it >= 11 and not X.cpu().numpy()[:, 2].any()
    Z, it0 = eng.cg_solve(phi, torch.zeros((500, 3), device="cuda", dtype=torch.float64), 0.2,
                          torch.from_numpy(tr))
    assert it0 == 0 and not Z.cpu().numpy().any()
    with pytest.raises(NotImplementedError):
        eng.cg_solve(phi, torch.zeros((500, 257), device="cuda"), 0.2, torch.from_numpy(tr))


@pytest.mark.parametrize("max_iter", [3, 1000])
def test_pathwise_predict_vs_oracle(eng, phi, max_iter):
    import torch
    n = phi.n_rows
    r = np.random.default_rng(42)
    perm = r.permutation(n)
    tr, te = perm[:1800], perm[1800:2400]               # unsorted indices, like x_train.int()
    y = r.standard_normal(1800).astype(np.float32)
    noise = 0.05
    e1 = r.standard_normal((64, n)).astype(np.float32)
    e2 = (np.float32(np.sqrt(noise)) * r.standard_normal((64, 1800))).astype(np.float32)
    out, it = eng.pathwise_predict(phi, torch.from_numpy(tr), torch.from_numpy(te), torch.from_numpy(y), noise,
                                   torch.from_numpy(e1).cuda(), torch.from_numpy(e2).cuda(), max_iter=max_iter)
    want, ito = OCG.pathwise_predict(_phi32(phi), tr, te, y, noise, e1, e2, max_iter=max_iter)
    assert out.shape == (64, 600) and out.dtype == torch.float64
    out = out.cpu().numpy()
    rel = np.linalg.norm(out - want) / np.linalg.norm(want)
    if max_iter == 3:
        assert it == ito == 3 and rel <= 1e-10, rel
    else:
        # (beyond ~10 iterations both are single draws of linear_cg's rounding-sensitive
        # trajectory; the posterior mean part is what they share)
        assert it >= 11 and ito >= 11 and rel <= 0.2, rel


def test_sparse_graph_gp_predict_mirror(tmp_path):
    """models/sparse_grf_model.py:21-45 through the mirror: the GP's own Phi (current modulator),
    its own eps draws (torch.randn on the device, reference order), checked against the oracle
    fed with the same draws (3 CG iterations: the rounding-determined window)."""
    import torch
    from efficient_graph_gp_sparse.models import SparseGraphGP
    from efficient_graph_gp_sparse.preprocessor import GraphPreprocessor

    A = _graph(600, 6, 21)
    pre = GraphPreprocessor(A, walks_per_node=16, p_halt=0.2, max_walk_length=4, random_walk_seed=3)
    ops = pre.preprocess_graph()

    class Lik:
        noise = torch.tensor([0.05])

    r = np.random.default_rng(0)
    perm = r.permutation(600)
    x_train = torch.tensor(perm[:400], dtype=torch.float32, device="cuda").unsqueeze(1)
    y_train = torch.tensor(r.standard_normal(400), dtype=torch.float32, device="cuda")
    x_test = torch.tensor(perm[400:500], dtype=torch.float32, device="cuda").unsqueeze(1)
    gp = SparseGraphGP(x_train, y_train, Lik(), ops, 4).cuda()
    torch.manual_seed(123)
    out = gp.predict(x_test, n_samples=32, max_iter=3)
    assert out.shape == (32, 100) and out.dtype == torch.float32 and gp.last_cg_iterations == 3
    # the same draws, replayed
    torch.manual_seed(123)
    e1 = torch.randn(32, 600, device="cuda")
    e2 = torch.sqrt(torch.tensor(0.05, device="cuda")) * torch.randn(32, 400, device="cuda")
    f = gp.covar_module.modulator_vector.detach().cpu().numpy().astype(np.float64)
    Phi = sum(float(np.float32(fl)) * M for fl, M in zip(f, pre.step_matrices_scipy))
    Phi = sp.csr_matrix(Phi.astype(np.float32).astype(np.float64))
    want, it = OCG.pathwise_predict(Phi, perm[:400], perm[400:500], y_train.cpu().numpy(), 0.05,
                                    e1.cpu().numpy(), e2.cpu().numpy(), max_iter=3)
    rel = np.linalg.norm(out.cpu().numpy() - want) / np.linalg.norm(want)
    assert it == 3 and rel <= 1e-5, rel
    full = gp.predict(x_test, n_samples=64)
    assert full.shape == (64, 100) and torch.isfinite(full).all() and gp.last_cg_iterations >= 11
