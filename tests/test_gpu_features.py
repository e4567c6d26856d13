"""The GPyTorch surface on the HIP feature algebra (grf_amd/features.py).

Reference: efficient_graph_gp_sparse/gptorch_kernels_sparse/sparse_grf_kernel.py:24-61,
sparse_diffusion_kernel.py:27-96, preprocessor/graph_preprocessor.py:88-140.  GPyTorch and
linear_operator are absent here, so the arithmetic is pinned to a numpy fp64 restatement of the
reference's formulas on the reference's own golden step matrices (tests/golden/small_graphs.npz,
made by make_golden.py from SparseRandomWalk): Phi = sum_l f_l M_l, K = Phi[x1] Phi[x2]^T,
diag = rowwise Phi[x1] . Phi[x2], and the analytic gradient
dL/df_l = sum_{r,s} G[r,s] (M_l[x1_r] . Phi[x2_s] + Phi[x1_r] . M_l[x2_s]).
Tolerances: K / diag |d| <= 3e-5 (|Phi||Phi|^T) + 1e-7 max|K| (fp32 Phi, exact fixed-point Gram);
gradients rtol 1e-4 (fp32 Z = Phi^T G^T on the device).
"""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import csr, same_csr

pytestmark = pytest.mark.gpu


def _ops(mats):
    from efficient_graph_gp_sparse.preprocessor import GraphPreprocessor
    from efficient_graph_gp_sparse.utils_sparse.sparse_lo import SparseLinearOperator
    return [SparseLinearOperator(GraphPreprocessor.from_scipy_csr(M).to("cuda")) for M in mats]


def _close(got, ref, absbound):
    err = np.abs(np.asarray(got, np.float64) - ref)
    return bool(np.all(err <= 3e-5 * absbound + 1e-7 * max(np.abs(ref).max(), 1e-30))), float(err.max())


def test_sparse_grf_kernel_forward_diag_and_gradient(golden):
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseGRFKernel
    d = golden("small_graphs")
    steps = [csr(d, f"er40_sp_n3_s7_l{l}", 40) for l in range(4)]
    dense = [M.toarray().astype(np.float32).astype(np.float64) for M in steps]  # (the torch CSR's fp32 values)
    torch.manual_seed(0)
    kern = SparseGRFKernel(4, _ops(steps)).cuda()
    f = kern.modulator_vector.detach().cpu().numpy().astype(np.float64)
    Phi = sum(fl * M for fl, M in zip(f, dense))
    aPhi = np.abs(Phi)
    i1, i2 = [0, 3, 5, 17, 39, 3], [1, 3, 20]
    x1, x2 = torch.tensor(i1, device="cuda"), torch.tensor(i2, device="cuda")
    K = kern(x1, x2)
    assert K.is_cuda and K.shape == (6, 3)
    ok, e = _close(K.detach().cpu().numpy(), Phi[i1] @ Phi[i2].T, aPhi[i1] @ aPhi[i2].T)
    assert ok, e
    Kd = kern(x1, x1, diag=True)
    ok, e = _close(Kd.detach().cpu().numpy(), np.einsum("ij,ij->i", Phi[i1], Phi[i1]),
                   np.einsum("ij,ij->i", aPhi[i1], aPhi[i1]))
    assert ok, e
    Kfull = kern()
    ok, e = _close(Kfull.detach().cpu().numpy(), Phi @ Phi.T, aPhi @ aPhi.T)
    assert ok, e
    assert torch.equal(Kfull, Kfull.t())  # x1 == x2: symmetric enumeration + mirror
    # gradient of sum(W * K[x1, x2]) w.r.t. the modulator
    W = np.random.default_rng(1).standard_normal((6, 3))
    (kern(x1, x2) * torch.tensor(W, device="cuda", dtype=torch.float32)).sum().backward()
    gref = [np.sum(W * (dense[l][i1] @ Phi[i2].T + Phi[i1] @ dense[l][i2].T)) for l in range(4)]
    np.testing.assert_allclose(kern.raw_modulator_vector.grad.cpu().numpy(), gref, rtol=1e-4, atol=1e-6)
    kern.raw_modulator_vector.grad = None
    w = np.random.default_rng(2).standard_normal(6)
    (kern(x1, x1, diag=True) * torch.tensor(w, device="cuda", dtype=torch.float32)).sum().backward()
    gref = [np.sum(w * 2 * np.einsum("ij,ij->i", dense[l][i1], Phi[i1])) for l in range(4)]
    np.testing.assert_allclose(kern.raw_modulator_vector.grad.cpu().numpy(), gref, rtol=1e-4, atol=1e-6)
    # the feature matrix itself
    P = kern._get_feature_matrix()
    assert P.is_sparse_csr and P.is_cuda
    np.testing.assert_allclose(P.to_dense().cpu().numpy(), Phi, rtol=1e-6, atol=1e-7)


def test_sparse_diffusion_kernel_gradients(golden):
    """Autograd through the modulator formula to beta and sigma_f, against central finite
    differences of the numpy restatement (fp64)."""
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseDiffusionKernel
    d = golden("small_graphs")
    steps = [csr(d, f"wer30_sp_n3_s7_l{l}", 30) for l in range(4)]
    dense = [M.toarray().astype(np.float32).astype(np.float64) for M in steps]
    dk = SparseDiffusionKernel(4, _ops(steps)).cuda()
    x = torch.tensor([0, 2, 7, 11, 29], device="cuda")
    W = np.random.default_rng(3).standard_normal((5, 5))
    (dk(x, x) * torch.tensor(W, device="cuda", dtype=torch.float32)).sum().backward()

    def loss(rb, rs):
        beta, sig = np.log1p(np.exp(rb)), np.log1p(np.exp(rs))
        fm = [sig * (-beta) ** l / (2 ** l * np.prod(np.arange(1, l + 1))) for l in range(4)]
        Phi = sum(fl * M for fl, M in zip(fm, dense))[[0, 2, 7, 11, 29]]
        return np.sum(W * (Phi @ Phi.T))

    h = 1e-5
    gb = (loss(1.0 + h, 1.0) - loss(1.0 - h, 1.0)) / (2 * h)
    gs = (loss(1.0, 1.0 + h) - loss(1.0, 1.0 - h)) / (2 * h)
    np.testing.assert_allclose([dk.raw_beta.grad.item(), dk.raw_sigma_f.grad.item()], [gb, gs], rtol=2e-4)


def test_preprocessor_device_resident_steps(golden, tmp_path):
    """preprocess_graph keeps the step matrices on the device (no host scipy round trip); the host
    copy is made only when step_matrices_scipy is read, and equals the reference's golden steps."""
    from efficient_graph_gp_sparse.preprocessor import GraphPreprocessor
    d = golden("small_graphs")
    A = sp.csr_matrix(d["er40_A"])
    pre = GraphPreprocessor(A, walks_per_node=20, p_halt=0.2, max_walk_length=4, random_walk_seed=7,
                            cache_filename=str(tmp_path / "s.npz"), n_processes=3)
    ops = pre.preprocess_graph()
    assert pre._step_scipy is None  # nothing copied to the host yet
    assert all(op.sparse_csr_tensor.is_cuda and op.sparse_csr_tensor.values().dtype == torch.float32 for op in ops)
    for l, op in enumerate(ops):
        ref = csr(d, f"er40_sp_n3_s7_l{l}", 40)
        t = op.sparse_csr_tensor
        assert np.array_equal(t.crow_indices().cpu().numpy(), ref.indptr)
        assert np.array_equal(t.col_indices().cpu().numpy(), ref.indices)
        assert np.array_equal(t.values().cpu().numpy(), ref.data.astype(np.float32))
        assert same_csr(pre.step_matrices_scipy[l], ref)


def test_full_graph_forward_on_enron_without_densifying(golden):
    """Enron (36,692 nodes): the whole K from the kernel's forward, with the device's peak memory
    within K's own bytes plus a margin (a dense Phi alone would be another 5.4 GB), sampled rows
    against the fp64 restatement; and a 2,000-node gradient."""
    from golden_util import snap_adjacency
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseDiffusionKernel
    from efficient_graph_gp_sparse.preprocessor import GraphPreprocessor
    A = snap_adjacency(golden("snap"), "enron")
    n = A.shape[0]
    pre = GraphPreprocessor(A, walks_per_node=32, p_halt=0.1, max_walk_length=8, rng="philox")
    ops = pre.preprocess_graph()
    dk = SparseDiffusionKernel(8, ops).cuda()
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    K = dk()
    torch.cuda.synchronize()
    k_bytes = 4 * n * n
    assert torch.cuda.max_memory_allocated() - base < 1.25 * k_bytes + (1 << 30)
    fm = dk.modulator_vector.detach().cpu().numpy().astype(np.float64)
    steps = [M.astype(np.float32).astype(np.float64) for M in pre.step_matrices_scipy]
    Phi = sum(fl * M for fl, M in zip(fm, steps)).tocsr()
    rows = np.r_[0, 1, np.argsort(-np.diff(A.indptr), kind="stable")[:3], n - 1]
    Kr = K[torch.tensor(rows, device="cuda")].detach().cpu().numpy()
    ok, e = _close(Kr, (Phi[rows] @ Phi.T).toarray(), (abs(Phi)[rows] @ abs(Phi).T).toarray())
    assert ok, e
    del K
    x = torch.tensor(np.random.default_rng(4).choice(n, 2000, replace=False), device="cuda")
    dk(x, x).sum().backward()
    xs = x.cpu().numpy()
    P = Phi[xs]
    g_phi = [float(np.sum((steps[l][xs] @ P.T).toarray()) * 2) for l in range(8)]  # d sum(K)/d f_l
    beta, sig = float(dk.beta), float(dk.sigma_f)
    dfdsig = [fm[l] / sig for l in range(8)]
    np.testing.assert_allclose(dk.raw_sigma_f.grad.item(),
                               sum(g * df for g, df in zip(g_phi, dfdsig)) * (1 - np.exp(-sig)), rtol=1e-3)


def test_dense_steps_kernels_cora_size(golden):
    """The GPflow surface's per-call algebra on HIP (grf_dense_steps_phi / grf_dense_steps_grad,
    gpflow_kernels/general_kernel_fast_grf.py:74-77) at Cora size: F = the reference's own Cora step
    matrices (m = 16, 4 steps, tests/golden/cora.npz) as the dense (N, N, L) tensor, against the numpy
    restatement Phi = F f, K = Phi Phi^T, dL/df_l = <F_l, (G + G^T) Phi> (parity unpinned by the
    reference: GPflow / TF absent).  Phi fp64 within 1e-15 relative (order of the L-term sum), K within
    the fp32 MFMA tolerance, the gradient rtol 1e-9 (fp64 MFMA GEMM, fused reduction, fixed order)."""
    from grf_amd.engine import get_engine
    from grf_amd.features import DenseGramFunction, DenseSteps
    d = golden("cora")
    n = len(d["A_indptr"]) - 1
    L = 4
    F = np.zeros((n, n, L))
    for l in range(L):
        F[:, :, l] = csr(d, f"m16_l{l}", n).toarray()
    f = np.array([1.0, -0.5, 0.125, -0.0208])
    st = DenseSteps(F, get_engine())
    P = F @ f
    phi = st.phi(torch.from_numpy(f)).cpu().numpy()
    assert np.all(np.abs(phi - P) <= 1e-15 * np.abs(F) @ np.abs(f) + 1e-300)
    K = st.gram(torch.from_numpy(f)).cpu().numpy()
    aP = np.abs(P)
    ok, e = _close(K, P @ P.T, aP @ aP.T)
    assert ok, e
    # the learnable path: d sum(W * K) / d f through DenseGramFunction
    W = np.random.default_rng(5).standard_normal((n, n))
    fp = torch.tensor(f, device="cuda", requires_grad=True)
    (DenseGramFunction.apply(fp, st) * torch.tensor(W, device="cuda")).sum().backward()
    H = (W + W.T) @ P
    gref = np.einsum("ijl,ij->l", F, H)
    np.testing.assert_allclose(fp.grad.cpu().numpy(), gref, rtol=1e-9, atol=1e-12 * np.abs(gref).max())
    # a CPU modulator parameter gets its gradient on its own device
    fc = torch.tensor(f, requires_grad=True)
    (DenseGramFunction.apply(fc, st) * torch.tensor(W, device="cuda")).sum().backward()
    assert fc.grad.device.type == "cpu"
    np.testing.assert_allclose(fc.grad.numpy(), gref, rtol=1e-9, atol=1e-12 * np.abs(gref).max())


def test_kernel_block_shift_bound_takes_both_operands(golden):
    """K[x1, x2] with x1 one low-magnitude row and x2 holding the row with the largest |Phi|: the
    fixed-point shift of x1's row must bound its products with the OTHER operand's values too
    (shifts from Phi[x1] alone let terms pass 2^51 on degree-skewed graphs)."""
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseGRFKernel
    d = golden("small_graphs")
    steps = [csr(d, f"er40_sp_n3_s7_l{l}", 40) for l in range(4)]
    scale = np.ones(40)
    scale[7] = 1e6  # a hub-like row of huge loads
    steps = [sp.diags(scale) @ M for M in steps]
    dense = [M.toarray().astype(np.float32).astype(np.float64) for M in steps]
    kern = SparseGRFKernel(4, _ops(steps)).cuda()
    f = kern.modulator_vector.detach().cpu().numpy().astype(np.float64)
    Phi = sum(fl * M for fl, M in zip(f, dense))
    aPhi = np.abs(Phi)
    lo = int(np.argmin(np.where(aPhi.max(1) > 0, aPhi.max(1), np.inf)))
    i1, i2 = [lo], [7, lo, 3]
    K = kern(torch.tensor(i1, device="cuda"), torch.tensor(i2, device="cuda")).detach().cpu().numpy()
    # elementwise, relative to each entry's own |Phi||Phi|^T (no absolute slack from the huge row)
    err = np.abs(K.astype(np.float64) - Phi[i1] @ Phi[i2].T)
    assert np.all(err <= 3e-5 * (aPhi[i1] @ aPhi[i2].T) + 1e-30), err


def test_sparse_kernel_forward_backward_issue_no_host_sync(golden):
    """The GPyTorch forward + backward read nothing back to the host: after the
    one-time StepMatrices setup, K[x1, x2], K(x, x), the diagonal and the modulator gradient run under
    torch.cuda.set_sync_debug_mode("error"), which raises on any device->host synchronisation
    (.item(), .cpu(), torch.equal, ...).  Phi is sized by sum_l nnz(M_l), row gathers by rows x the
    row bound, the transposes by those bounds (the C side pads the tail), x1 == x2 is decided by
    identity, and the dense (GPflow) Gram cache is keyed by the modulator tensor's version counter."""
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseGRFKernel
    d = golden("small_graphs")
    steps = [csr(d, f"er40_sp_n3_s7_l{l}", 40) for l in range(4)]
    torch.manual_seed(0)
    kern = SparseGRFKernel(4, _ops(steps)).cuda()
    x1 = torch.tensor([0, 3, 5, 17, 39, 3], device="cuda")
    x2 = torch.tensor([1, 3, 20], device="cuda")
    W = torch.randn(6, 3, device="cuda")
    ref_K = kern(x1, x2).detach().clone()  # (warm-up: builds the StepMatrices, one-time host reads)
    kern.raw_modulator_vector.grad = None
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        K = kern(x1, x2)
        Ks = kern(x1, x1)
        Kd = kern(x1, x1, diag=True)
        loss = (K * W).sum() + Ks.sum() + Kd.sum()
        loss.backward()
    finally:
        torch.cuda.set_sync_debug_mode("default")
    torch.cuda.synchronize()
    assert torch.equal(K.detach(), ref_K)
    assert torch.equal(Ks.detach(), Ks.detach().t())
    assert kern.raw_modulator_vector.grad is not None and torch.isfinite(kern.raw_modulator_vector.grad).all()


def test_dense_gram_cache_keyed_without_host_copy():
    """DenseSteps.gram: the cache hits for the same modulator tensor (and a detached view or the tensor
    autograd saves), misses after an in-place update (its version counter) -- with no host copy of f."""
    from grf_amd.features import DenseSteps
    torch.manual_seed(0)
    F = torch.rand(64, 64, 3, dtype=torch.float64) * (torch.rand(64, 64, 3, dtype=torch.float64) < 0.2)
    ds = DenseSteps(F)
    f = torch.tensor([1.0, -0.5, 0.25], dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        K1 = ds.gram(f)
        assert ds.gram(f) is K1 and ds.gram(f.detach()) is K1
        f.mul_(2.0)  # (an optimiser step: in place)
        K2 = ds.gram(f)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert K2 is not K1
    torch.testing.assert_close(K2, 4.0 * K1, rtol=1e-5, atol=1e-6)


def test_dense_gram_cache_sees_writes_that_bypass_the_version_counter():
    """a CPU modulator is keyed by value (a numpy write into a torch.from_numpy tensor is
    seen); the GPflow wrapper's host-returning K / K_diag key by the modulator's values (a write
    through ``.data`` is seen); the device path (K_torch) is sync-free and keyed by the version counter,
    and ``invalidate()`` drops the cache after a ``.data`` write."""
    from efficient_graph_gp.gpflow_kernels import GraphGeneralFastGRFKernel
    from grf_amd.features import DenseSteps
    torch.manual_seed(0)
    F = torch.rand(48, 48, 3, dtype=torch.float64) * (torch.rand(48, 48, 3, dtype=torch.float64) < 0.3)
    ds = DenseSteps(F)
    arr = np.array([1.0, -0.5, 0.25])
    fh = torch.from_numpy(arr)
    K1 = ds.gram(fh).clone()
    arr *= 2.0  # (no version bump: numpy writes the shared memory)
    torch.testing.assert_close(ds.gram(fh), 4.0 * K1, rtol=1e-5, atol=1e-6)
    # the GPflow-style wrapper
    r = np.random.default_rng(2)
    A = (r.random((40, 40)) < 0.15).astype(np.float64)
    A = np.maximum(A, A.T)
    np.fill_diagonal(A, 0.0)
    kern = GraphGeneralFastGRFKernel(A, walks_per_node=16, p_halt=0.2, max_walk_length=3, random_walk_seed=1)
    X = np.arange(40)
    Ka = kern.K(X)
    with torch.no_grad():
        kern.modulator_vector.data.copy_(2.0 * kern.modulator_vector.detach())  # (bypasses _version)
    np.testing.assert_allclose(kern.K(X), 4.0 * Ka, rtol=1e-5, atol=1e-6)
    Kt1 = kern.K_torch(X).detach().clone()
    kern.modulator_vector.data.mul_(0.5)
    kern.invalidate()
    np.testing.assert_allclose(kern.K_torch(X).detach().cpu().numpy(), Kt1.cpu().numpy() / 4.0, rtol=1e-5, atol=1e-6)


def test_row_selection_bounds_fall_back_to_exact_counts_on_hub_rows():
    """a row selection's buffers use rows x row_bound only while that stays near the
    matrix's own entries; one dense (hub) row makes row_bound ~ n_cols, and the exact count is used."""
    from grf_amd.engine import DeviceCSR, GRFEngine
    from grf_amd.features import gather_rows
    eng = GRFEngine("cuda:0")
    n = 20000
    r = np.random.default_rng(3)
    rows = np.repeat(np.arange(n), 3)
    cols = r.integers(0, n, rows.size)
    A = sp.csr_matrix((np.ones(rows.size), (rows, cols)), shape=(n, n))
    A = A + sp.csr_matrix((np.ones(n), (np.zeros(n, int), np.arange(n))), shape=(n, n))  # row 0: dense
    A = sp.csr_matrix(A)
    Ad = DeviceCSR.from_scipy(A, eng.device)
    Ad.val32 = Ad.val.float()
    Ad.row_bound = int(np.diff(A.indptr).max())
    sel = torch.arange(0, n, 2, device=eng.device)
    assert Ad.rows_entry_bound(sel.numel()) is None  # (10k x 20k entries would be 200 M)
    G = gather_rows(eng, Ad, sel)
    want = A[np.arange(0, n, 2)]
    assert G.nnz_bound == want.nnz
    assert same_csr(G.to_scipy().astype(np.float64), want.astype(np.float32).astype(np.float64))
    small = torch.arange(1, 200, device=eng.device)  # (199 rows x the bound: within the floor)
    assert Ad.rows_entry_bound(small.numel()) == small.numel() * Ad.row_bound


def test_kernel_block_equal_valued_indices_is_exactly_symmetric(golden):
    """K(x1, x2) with x1, x2 equal-valued but different tensors (a caller that clones
    the inputs) comes out exactly symmetric (decided on the device, no host read); different values of
    the same length are left as computed."""
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseGRFKernel
    d = golden("small_graphs")
    steps = [csr(d, f"er40_sp_n3_s7_l{l}", 40) for l in range(4)]
    torch.manual_seed(0)
    kern = SparseGRFKernel(4, _ops(steps)).cuda()
    x = torch.tensor([0, 3, 5, 17, 39, 8, 21], device="cuda")
    K = kern(x, x.clone()).detach()
    assert torch.equal(K, K.t())
    torch.testing.assert_close(K, kern(x, x).detach(), rtol=1e-6, atol=1e-7)
    y = torch.tensor([1, 3, 5, 17, 39, 8, 22], device="cuda")
    Ky = kern(x, y).detach()
    Kxy = kern(x, y.clone()).detach()
    assert torch.equal(Ky, Kxy)
