"""The reference's public API, re-pointed at the MI355X engine (GPU).

Mirrors the reference's own tests (tests/test_grf_dense.py, tests/test_grf_sparse.py)
and checks every entry point against golden vectors made by the reference.
Step matrices / Laplacians: bit-exact.  K (float32 on the GPU vs float64
reference): |dK| <= 3e-5 (|Phi||Phi|^T) + 1e-12 scale, checked here as
rtol=3e-5 against the reference values.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from golden_util import csr, same_csr

pytestmark = pytest.mark.gpu


# ------------------------------------------------ the reference's own 4 tests
def test_random_walk_shapes(toy_cycle_adj):
    from efficient_graph_gp.random_walk_samplers.sampler import Graph, RandomWalk
    graph = Graph(toy_cycle_adj)
    rw = RandomWalk(graph, seed=0)
    mats = rw.get_random_walk_matrices(num_walks=5, p_halt=0.2, max_walk_length=3, n_processes=1)
    assert mats.shape == (4, 4, 3)
    assert np.allclose(np.diag(mats[:, :, 0]), 1.0, atol=1e-6)


def test_fast_general_grf_kernel_psd(toy_cycle_adj):
    from efficient_graph_gp.graph_kernels.fast_grf_kernel_general import fast_general_grf_kernel
    k = fast_general_grf_kernel(adj_matrix=toy_cycle_adj, modulator_vector=np.array([1.0, 0.5, 0.25]),
                                walks_per_node=10, p_halt=0.2, max_walk_length=3)
    assert np.allclose(k, k.T, atol=1e-8)
    assert np.linalg.eigvalsh(k).min() >= -1e-8


def test_sparse_random_walk_shapes(toy_cycle_csr):
    from efficient_graph_gp_sparse.random_walk_samplers_sparse.sparse_sampler import SparseRandomWalk
    rw = SparseRandomWalk(toy_cycle_csr, seed=0)
    mats = rw.get_random_walk_matrices(num_walks=5, p_halt=0.2, max_walk_length=3, n_processes=1)
    assert len(mats) == 3 and all(m.shape == (4, 4) for m in mats)
    assert np.allclose(mats[0].diagonal(), 1.0, atol=1e-6)


def test_fast_general_grf_kernel_sparse_psd(toy_cycle_csr):
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel
    k = fast_general_grf_kernel(adj_matrix=toy_cycle_csr, modulator_vector=np.array([1.0, 0.5, 0.25]),
                                walks_per_node=10, p_halt=0.2, max_walk_length=3)
    kd = k.toarray()
    assert np.allclose(kd, kd.T, atol=1e-8)
    assert np.linalg.eigvalsh(kd).min() >= -1e-8


# ------------------------------------------------------------ golden vectors
def test_entry_points_match_reference(golden):
    from efficient_graph_gp.graph_kernels.fast_grf_kernel_diffusion import fast_diffusion_grf_kernel
    from efficient_graph_gp.graph_kernels.fast_grf_kernel_general import fast_general_grf_kernel as dense_k
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel as sk
    d = golden("entry_points")
    g = golden("small_graphs")
    nproc = int(d["cpu_count"][0])  # the host the vectors were made on
    f = [1.0, 0.5, 0.25]
    K = dense_k(g["readme_A"], f, walks_per_node=50, p_halt=0.1, max_walk_length=3, n_processes=nproc)
    np.testing.assert_allclose(K, d["readme_dense_K"], rtol=3e-5, atol=1e-6)
    assert abs(K[0, 0] - 2.1806250000000005) < 1e-4  # README quickstart value quoted in SURVEY.md
    K = fast_diffusion_grf_kernel(g["readme_A"], walks_per_node=50, p_halt=0.1, max_walk_length=3, beta=1.0,
                                  n_processes=nproc)
    np.testing.assert_allclose(K, d["readme_dense_diff_K"], rtol=3e-5, atol=1e-6)
    for name, ff, m, p, L in [("readme", f, 50, 0.1, 3), ("cycle4", f, 10, 0.2, 3),
                              ("er40", [1.0, -0.4, 0.3, 0.1, -0.05], 32, 0.15, 5)]:
        K = sk(sp.csr_matrix(g[f"{name}_A"]), ff, walks_per_node=m, p_halt=p, max_walk_length=L, n_processes=nproc)
        ref = d[f"{name}_sparse_K"]
        np.testing.assert_allclose(K.toarray(), ref, rtol=3e-5, atol=1e-6 * np.abs(ref).max())
    with pytest.raises(ValueError):
        dense_k(g["readme_A"], [1.0, 0.5], walks_per_node=5, max_walk_length=3)


def test_samplers_match_reference_bitwise(golden):
    from efficient_graph_gp.random_walk_samplers.sampler import Graph, RandomWalk
    from efficient_graph_gp_sparse.random_walk_samplers_sparse.sparse_sampler import SparseRandomWalk
    d = golden("small_graphs")
    for name in d["names"]:
        n = d[f"{name}_A"].shape[0]
        p = 0.0 if name == "perm12" else 0.2
        Ls = csr(d, f"{name}_Lsp", n)
        for nproc in (1, 3, 8):
            for seed in (None, 7):
                mats = SparseRandomWalk(Ls, seed=seed).get_random_walk_matrices(20, p, 4, n_processes=nproc)
                for l, M in enumerate(mats):
                    assert same_csr(M, csr(d, f"{name}_sp_n{nproc}_s{seed}_l{l}", n)), (name, nproc, seed, l)
        mats = SparseRandomWalk(sp.csr_matrix(d[f"{name}_A"]), seed=0).get_random_walk_matrices(15, 0.3, 3,
                                                                                               n_processes=2)
        for l, M in enumerate(mats):
            assert same_csr(M, csr(d, f"{name}_spA_l{l}", n)), (name, l)
        Ld = d[f"{name}_Ld"]
        for seed in (0, 5):
            F = RandomWalk(Graph(Ld), seed=seed).get_random_walk_matrices(12, p, 4, n_processes=1)
            assert np.array_equal(F, d[f"{name}_dseq_s{seed}"]), (name, seed)
        F = RandomWalk(Graph(Ld), seed=0).get_random_walk_matrices(12, p, 4, n_processes=1, ablation=True)
        assert np.array_equal(F, d[f"{name}_dabl_s0"]), name
        for nproc in (2, 3):
            key = f"{name}_dpar_n{nproc}"
            if key in d:
                F = RandomWalk(Graph(Ld), seed=None).get_random_walk_matrices(12, p, 4, n_processes=nproc)
                assert np.array_equal(F, d[key]), (name, nproc)


def test_laplacian_mirrors_bitwise(golden):
    from efficient_graph_gp.graph_kernels.utils import get_normalized_laplacian as lap_d
    from efficient_graph_gp.preprocessing.laplacian_np import get_laplacian, get_normalized_laplacian as lap_np
    from efficient_graph_gp_sparse.utils_sparse.graph_utils import get_normalized_laplacian as lap_sp
    d = golden("small_graphs")
    for name in d["names"]:
        A = d[f"{name}_A"]
        assert same_csr(lap_sp(sp.csr_matrix(A)), csr(d, f"{name}_Lsp", A.shape[0])), name
        assert np.array_equal(lap_d(A), d[f"{name}_Ld"]), name
        assert np.array_equal(lap_np(A), d[f"{name}_Lnp"]), name
        assert np.array_equal(get_laplacian(A), d[f"{name}_Lcomb"]), name


# ---------------------------------------------------------- GPyTorch surface
def _phi_dense(steps, f):
    return sum(fl * M.toarray() for fl, M in zip(f, steps))


def test_graph_preprocessor_and_sparse_kernels(golden, tmp_path):
    from efficient_graph_gp_sparse.gptorch_kernels_sparse import SparseDiffusionKernel, SparseGRFKernel
    from efficient_graph_gp_sparse.preprocessor import GraphPreprocessor
    d = golden("small_graphs")
    A = sp.csr_matrix(d["er40_A"])
    with pytest.raises(ValueError):
        GraphPreprocessor(sp.csr_matrix(np.ones((3, 4))))
    with pytest.raises(ValueError):
        GraphPreprocessor.from_scipy_csr(A.tocoo())
    cache = str(tmp_path / "steps.npz")
    pre = GraphPreprocessor(A, walks_per_node=20, p_halt=0.2, max_walk_length=4, random_walk_seed=7,
                            cache_filename=cache, n_processes=3)
    ops = pre.preprocess_graph(save_to_disk=True)
    assert len(ops) == 4 and all(op.sparse_csr_tensor.device.type == "cuda" for op in ops)
    for l, M in enumerate(pre.step_matrices_scipy):
        assert same_csr(M, csr(d, f"er40_sp_n3_s7_l{l}", 40)), l
    again = GraphPreprocessor(A, walks_per_node=20, p_halt=0.2, max_walk_length=4, random_walk_seed=7,
                              cache_filename=cache, load_from_disk=True)
    for M1, M2 in zip(again.step_matrices_scipy, pre.step_matrices_scipy):
        assert same_csr(M1, M2)
    with pytest.raises(FileNotFoundError):
        GraphPreprocessor(A, cache_filename=str(tmp_path / "missing.npz"), load_from_disk=True)

    kern = SparseGRFKernel(4, ops).cuda()
    x = torch.tensor([0, 3, 5], device="cuda")
    f = kern.modulator_vector.detach().cpu().numpy().astype(np.float64)
    Phi = _phi_dense(pre.step_matrices_scipy, f)
    np.testing.assert_allclose(kern(x, x).detach().cpu().numpy(), Phi[[0, 3, 5]] @ Phi[[0, 3, 5]].T,
                               rtol=2e-5, atol=1e-6)
    assert SparseDiffusionKernel(4, ops).cuda()().shape == (40, 40)


def test_gpflow_style_kernels(golden):
    """GPflow-surface wrappers (gpflow_kernels/general_kernel_fast_grf.py:9-77,
    diffusion_kernel_fast_grf.py:8-60; GPflow/TF absent: parity unpinned by the reference, pinned to
    the numpy restatement K = (F f)(F f)^T on the reference's own golden step tensors)."""
    import torch
    from efficient_graph_gp.gpflow_kernels import GraphDiffusionFastGRFKernel, GraphGeneralFastGRFKernel
    r = np.random.default_rng(8)
    U = np.triu((r.random((30, 30)) < 0.2).astype(float), 1)
    A = U + U.T
    with pytest.raises(AssertionError):
        GraphGeneralFastGRFKernel(np.ones((3, 4)))
    with pytest.raises(ValueError):
        GraphGeneralFastGRFKernel(A, max_walk_length=4, modulator_vector=[1.0, 2.0])
    k = GraphGeneralFastGRFKernel(A, walks_per_node=16, p_halt=0.2, max_walk_length=4)
    np.random.seed(42)
    np.testing.assert_array_equal(k.modulator_vector.detach().cpu().numpy(), np.random.randn(4))
    assert isinstance(k.modulator_vector, torch.nn.Parameter) and k.modulator_vector.requires_grad
    Phi = k.feature_matrices @ k.modulator_vector.detach().cpu().numpy()
    X = np.array([[0], [4], [29]])
    np.testing.assert_allclose(k.K(X), (Phi @ Phi.T)[np.ix_([0, 4, 29], [0, 4, 29])], rtol=3e-5, atol=1e-6)
    Kc = k._steps._K
    np.testing.assert_allclose(k.K_diag(X), np.diag(Phi @ Phi.T)[[0, 4, 29]], rtol=3e-5, atol=1e-6)
    assert k._steps._K is Kc  # K / K_diag gather from one cached Gram per modulator value
    # the golden step tensor of the reference's own dense sampler (step_matrices=)
    F = golden("small_graphs")["er40_dpar_n3"]
    f = np.array([0.9, -0.4, 0.2, 0.05])
    kg = GraphGeneralFastGRFKernel(golden("small_graphs")["er40_A"], max_walk_length=4, modulator_vector=f,
                                   step_matrices=F)
    P = F @ f
    np.testing.assert_allclose(kg.K(np.arange(40)), P @ P.T, rtol=3e-5, atol=1e-6 * np.abs(P @ P.T).max())
    # learnable: d sum(W * K[X, Y]) / d f against the analytic gradient
    W = r.standard_normal((3, 5))
    Y = np.array([1, 2, 3, 4, 39])
    (kg.K_torch(X, Y) * torch.tensor(W, device=kg.device)).sum().backward()
    xs = [0, 4, 29]
    gref = [np.sum(W * (F[xs, :, l] @ P[Y].T + P[xs] @ F[Y, :, l].T)) for l in range(4)]
    np.testing.assert_allclose(kg.modulator_vector.grad.cpu().numpy(), gref, rtol=1e-4, atol=1e-6)
    kd = GraphDiffusionFastGRFKernel(A, walks_per_node=16, p_halt=0.2, max_walk_length=4, beta=2.0, sigma_f=1.5)
    np.testing.assert_allclose([float(kd.beta), float(kd.sigma_f)], [2.0, 1.5], rtol=1e-12)
    fm = np.array([(-2.0) ** l / (2 ** l * np.prod(np.arange(1, l + 1))) for l in range(4)])
    Phi = kd.feature_matrices @ fm
    np.testing.assert_allclose(kd.K(np.arange(30)), 2.25 * Phi @ Phi.T, rtol=3e-5, atol=1e-6)
    # gradients w.r.t. beta and sigma_f: central differences of the numpy restatement
    (kd.K_torch(np.arange(30)) * torch.tensor(np.eye(30), device=kd.device)).sum().backward()

    def trace(beta, sig):
        f_ = np.array([(-beta) ** l / (2 ** l * np.prod(np.arange(1, l + 1))) for l in range(4)])
        P_ = kd.feature_matrices @ f_
        return sig ** 2 * np.trace(P_ @ P_.T)

    h = 1e-6
    gb = (trace(2.0 + h, 1.5) - trace(2.0 - h, 1.5)) / (2 * h) * (1 - np.exp(-2.0))  # d softplus = sigmoid
    gs = (trace(2.0, 1.5 + h) - trace(2.0, 1.5 - h)) / (2 * h) * (1 - np.exp(-1.5))
    np.testing.assert_allclose([kd.raw_beta.grad.item(), kd.raw_sigma_f.grad.item()], [gb, gs], rtol=1e-4)


def test_philox_mode_through_api_matches_oracle():
    from efficient_graph_gp_sparse.random_walk_samplers_sparse.sparse_sampler import SparseRandomWalk
    from oracle import oracle as O
    U = sp.random(500, 500, density=0.02, random_state=3, format="csr")
    A = ((U + U.T) > 0).astype(np.float64).tocsr()
    A.setdiag(0)
    A.eliminate_zeros()
    A.sort_indices()
    L, _ = O.laplacian_sparse(A)
    mats = SparseRandomWalk(L, seed=11, rng="philox").get_random_walk_matrices(24, 0.15, 5)
    ip, ix, dx = O._csr_arrays(L)
    node, load = O.walk_slots(ip, ix, dx, 24, 0.15, 5, rng=O.RNG_PHILOX, seed=11)
    ref = O.reduce_steps(node, load, O.NORM_MUL_RECIP)
    for a, b in zip(mats, ref):
        assert same_csr(a, b)


def test_sparse_entry_point_many_walks():
    """The drop-in sparse entry point with walks_per_node * max_walk_length > 4096 (the walk matrix
    goes through the step kernels instead of the fused Phi kernel), reference stream: step matrices
    bit-exact against the oracle, K within the K tolerance of the oracle's fp64 Gram."""
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel
    from oracle import oracle as O
    from test_gpu_parity import gram_close
    U = sp.random(300, 300, density=0.03, random_state=5, format="csr")
    A = ((U + U.T) > 0).astype(np.float64).tocsr()
    A.setdiag(0)
    A.eliminate_zeros()
    A.sort_indices()
    f = [1.0, -0.5, 0.25, -0.125, 0.0625, -0.03125, 0.015625, -0.0078125]
    K = fast_general_grf_kernel(A, f, walks_per_node=600, p_halt=0.2, max_walk_length=8, n_processes=3)
    L, _ = O.laplacian_sparse(A)
    ip, ix, dx = O._csr_arrays(L)
    node, load = O.walk_slots(ip, ix, dx, 600, 0.2, 8, rng=O.RNG_PCG64, seed=42, n_chunks=3)
    phi = O.phi_sparse(O.reduce_steps(node, load, O.NORM_MUL_RECIP), np.asarray(f))
    ok, fro = gram_close(K.toarray(), phi)
    assert ok, fro


def _degenerate_graphs():
    """Edge cases the path has to survive: one node, no edges, a star (one hub of degree n - 1),
    disjoint components with isolated nodes, a path, a weighted pair."""
    r = np.random.default_rng(0)
    star = np.zeros((200, 200))
    star[0, 1:] = star[1:, 0] = 1.0
    comp = np.zeros((60, 60))
    for a, b in [(0, 1), (1, 2), (2, 0), (10, 11), (30, 31), (31, 32), (32, 33)]:
        comp[a, b] = comp[b, a] = 1.0
    path = np.diag(np.ones(39), 1)
    path = path + path.T
    pair = np.array([[0.0, 2.5], [2.5, 0.0]])
    er = (r.random((90, 90)) < 0.04).astype(float)
    er = np.triu(er, 1)
    er = er + er.T
    return {"single": np.zeros((1, 1)), "empty": np.zeros((50, 50)), "star": star, "components": comp,
            "path": path, "pair": pair, "er_sparse": er}


@pytest.mark.parametrize("name", list(_degenerate_graphs()))
def test_degenerate_graphs_match_oracle(name):
    """Both drop-in entry points on degenerate graphs (reference stream, 3 chunks) against the C
    oracle's restatement of the reference: sparse K within the fp32 Gram tolerance, dense K too."""
    from efficient_graph_gp.graph_kernels.fast_grf_kernel_general import fast_general_grf_kernel as dense_k
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel as sk
    from oracle import oracle as O
    A = _degenerate_graphs()[name]
    f = [1.0, -0.5, 0.25, -0.125]
    m, p, L, nproc = 16, 0.2, 4, 3
    Ls, _ = O.laplacian_sparse(sp.csr_matrix(A))
    phi = O.phi_sparse(O.sparse_random_walk(Ls, m, p, L, n_processes=nproc, seed=None), f)
    ref = O.gram_rows(phi)
    K = sk(sp.csr_matrix(A), f, walks_per_node=m, p_halt=p, max_walk_length=L, n_processes=nproc)
    assert K.shape == A.shape
    np.testing.assert_allclose(K.toarray(), ref, rtol=3e-5, atol=1e-6 * max(np.abs(ref).max(), 1e-30))
    if A.shape[0] >= 2 * nproc:  # (below that the dense reference takes its sequential path)
        F = O.dense_random_walk(O.laplacian_dense(A, 0), m, p, L, n_processes=nproc, seed=42)
        Phi = np.einsum("ijl,l->ij", F, np.asarray(f))
        Kd = dense_k(A, f, walks_per_node=m, p_halt=p, max_walk_length=L, n_processes=nproc)
        np.testing.assert_allclose(Kd, Phi @ Phi.T, rtol=3e-5, atol=1e-6 * max(np.abs(Phi @ Phi.T).max(), 1e-30))


def test_sparse_api_philox_routes_through_bench_path(golden):
    """The drop-in sparse entry point (graph_kernels_sparse/fast_grf_kernel_general.py:20-55) with
    rng="philox" runs the benchmarked machinery: fused Philox walks straight to Phi rows (no visit
    slots) and the bench's K assembly, hub-column split included (Enron: hub_count = the bench's
    --hubs auto).  Its K equals the bench pipeline's K (grf_amd.pipeline, the code bench.py times)
    on the reference's Enron graph, bit for bit."""
    import math
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel
    from golden_util import snap_adjacency
    from grf_amd import pipeline as P
    from grf_amd.dist import setup_phi
    from grf_amd.engine import DeviceCSR, get_engine
    A = snap_adjacency(golden("snap"), "enron")
    n, m, L, p = A.shape[0], 128, 8, 0.1
    f = np.array([(-1.0) ** l / (2.0 ** l * math.factorial(l)) for l in range(L)])
    K_api = fast_general_grf_kernel(A, f, m, p, L, rng="philox", return_format="torch")
    eng = get_engine()
    A_dev = DeviceCSR.from_scipy(A, eng.device)
    pl = P.plan_step(n, m, L, p, f)
    pl.hubs = eng.hub_count(setup_phi(eng, A_dev, m, p, L, f))
    assert pl.mode == "sym" and pl.hubs > 0  # (Enron's hubs: the split is on)
    Kb, _ = P.kernel_step(eng, A_dev, pl)
    assert torch.equal(K_api, P.k_view(Kb, pl))
    del K_api, Kb


@pytest.mark.parametrize("n_rows,n_cols", [(1, 1), (3, 5), (7, 63), (130, 200), (1000, 1000)])
def test_dense_to_scipy_csr_matches_scipy(n_rows, n_cols):
    """The drop-in sparse entry point's return format, built on the device (grf_dense_to_csr_count /
    _fill): identical to scipy's own dense -> CSR of the float64-widened K (exact zeros and -0.0 dropped,
    sorted columns, empty rows), on ragged shapes and a pitched view."""
    from grf_amd.engine import get_engine
    eng = get_engine()
    r = np.random.default_rng(n_rows * 7 + n_cols)
    Kh = (r.standard_normal((n_rows, n_cols)) * (r.random((n_rows, n_cols)) < 0.4)).astype(np.float32)
    Kh[r.random((n_rows, n_cols)) < 0.05] = -0.0
    if n_rows > 2:
        Kh[1] = 0.0  # an empty row
    if (n_rows, n_cols) == (3, 5):
        Kh[:] = -0.0  # no entry at all (nnz = 0)
    pitch = -(-n_cols // 64) * 64 + 64
    Kd = torch.zeros((n_rows, pitch), dtype=torch.float32, device=eng.device)
    Kd[:, :n_cols] = torch.from_numpy(Kh).to(eng.device)
    got = eng.dense_to_scipy_csr(Kd[:, :n_cols])
    ref = sp.csr_matrix(Kh.astype(np.float64))
    ref.sort_indices()
    assert got.dtype == np.float64 and got.shape == ref.shape and got.has_sorted_indices
    assert np.array_equal(got.indptr, ref.indptr) and np.array_equal(got.indices, ref.indices)
    assert np.array_equal(got.data, ref.data)
