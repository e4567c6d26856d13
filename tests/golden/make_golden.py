"""Generate golden vectors by running the *reference* implementation.

Runs ONLY in the build container, where the read-only reference checkout is at
/root/reference.  The reference's sparse package imports ``linear_operator``
(absent here; an ordinary ImportError, no permission denial) through
``utils_sparse/__init__.py:2``; a tiny ``sys.modules`` stand-in for
``linear_operator.operators.LinearOperator`` is installed so the modules import.
No code path that generates these vectors touches that stand-in.

Outputs are data only (inputs + expected outputs) in ``tests/golden/*.npz``;
nothing from the reference's source is stored.  Re-run with
``python tests/golden/make_golden.py`` (takes ~1 minute on 8 cores).
"""
from __future__ import annotations

import hashlib
import os
import sys
import types

import numpy as np
import scipy.sparse as sp

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_linear_operator_standin():
    lo = types.ModuleType("linear_operator")
    ops = types.ModuleType("linear_operator.operators")

    class LinearOperator:  # pragma: no cover - only satisfies an import
        def __init__(self, *a, **k):
            pass

    ops.LinearOperator = LinearOperator
    lo.operators = ops
    sys.modules.setdefault("linear_operator", lo)
    sys.modules.setdefault("linear_operator.operators", ops)


def _install_gpflow_standin():
    """``efficient_graph_gp.gpflow_kernels`` imports gpflow and tensorflow at module level (absent here:
    an ordinary ImportError).  These stand-ins only let the module import, so that the numpy function
    ``compute_pstep_walk_matrix`` (general_kernel_pofm.py:7-42) can be called; no class or TF op is used."""
    class _Meta(type):
        def __getattr__(cls, name):  # gpflow.kernels.Kernel etc.: the placeholder class itself
            return cls

    class _Any(metaclass=_Meta):
        def __init__(self, *a, **k):
            pass

        def __getattr__(self, name):
            return _Any()

        def __call__(self, *a, **k):
            return _Any()

    def _module_getattr(attr):  # PEP 562: every public attribute is the placeholder class
        if attr.startswith("__"):
            raise AttributeError(attr)
        return _Any

    for name in ("gpflow", "tensorflow"):
        mod = types.ModuleType(name)
        mod.__getattr__ = _module_getattr
        sys.modules.setdefault(name, mod)


def pstep_golden():
    """Exact walk tensors E[M_l] = L^l for the statistical test of the Philox estimator: the
    reference's own compute_pstep_walk_matrix on the sparse Laplacians of the small graphs (and on
    the raw permutation matrix, walked as given)."""
    sys.path.insert(0, REF)
    _install_linear_operator_standin()
    _install_gpflow_standin()
    from efficient_graph_gp.gpflow_kernels.general_kernel_pofm import compute_pstep_walk_matrix
    from efficient_graph_gp_sparse.utils_sparse.graph_utils import get_normalized_laplacian as lap_sparse

    G = graphs()
    d = {"names": np.array(sorted(G)), "p_max": np.array([5])}
    for name in sorted(G):
        Ls = lap_sparse(sp.csr_matrix(G[name])).toarray()
        d[f"{name}_pstep"] = compute_pstep_walk_matrix(Ls, 5)
        # row-stochastic walk matrix P = D^-1 W (isolated rows stay zero): deg * w = 1, so the
        # estimator's loads stay bounded by (1-p)^-l and its CLT bounds are tight
        W = np.asarray(G[name], np.float64)
        deg = W.sum(axis=1)
        P = np.divide(W, deg[:, None], out=np.zeros_like(W), where=deg[:, None] > 0)
        d[f"{name}_P"] = P
        d[f"{name}_rw_pstep"] = compute_pstep_walk_matrix(P, 5)
    d["perm12_raw_pstep"] = compute_pstep_walk_matrix(G["perm12"], 5)
    np.savez_compressed(os.path.join(OUT, "pstep.npz"), **d)
    print("pstep fixtures written to", OUT)


def graphs():
    g = {}
    A = np.zeros((4, 4))
    for u, v in [(0, 1), (1, 2), (2, 3), (3, 0)]:
        A[u, v] = A[v, u] = 1.0
    g["cycle4"] = A
    g["readme"] = np.array([[0, 1, 1, 0], [1, 0, 0, 1], [1, 0, 0, 1], [0, 1, 1, 0]], dtype=float)
    r = np.random.default_rng(3)
    U = np.triu((r.random((40, 40)) < 0.15).astype(float), 1)
    g["er40"] = U + U.T
    r = np.random.default_rng(4)
    U = np.triu((r.random((30, 30)) < 0.2) * r.uniform(0.1, 2.0, (30, 30)), 1)
    g["wer30"] = U + U.T
    r = np.random.default_rng(5)
    U = np.triu((r.random((25, 25)) < 0.2).astype(float), 1)
    W = U + U.T
    W[3, :] = W[:, 3] = 0.0
    W[17, :] = W[:, 17] = 0.0
    W[5, 5] = 1.0
    g["iso25"] = W
    P = np.zeros((12, 12))
    perm = np.random.default_rng(6).permutation(12)
    P[np.arange(12), perm] = 1.0
    g["perm12"] = P
    S = np.zeros((10, 10))
    S[0, 1:] = S[1:, 0] = 1.0
    g["star10"] = S
    return g


def csr_pack(prefix, M, d):
    M = sp.csr_matrix(M)
    d[prefix + "_indptr"] = np.asarray(M.indptr, np.int64)
    d[prefix + "_indices"] = np.asarray(M.indices, np.int32)
    d[prefix + "_data"] = np.asarray(M.data, np.float64)


def digest_csr(M) -> str:
    M = sp.csr_matrix(M)
    h = hashlib.sha256()
    for a in (np.asarray(M.indptr, np.int64), np.asarray(M.indices, np.int32), np.asarray(M.data, np.float64)):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    sys.path.insert(0, REF)
    _install_linear_operator_standin()
    from efficient_graph_gp.graph_kernels.fast_grf_kernel_diffusion import fast_diffusion_grf_kernel
    from efficient_graph_gp.graph_kernels.fast_grf_kernel_general import fast_general_grf_kernel as dense_kernel
    from efficient_graph_gp.graph_kernels.utils import get_normalized_laplacian as lap_dense
    from efficient_graph_gp.modulation_functions import diffusion_modulator
    from efficient_graph_gp.preprocessing.laplacian_np import get_laplacian as lap_comb
    from efficient_graph_gp.preprocessing.laplacian_np import get_normalized_laplacian as lap_np
    from efficient_graph_gp.random_walk_samplers.sampler import Graph, RandomWalk
    from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import (
        fast_general_grf_kernel as sparse_kernel,
    )
    from efficient_graph_gp_sparse.random_walk_samplers_sparse.sparse_sampler import SparseRandomWalk
    from efficient_graph_gp_sparse.utils_sparse.graph_utils import get_normalized_laplacian as lap_sparse

    meta = {"numpy": np.__version__, "cpu_count": os.cpu_count()}

    # ---- 1. RNG streams straight from numpy (Generator.random / integers / choice)
    d = {}
    for si, seed in enumerate([0, 1, 42, 43, 2**40 + 5, 2**70 + 3]):
        r = np.random.default_rng(seed)
        ops = np.array([0 if t % 3 == 0 else ((t * 7919) % 50) + 1 for t in range(600)], np.uint32)
        out = np.array([r.random() if o == 0 else float(r.integers(int(o))) for o in ops])
        st = np.random.default_rng(seed).bit_generator.state["state"]
        d[f"seed{si}"] = np.array([seed], dtype=object).astype(str)
        d[f"ops{si}"] = ops
        d[f"out{si}"] = out
        d[f"state{si}"] = np.array([str(st["state"]), str(st["inc"])])
    np.savez_compressed(os.path.join(OUT, "rng.npz"), **d)

    # ---- 2. Laplacians + 3. samplers on every small graph
    G = graphs()
    d = {"names": np.array(sorted(G))}
    for name in sorted(G):
        A = G[name]
        Acsr = sp.csr_matrix(A)
        d[f"{name}_A"] = A
        Ls = lap_sparse(Acsr)
        csr_pack(f"{name}_Lsp", Ls, d)
        d[f"{name}_Ld"] = lap_dense(A)
        d[f"{name}_Lnp"] = lap_np(A)
        d[f"{name}_Lcomb"] = lap_comb(A)
        p = 0.0 if name == "perm12" else 0.2
        # sparse sampler on the Laplacian (the path the entry point takes) and on raw A
        for nproc in (1, 3, 8):
            for seed in (None, 7):
                mats = SparseRandomWalk(Ls, seed=seed).get_random_walk_matrices(20, p, 4, n_processes=nproc)
                for l, M in enumerate(mats):
                    csr_pack(f"{name}_sp_n{nproc}_s{seed}_l{l}", M, d)
        mats = SparseRandomWalk(Acsr, seed=0).get_random_walk_matrices(15, 0.3, 3, n_processes=2)
        for l, M in enumerate(mats):
            csr_pack(f"{name}_spA_l{l}", M, d)
        # dense sampler: sequential (non-cumulative / ablation) and pool paths
        Ld = lap_dense(A)
        for seed in (0, 5):
            F = RandomWalk(Graph(Ld), seed=seed).get_random_walk_matrices(12, p, 4, n_processes=1)
            d[f"{name}_dseq_s{seed}"] = F
        d[f"{name}_dabl_s0"] = RandomWalk(Graph(Ld), seed=0).get_random_walk_matrices(
            12, p, 4, n_processes=1, ablation=True)
        for nproc in (2, 3):
            if A.shape[0] >= 2 * nproc:
                d[f"{name}_dpar_n{nproc}"] = RandomWalk(Graph(Ld), seed=None).get_random_walk_matrices(
                    12, p, 4, n_processes=nproc)
    np.savez_compressed(os.path.join(OUT, "small_graphs.npz"), **d)

    # ---- 4. entry points (README quickstart + reference tests' fixtures)
    d = {}
    A = G["readme"]
    f = np.array([1.0, 0.5, 0.25])
    d["readme_dense_K"] = dense_kernel(A, f, walks_per_node=50, p_halt=0.1, max_walk_length=3)
    d["readme_dense_diff_K"] = fast_diffusion_grf_kernel(A, walks_per_node=50, p_halt=0.1, max_walk_length=3, beta=1.0)
    d["readme_sparse_K"] = sparse_kernel(sp.csr_matrix(A), f, walks_per_node=50, p_halt=0.1,
                                         max_walk_length=3).toarray()
    d["cycle4_sparse_K"] = sparse_kernel(sp.csr_matrix(G["cycle4"]), f, walks_per_node=10, p_halt=0.2,
                                         max_walk_length=3).toarray()
    d["er40_sparse_K"] = sparse_kernel(sp.csr_matrix(G["er40"]), [1.0, -0.4, 0.3, 0.1, -0.05], walks_per_node=32,
                                       p_halt=0.15, max_walk_length=5).toarray()
    d["diff_mod_b1"] = np.array([diffusion_modulator(l, 1.0) for l in range(8)])
    d["diff_mod_b2"] = np.array([diffusion_modulator(l, 2.5) for l in range(8)])
    d["cpu_count"] = np.array([os.cpu_count()])
    np.savez_compressed(os.path.join(OUT, "entry_points.npz"), **d)

    # ---- 5. Cora (real graph shipped with the reference): sparse path
    cites = np.loadtxt(os.path.join(REF, "experiments/dense/cora/data/cora/cora.cites"), dtype=np.int64)
    ids, inv = np.unique(cites.ravel(), return_inverse=True)
    e = inv.reshape(-1, 2)
    n = len(ids)
    C = sp.coo_matrix((np.ones(len(e)), (e[:, 0], e[:, 1])), shape=(n, n)).tocsr()
    C = ((C + C.T) > 0).astype(np.float64).tocsr()
    C.setdiag(0)
    C.eliminate_zeros()
    C.sort_indices()
    d = {}
    csr_pack("A", C, d)
    Lc = lap_sparse(C)
    d["L_digest"] = np.array([digest_csr(Lc)])
    mats = SparseRandomWalk(Lc, seed=None).get_random_walk_matrices(16, 0.1, 4, n_processes=8)
    for l, M in enumerate(mats):
        csr_pack(f"m16_l{l}", M, d)
    mats = SparseRandomWalk(Lc, seed=None).get_random_walk_matrices(128, 0.1, 8, n_processes=8)
    d["m128_digests"] = np.array([digest_csr(M) for M in mats])
    fmod = np.array([diffusion_modulator(l, 1.0) for l in range(8)])
    Phi = sp.csr_matrix((n, n))
    for l, fp in enumerate(fmod):
        Phi += fp * mats[l]
    d["m128_phi_digest"] = np.array([digest_csr(Phi)])
    K = (Phi @ Phi.T)
    d["m128_K_rows0_16"] = K[:16].toarray()
    d["m128_K_diag"] = K.diagonal()
    d["m128_K_fro"] = np.array([sp.linalg.norm(K)])
    np.savez_compressed(os.path.join(OUT, "cora.npz"), **d)

    with open(os.path.join(OUT, "META.txt"), "w") as fh:
        for k, v in meta.items():
            fh.write(f"{k}: {v}\n")
    print("golden vectors written to", OUT, meta)


if __name__ == "__main__":
    if sys.argv[1:] == ["pstep"]:
        pstep_golden()
    else:
        main()
        pstep_golden()
