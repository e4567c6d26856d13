"""Golden vectors for the two real social graphs the reference ships (SURVEY.md §8d cross-checks).

Runs ONLY in the build container (needs /root/reference).  Inputs are the SNAP / MUSAE edge lists
the reference holds as data files:
  experiments/sparse/social_networks/facebook/facebook_large/musae_facebook_edges.csv  (22,470 nodes)
  experiments/sparse/social_networks/enron/email-Enron.txt.gz                          (36,692 nodes)
The adjacency is built with the reference loaders' semantics (networkx Graph in edge-insertion
order, ``nx.adjacency_matrix(G).tocsr()``: experiments/graph_bo/data/database.py:196-215 facebook,
:265-287 enron), self-loops included as the loaders keep them.  Expected outputs come from the
reference's own sparse path run here: its Laplacian (utils_sparse/graph_utils.py:5-30), its
SparseRandomWalk sampler (sparse_sampler.py, 8 processes, seed None -> 42 + chunk), Phi with the
diffusion modulator, and rows of K = Phi Phi^T.  Stored: A as CSR, sha256 digests of L / every
step matrix / Phi, six rows of K (CSR) and diag(K).  Data only; re-run with
``python tests/golden/make_snap.py`` (~2 minutes on 8 cores).
"""
from __future__ import annotations

import gzip
import os
import sys

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden import REF, _install_linear_operator_standin, digest_csr  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SOC = os.path.join(REF, "experiments/sparse/social_networks")
# (walks_per_node, p_halt, max_walk_length) of the cross-check: the headline's p and L, fewer walks
WALK = {"facebook": (32, 0.1, 8), "enron": (32, 0.1, 8)}


def _nx_adjacency(edges):
    import networkx as nx
    G = nx.Graph()
    G.add_edges_from(edges)
    return nx.adjacency_matrix(G).tocsr()


def load_facebook():
    e = np.loadtxt(os.path.join(SOC, "facebook/facebook_large/musae_facebook_edges.csv"), delimiter=",",
                   skiprows=1, dtype=np.int64)
    return _nx_adjacency(map(tuple, e.tolist()))


def load_enron():
    rows = []
    with gzip.open(os.path.join(SOC, "enron/email-Enron.txt.gz"), "rt") as fh:
        for line in fh:
            if not line.startswith("#"):
                u, v = line.split()
                rows.append((int(u), int(v)))
    return _nx_adjacency(rows)


def main():
    sys.path.insert(0, REF)
    _install_linear_operator_standin()
    from efficient_graph_gp.modulation_functions import diffusion_modulator
    from efficient_graph_gp_sparse.random_walk_samplers_sparse.sparse_sampler import SparseRandomWalk
    from efficient_graph_gp_sparse.utils_sparse.graph_utils import get_normalized_laplacian as lap_sparse

    d = {}
    for name, loader in (("facebook", load_facebook), ("enron", load_enron)):
        A = loader().astype(np.float64)
        A.sort_indices()
        n = A.shape[0]
        m, p, L = WALK[name]
        d[f"{name}_indptr"] = np.asarray(A.indptr, np.int32)
        d[f"{name}_indices"] = np.asarray(A.indices, np.int32)
        d[f"{name}_walk"] = np.array([m, p, L], np.float64)
        Ls = lap_sparse(A)
        d[f"{name}_L_digest"] = np.array([digest_csr(Ls)])
        mats = SparseRandomWalk(Ls, seed=None).get_random_walk_matrices(m, p, L, n_processes=8)
        d[f"{name}_step_digests"] = np.array([digest_csr(M) for M in mats])
        fmod = np.array([diffusion_modulator(l, 1.0) for l in range(L)])
        Phi = sp.csr_matrix((n, n))
        for l, fp in enumerate(fmod):
            Phi += fp * mats[l]
        d[f"{name}_phi_digest"] = np.array([digest_csr(Phi)])
        d[f"{name}_phi_nnz"] = np.array([Phi.nnz])
        # rows 0..2 and the three highest-degree nodes (hubs: the heaviest Gram rows), stored sparse
        deg = np.diff(A.indptr)
        krows = np.r_[0, 1, 2, np.argsort(-deg, kind="stable")[:3]].astype(np.int64)
        Kr = sp.csr_matrix(Phi[krows] @ Phi.T)
        Kr.sort_indices()
        d[f"{name}_K_rows"] = krows
        d[f"{name}_K_rows_indptr"] = np.asarray(Kr.indptr, np.int32)
        d[f"{name}_K_rows_indices"] = np.asarray(Kr.indices, np.int32)
        d[f"{name}_K_rows_data"] = np.asarray(Kr.data, np.float64)
        d[f"{name}_K_diag"] = np.asarray(Phi.multiply(Phi).sum(axis=1)).ravel()
        print(name, n, A.nnz, "Phi nnz", Phi.nnz, flush=True)
    np.savez_compressed(os.path.join(OUT, "snap.npz"), **d)


if __name__ == "__main__":
    main()
