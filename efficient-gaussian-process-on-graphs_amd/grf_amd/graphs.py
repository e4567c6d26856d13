"""Synthetic and shipped graphs of the benchmark configurations.

* ``er_graph_exact_edges``: C4 / C2 -- undirected Erdos-Renyi with an exact edge count.
* ``powerlaw_graph``: C5 -- Chung-Lu graph with a power-law expected degree sequence.
* ``snap_graph``: the Facebook (22,470 nodes) and Enron (36,692 nodes) social graphs the
  reference ships under experiments/sparse/social_networks/, as committed in
  tests/golden/snap.npz (built with the reference loaders' semantics, see make_snap.py).

All return a scipy CSR adjacency (float64 unit weights, sorted indices).
"""
from __future__ import annotations

import os

import numpy as np
import scipy.sparse as sp

_SNAP = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                     "tests", "golden", "snap.npz")


def er_graph_exact_edges(n: int, n_edges: int, seed: int = 0) -> sp.csr_matrix:
    """Undirected Erdos-Renyi graph with exactly n_edges distinct edges, unit weights, no self-loops."""
    rng = np.random.default_rng(seed)
    keys = np.empty(0, np.int64)
    while keys.size < n_edges:
        k = n_edges - keys.size
        u = rng.integers(0, n, int(k * 1.2) + 16)
        v = rng.integers(0, n, int(k * 1.2) + 16)
        lo, hi = np.minimum(u, v), np.maximum(u, v)
        cand = (lo * n + hi)[lo != hi]
        keys = np.concatenate([keys, cand])
        _, first = np.unique(keys, return_index=True)
        keys = keys[np.sort(first)]
    keys = keys[:n_edges]
    u, v = keys // n, keys % n
    A = sp.coo_matrix((np.ones(2 * n_edges), (np.r_[u, v], np.r_[v, u])), shape=(n, n)).tocsr()
    A.sort_indices()
    return A


def powerlaw_graph(n: int, avg_degree: float = 10.0, exponent: float = 2.5, seed: int = 0) -> sp.csr_matrix:
    """Undirected Chung-Lu graph: node i has expected degree proportional to (i + i0)^(-1/(exponent-1))
    (a power-law degree distribution with the given exponent), scaled to ``avg_degree``.
    n * avg_degree / 2 endpoint pairs are drawn in proportion to the weights; self-loops and
    repeated pairs are dropped (so the realised mean degree is slightly lower).  Unit weights."""
    rng = np.random.default_rng(seed)
    i0 = 10.0
    w = (np.arange(n, dtype=np.float64) + i0) ** (-1.0 / (exponent - 1.0))
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    n_pairs = int(n * avg_degree / 2)
    u = np.searchsorted(cdf, rng.random(n_pairs), side="right")
    v = np.searchsorted(cdf, rng.random(n_pairs), side="right")
    np.minimum(u, n - 1, out=u)
    np.minimum(v, n - 1, out=v)
    lo, hi = np.minimum(u, v), np.maximum(u, v)
    keys = np.unique((lo * n + hi)[lo != hi])
    u, v = keys // n, keys % n
    # a random relabelling: hubs are not clustered at the low node ids
    perm = rng.permutation(n)
    u, v = perm[u], perm[v]
    A = sp.coo_matrix((np.ones(2 * len(keys)), (np.r_[u, v], np.r_[v, u])), shape=(n, n)).tocsr()
    A.sort_indices()
    return A


def snap_graph(name: str) -> sp.csr_matrix:
    """The reference's shipped social graph ``name`` ("facebook" or "enron"), as its loaders build it."""
    d = np.load(_SNAP, allow_pickle=False)
    if name + "_indptr" not in d.files:
        raise ValueError(f"unknown graph {name!r} (have: facebook, enron)")
    ip, ix = d[name + "_indptr"], d[name + "_indices"]
    n = len(ip) - 1
    return sp.csr_matrix((np.ones(len(ix)), ix, ip), shape=(n, n))
