"""CSR random-walk sampler: mirror of random_walk_samplers_sparse/sparse_sampler.py:59-132.

The reference forks ``n_processes`` workers, each consuming one numpy PCG64 stream
(seed ``(seed or 42) + i``) over a contiguous node chunk, and merges Python dicts.
Here every chunk's stream is replayed on the GPU (``rng="reference"``, bit-identical
step matrices) or all walks run with Philox (``rng="philox"``); the per-(source,
step) reduction, normalisation (``* (1/m)``) and CSR assembly are HIP kernels.
"""
from typing import List, Optional

import numpy as np
import scipy.sparse as sp

from grf_amd import api


class SparseRandomWalk:
    """Per-step occupancy matrices of random walks on a CSR matrix (reference :59-132)."""

    def __init__(self, adjacency_matrix: sp.spmatrix, seed: Optional[int] = None, *, rng: Optional[str] = None,
                 device=None) -> None:
        self.adjacency = adjacency_matrix.tocsr()
        self.num_nodes = self.adjacency.shape[0]
        self.seed = seed or 42
        self.indptr = self.adjacency.indptr
        self.indices = self.adjacency.indices
        self.data = self.adjacency.data.astype(float, copy=False)
        self.rng = rng
        self.device = device

    def get_random_walk_matrices(self, num_walks: int, p_halt: float, max_walk_length: int, use_tqdm: bool = False,
                                 n_processes: Optional[int] = None) -> List[sp.csr_matrix]:
        """List of ``max_walk_length`` CSR matrices (N, N): entry (i, j) of step l is the
        load-weighted number of visits to j at step l of the walks from i, times 1/num_walks."""
        if self.num_nodes == 0:
            return [sp.csr_matrix((0, 0)) for _ in range(max_walk_length)]
        return api.sparse_step_matrices(self.adjacency, num_walks, p_halt, max_walk_length, seed=self.seed,
                                        n_processes=n_processes, rng=self.rng, device=self.device)
