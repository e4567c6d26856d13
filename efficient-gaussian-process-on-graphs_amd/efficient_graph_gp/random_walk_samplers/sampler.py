"""Dense random-walk sampler: mirror of efficient_graph_gp/random_walk_samplers/sampler.py:63-203.

``Graph`` wraps a dense walk matrix; ``RandomWalk.get_random_walk_matrices``
returns the (N, N, L) float64 occupancy tensor.  The reference's path selection
is kept: one sequential ``default_rng(seed)`` stream with the non-cumulative (or
ablation) load rule when ``n_processes == 1 or N < 2 * n_processes``
(sampler.py:115-116,148-186); otherwise chunks seeded ``(seed or 42) + i`` with the
cumulative rule (sampler.py:119-146).  All walks run on the GPU.
"""
from typing import Optional

import numpy as np

from grf_amd import api


class Graph:
    """Dense walk matrix holder (reference sampler.py:63-82)."""

    def __init__(self, adjacency_matrix: Optional[np.ndarray] = None) -> None:
        if adjacency_matrix is not None:
            self.adjacency_matrix = adjacency_matrix
            self.num_nodes = adjacency_matrix.shape[0]
        else:
            self.adjacency_matrix = None
            self.num_nodes = 0

    def get_neighbors(self, node: int) -> np.ndarray:
        return np.flatnonzero(self.adjacency_matrix[node])

    def get_num_nodes(self) -> int:
        return self.num_nodes

    def get_edge_weight(self, node1: int, node2: int) -> float:
        return self.adjacency_matrix[node1, node2]


class RandomWalk:
    """Step-resolved random-walk occupancies (reference sampler.py:85-203)."""

    def __init__(self, graph: Graph, seed: Optional[int] = None, *, rng: Optional[str] = None, device=None) -> None:
        self.graph = graph
        self.seed_arg = seed          # the sequential path's default_rng(seed)
        self.seed = seed or 42        # the pool path's base seed
        self.rng = rng
        self.device = device

    def get_random_walk_matrices(self, num_walks: int, p_halt: float, max_walk_length: int, use_tqdm: bool = False,
                                 n_processes: Optional[int] = None, ablation: bool = False) -> np.ndarray:
        if self.graph.get_num_nodes() == 0:
            return np.zeros((0, 0, max_walk_length))
        return api.dense_step_tensor(self.graph.adjacency_matrix, num_walks, p_halt, max_walk_length,
                                     seed=self.seed_arg, n_processes=n_processes, ablation=ablation, rng=self.rng,
                                     device=self.device)
