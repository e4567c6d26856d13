"""Dense-path GRF kernel: mirror of efficient_graph_gp/graph_kernels/fast_grf_kernel_general.py:11-39."""
from typing import Optional, Sequence

import numpy as np

from grf_amd import api


def fast_general_grf_kernel(adj_matrix: np.ndarray, modulator_vector: Sequence[float], walks_per_node: int = 50,
                            p_halt: float = 0.1, max_walk_length: int = 10, *, rng: Optional[str] = None,
                            n_processes: Optional[int] = None, device=None) -> np.ndarray:
    """K ~= Phi Phi^T on the normalised Laplacian of a dense adjacency (reference :11-39).

    Laplacian (numpy semantics), walks with seed 42 and the reference's path
    selection (sequential when N < 2 * n_processes), Phi = F f, K = Phi Phi^T
    (fp32 MFMA on the GPU, returned as float64).  ``modulator_vector`` must have
    ``max_walk_length`` entries (the reference's matmul raises otherwise).
    """
    return api.dense_kernel(adj_matrix, modulator_vector, walks_per_node, p_halt, max_walk_length, seed=42,
                            n_processes=n_processes, rng=rng, device=device)
