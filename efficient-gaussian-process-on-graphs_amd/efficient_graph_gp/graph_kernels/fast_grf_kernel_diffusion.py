"""Diffusion-modulated dense GRF kernel: mirror of graph_kernels/fast_grf_kernel_diffusion.py:7-21."""
from typing import Optional

import numpy as np

from grf_amd import api


def fast_diffusion_grf_kernel(adj_matrix, walks_per_node=50, p_halt=0.1, max_walk_length=10, beta=1.0, *,
                              rng: Optional[str] = None, n_processes: Optional[int] = None, device=None) -> np.ndarray:
    """fast_general_grf_kernel with f_l = (-beta)^l / (2^l l!), l < max_walk_length."""
    f = np.array([api.diffusion_modulator(step, beta) for step in range(max_walk_length)])
    return api.dense_kernel(adj_matrix, f, walks_per_node, p_halt, max_walk_length, seed=42, n_processes=n_processes,
                            rng=rng, device=device)
