"""Diffusion fast GRF kernel: mirror of gpflow_kernels/diffusion_kernel_fast_grf.py:8-60."""
from typing import Optional

import numpy as np

from grf_amd import _lib as C
from grf_amd import api


class GraphDiffusionFastGRFKernel:
    def __init__(self, adjacency_matrix, walks_per_node: int = 50, p_halt: float = 0.1, max_walk_length: int = 10,
                 beta: float = 2.0, sigma_f: float = 1.0, random_walk_seed: int = 42, normalize_laplacian: bool = True,
                 use_tqdm: bool = False, *, rng: Optional[str] = None, device=None, **kwargs):
        adjacency_matrix = np.asarray(adjacency_matrix, dtype=np.float64)
        assert adjacency_matrix.shape[0] == adjacency_matrix.shape[1], "Adjacency matrix must be square."
        if beta <= 0 or sigma_f <= 0:
            raise ValueError("beta and sigma_f must be positive")
        self.adjacency_matrix = adjacency_matrix
        self.walks_per_node = walks_per_node
        self.p_halt = p_halt
        self.max_walk_length = max_walk_length
        self.beta = float(beta)
        self.sigma_f = float(sigma_f)
        self.device = device
        mode = C.LAP_NUMPY_SAFE if normalize_laplacian else C.LAP_COMBINATORIAL
        self.laplacian = api.dense_laplacian(adjacency_matrix, mode, device)
        self.feature_matrices = api.dense_step_tensor(self.laplacian, walks_per_node, p_halt, max_walk_length,
                                                      seed=random_walk_seed, rng=rng, device=device)

    def grf_kernel(self, beta, sigma_f) -> np.ndarray:
        f = np.array([api.diffusion_modulator(l, float(beta)) for l in range(self.max_walk_length)])
        return float(sigma_f) ** 2 * api.gram_from_features(self.feature_matrices, f, self.device)

    def K(self, X1, X2=None) -> np.ndarray:
        X2 = X1 if X2 is None else X2
        Kf = self.grf_kernel(self.beta, self.sigma_f)
        i1 = np.asarray(X1).reshape(-1).astype(np.int64)
        i2 = np.asarray(X2).reshape(-1).astype(np.int64)
        return Kf[np.ix_(i1, i2)]

    def K_diag(self, X) -> np.ndarray:
        Kf = self.grf_kernel(self.beta, self.sigma_f)
        return np.diag(Kf)[np.asarray(X).reshape(-1).astype(np.int64)]

    def __call__(self, X1, X2=None, full_cov=True):
        return self.K(X1, X2) if full_cov else self.K_diag(X1)
