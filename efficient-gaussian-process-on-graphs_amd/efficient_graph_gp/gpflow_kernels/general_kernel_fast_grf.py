"""General-modulator fast GRF kernel: mirror of gpflow_kernels/general_kernel_fast_grf.py:9-77.

The (N, N, L) step tensor is sampled once at construction on the GPU (Laplacian
with safe degrees as in preprocessing/laplacian_np.py, or the raw adjacency with
the ablation rule); ``K`` computes Phi = F f and K = Phi Phi^T on the GPU (fp32
MFMA) and gathers rows / columns by the integer node indices in X.
"""
from typing import Optional

import numpy as np

from grf_amd import _lib as C
from grf_amd import api


class GraphGeneralFastGRFKernel:
    def __init__(self, adjacency_matrix, walks_per_node: int = 50, p_halt: float = 0.1, max_walk_length: int = 10,
                 random_walk_seed: int = 42, modulator_vector: np.ndarray = None, step_matrices: np.ndarray = None,
                 use_tqdm: bool = False, ablation: bool = False, *, rng: Optional[str] = None, device=None, **kwargs):
        adjacency_matrix = np.asarray(adjacency_matrix, dtype=np.float64)
        assert adjacency_matrix.shape[0] == adjacency_matrix.shape[1], "Adjacency matrix must be square."
        self.adjacency_matrix = adjacency_matrix
        self.walks_per_node = walks_per_node
        self.p_halt = p_halt
        self.max_walk_length = max_walk_length
        self.device = device
        if modulator_vector is None:
            np.random.seed(42)
            self.modulator_vector = np.random.randn(max_walk_length)
        else:
            if len(modulator_vector) != max_walk_length:
                raise ValueError("The length of the modulator vector must be equal to the max_walk_length.")
            self.modulator_vector = np.asarray(modulator_vector, dtype=np.float64)
        if step_matrices is not None:
            self.feature_matrices = np.asarray(step_matrices, dtype=np.float64)
        elif ablation:
            self.feature_matrices = api.dense_step_tensor(adjacency_matrix, walks_per_node, p_halt, max_walk_length,
                                                          seed=random_walk_seed, ablation=True, rng=rng,
                                                          device=device)
        else:
            self.laplacian = api.dense_laplacian(adjacency_matrix, C.LAP_NUMPY_SAFE, device)
            self.feature_matrices = api.dense_step_tensor(self.laplacian, walks_per_node, p_halt, max_walk_length,
                                                          seed=random_walk_seed, rng=rng, device=device)

    def grf_kernel(self, modulator_vector) -> np.ndarray:
        return api.gram_from_features(self.feature_matrices, modulator_vector, self.device)

    def K(self, X1, X2=None) -> np.ndarray:
        X2 = X1 if X2 is None else X2
        Kf = self.grf_kernel(self.modulator_vector)
        i1 = np.asarray(X1).reshape(-1).astype(np.int64)
        i2 = np.asarray(X2).reshape(-1).astype(np.int64)
        return Kf[np.ix_(i1, i2)]

    def K_diag(self, X) -> np.ndarray:
        Kf = self.grf_kernel(self.modulator_vector)
        return np.diag(Kf)[np.asarray(X).reshape(-1).astype(np.int64)]

    def __call__(self, X1, X2=None, full_cov=True):
        return self.K(X1, X2) if full_cov else self.K_diag(X1)
