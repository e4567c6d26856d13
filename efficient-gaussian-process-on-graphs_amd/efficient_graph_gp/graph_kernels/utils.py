"""Laplacian helpers: mirror of efficient_graph_gp/graph_kernels/utils.py:6-47."""
import numpy as np

from grf_amd import _lib as C
from grf_amd import api


def get_normalized_laplacian(W, sparse=False):
    """I - D^-1/2 W D^-1/2 (numpy semantics, bit-identical) computed on the GPU.

    ``sparse=True`` returns scipy CSR with the sparse package's semantics
    (utils_sparse/graph_utils.py), which can differ from the reference's own
    sparse branch of this helper in the last ulp of the diagonal.
    """
    if sparse:
        return api.sparse_laplacian(W)
    return api.dense_laplacian(W, C.LAP_NUMPY)


def generate_noisy_samples(K, noise_std=0.1, seed=42):
    """GP sample + noise for experiments (reference utils.py:30-47); host numpy, not on the GRF path."""
    np.random.seed(seed)
    n = K.shape[0]
    chol = np.linalg.cholesky(K + 1e-6 * np.eye(n))
    true_samples = chol @ np.random.normal(size=(n, 1))
    return true_samples + noise_std * np.random.randn(n, 1)
