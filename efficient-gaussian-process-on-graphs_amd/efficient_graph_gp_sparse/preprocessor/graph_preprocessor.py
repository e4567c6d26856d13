"""Graph preprocessor: mirror of efficient_graph_gp_sparse/preprocessor/graph_preprocessor.py:10-165.

Laplacian -> walks -> per-step matrices run on the GPU; the step matrices are
returned as ``SparseLinearOperator`` over torch CSR (float32 values, int64
indices) built from the device buffers directly -- no host round trip (the
reference builds them on the host and the experiments copy them over,
experiments/graph_bo/utils/device.py:9-14).  ``step_matrices_scipy`` (the
reference's attribute, used for the cache) is copied to the host only when read.

Cache format: the reference pickles a list of scipy matrices; this engine writes
a binary ``.npz`` bundle (per step: indptr, indices, data, shape) under the same
md5-keyed name with a ``.npz`` suffix, read back with ``allow_pickle=False``.
"""
import hashlib
import os
from typing import List, Optional

import numpy as np
import scipy.sparse as sp
import torch

from grf_amd import api
from grf_amd.engine import get_engine

from ..utils_sparse import SparseLinearOperator


class GraphPreprocessor:
    """Random-walk step matrices of a graph for GP kernels (reference :10-165)."""

    def __init__(self, adjacency_matrix: sp.csr_matrix, walks_per_node: int = 10, p_halt: float = 0.5,
                 max_walk_length: int = 10, random_walk_seed: int = 42, load_from_disk: bool = False,
                 use_tqdm: bool = True, cache_filename: Optional[str] = None, n_processes: int = None, *,
                 rng: Optional[str] = None, device=None) -> None:
        if adjacency_matrix.shape[0] != adjacency_matrix.shape[1]:
            raise ValueError("Adjacency matrix must be square.")
        self.adj_matrix = adjacency_matrix
        self.walks_per_node = walks_per_node
        self.p_halt = p_halt
        self.max_walk_length = max_walk_length
        self.random_walk_seed = random_walk_seed
        self.use_tqdm = use_tqdm
        self.cache_filename = cache_filename or self._generate_cache_filename()
        self.n_processes = n_processes
        self.rng = rng
        self.device = get_engine(device).device
        self._step_device = None
        self._step_scipy = None
        if load_from_disk:
            if os.path.exists(self.cache_filename):
                self.step_matrices_scipy = self.load_step_matrices(self.cache_filename)
                self.step_matrices_torch = [SparseLinearOperator(self._to_device(self.from_scipy_csr(m)))
                                            for m in self.step_matrices_scipy]
            else:
                raise FileNotFoundError(f"Cache file {self.cache_filename} not found.")

    def _generate_cache_filename(self) -> str:
        A = sp.csr_matrix(self.adj_matrix)
        adj_hash = hashlib.md5(A.data.tobytes() + A.indices.tobytes() + A.indptr.tobytes()).hexdigest()[:8]
        params = f"{A.shape[0]}_{self.walks_per_node}_{self.p_halt}_{self.max_walk_length}_{self.random_walk_seed}"
        return f"experiments_sparse/step_matrices/step_matrices_{adj_hash}_{params}.npz"

    def _to_device(self, t):
        return t.to(self.device)

    @property
    def step_matrices_scipy(self) -> List[sp.csr_matrix]:
        """The step matrices as scipy CSR (fp64), copied from the device on first access."""
        if self._step_scipy is None and self._step_device is not None:
            self._step_scipy = [M.to_scipy() for M in self._step_device]
        return self._step_scipy

    @step_matrices_scipy.setter
    def step_matrices_scipy(self, mats) -> None:
        self._step_scipy = mats

    def preprocess_graph(self, save_to_disk: bool = False) -> List[SparseLinearOperator]:
        """Laplacian -> walks -> step matrices on the GPU (reference :88-115); returns device-resident
        linear operators over torch CSR views of the device buffers (values cast to float32)."""
        self._step_scipy = None
        self._step_device = api.sparse_step_matrices_device(
            self.adj_matrix, self.walks_per_node, self.p_halt, self.max_walk_length, seed=self.random_walk_seed,
            n_processes=self.n_processes, rng=self.rng, device=self.device, laplacian=True)
        if save_to_disk:
            self.save_step_matrices(self.step_matrices_scipy, self.cache_filename)
        n = self.adj_matrix.shape[0]
        self.step_matrices_torch = [
            SparseLinearOperator(torch.sparse_csr_tensor(M.ptr, M.idx[:M.nnz].long(), M.val[:M.nnz].float(), (n, n),
                                                         dtype=torch.float32))
            for M in self._step_device]
        return self.step_matrices_torch

    @staticmethod
    def from_scipy_csr(scipy_csr: sp.csr_matrix) -> torch.Tensor:
        """scipy CSR -> torch sparse CSR (int64 crow/col, float32 values), as the reference (:117-139)."""
        if not isinstance(scipy_csr, sp.csr_matrix):
            raise ValueError("Input must be a scipy CSR matrix.")
        crow = torch.from_numpy(np.asarray(scipy_csr.indptr)).long()
        col = torch.from_numpy(np.asarray(scipy_csr.indices)).long()
        vals = torch.from_numpy(np.asarray(scipy_csr.data)).float()
        return torch.sparse_csr_tensor(crow, col, vals, (scipy_csr.shape[0], scipy_csr.shape[1]),
                                       dtype=torch.float32)

    @staticmethod
    def save_step_matrices(step_matrices: List[sp.csr_matrix], filename: str) -> None:
        """Binary CSR bundle (no pickle)."""
        d = {"n_steps": np.array([len(step_matrices)])}
        for l, m in enumerate(step_matrices):
            m = sp.csr_matrix(m)
            d[f"indptr_{l}"] = m.indptr
            d[f"indices_{l}"] = m.indices
            d[f"data_{l}"] = m.data
            d[f"shape_{l}"] = np.array(m.shape)
        dirname = os.path.dirname(filename)
        if dirname:
            os.makedirs(dirname, exist_ok=True)
        with open(filename, "wb") as fh:
            np.savez(fh, **d)

    @staticmethod
    def load_step_matrices(filename: str) -> List[sp.csr_matrix]:
        if filename.endswith(".pkl"):
            raise ValueError("pickle caches are not loaded (they can execute code); regenerate as .npz")
        with np.load(filename, allow_pickle=False) as z:
            return [sp.csr_matrix((z[f"data_{l}"], z[f"indices_{l}"], z[f"indptr_{l}"]), shape=tuple(z[f"shape_{l}"]))
                    for l in range(int(z["n_steps"][0]))]
