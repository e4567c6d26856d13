"""Sparse-path GRF kernel: mirror of efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:20-55."""
from typing import Optional, Sequence

from grf_amd import api


def fast_general_grf_kernel(adj_matrix, modulator_vector: Sequence[float], walks_per_node: int = 50,
                            p_halt: float = 0.1, max_walk_length: int = 10, *, rng: Optional[str] = None,
                            n_processes: Optional[int] = None, return_format: str = "scipy", device=None):
    """K ~= Phi Phi^T with Phi = sum_l f_l M_l on the normalised Laplacian of a CSR graph.

    As in the reference: scipy-semantics Laplacian, ``SparseRandomWalk(L, seed=None)``
    (base seed 42) with ``n_processes = os.cpu_count()`` chunks unless given, steps
    beyond ``len(modulator_vector)`` ignored, exact zeros dropped.  K is computed on
    the GPU in float32 and returned as scipy CSR (default, like the reference) or,
    with ``return_format="torch"``, as a dense float32 tensor left in HBM (the only
    viable form at N ~ 1e5, where the reference cannot materialise K).
    """
    return api.sparse_kernel(adj_matrix, modulator_vector, walks_per_node, p_halt, max_walk_length,
                             n_processes=n_processes, rng=rng, return_format=return_format, device=device)
