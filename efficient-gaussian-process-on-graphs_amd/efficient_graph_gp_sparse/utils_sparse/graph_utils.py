"""Sparse normalised Laplacian: mirror of utils_sparse/graph_utils.py:5-30 (computed on the GPU, bit-identical)."""
from grf_amd import api


def get_normalized_laplacian(adj_matrix):
    """D^-1/2 (D - A) D^-1/2 as scipy CSR (sorted columns, exact zeros dropped, diagonal stored)."""
    return api.sparse_laplacian(adj_matrix)
