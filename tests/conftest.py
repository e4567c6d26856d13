"""Shared pytest configuration.

Markers: ``gpu`` -- needs a real MI355X (run on the GPU box with ``-m gpu``).
Everything unmarked runs on CPU in the build container.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load


@pytest.fixture
def toy_cycle_adj() -> np.ndarray:
    """Undirected 4-node cycle adjacency (the reference's tests/conftest.py fixture)."""
    adj = np.zeros((4, 4))
    for u, v in [(0, 1), (1, 2), (2, 3), (3, 0)]:
        adj[u, v] = adj[v, u] = 1.0
    return adj


@pytest.fixture
def toy_cycle_csr(toy_cycle_adj):
    import scipy.sparse as sp
    return sp.csr_matrix(toy_cycle_adj)
