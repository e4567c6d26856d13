"""Drop-in API on C2 (G(10k, 0.001), m = 128, L = 8): the sparse entry point in reference-stream mode (PCG64
replay, n_processes chunks) and Philox mode, wall time per call (K returned as scipy CSR, as the reference does)."""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from efficient_graph_gp_sparse.graph_kernels_sparse.fast_grf_kernel_general import fast_general_grf_kernel  # noqa

r = np.random.default_rng(0)
n = 10_000
A = sp.random(n, n, density=0.001, random_state=1, format="csr")
A = ((A + A.T) > 0).astype(np.float64)
A.setdiag(0)
A.eliminate_zeros()
f = [(-1.0) ** l / 2.0 ** l for l in range(8)]
for rng, nproc in (("reference", 8), ("reference", 64), ("philox", 8)):
    fast_general_grf_kernel(A, f, walks_per_node=128, p_halt=0.1, max_walk_length=8, rng=rng, n_processes=nproc)
    t = time.perf_counter()
    K = fast_general_grf_kernel(A, f, walks_per_node=128, p_halt=0.1, max_walk_length=8, rng=rng, n_processes=nproc)
    print(f"{rng:9s} n_processes={nproc:3d}: {time.perf_counter() - t:.3f} s per call, nnz(K) = {K.nnz}", flush=True)
