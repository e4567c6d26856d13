"""Run the Gram kernel alone on the C4 workload (for rocprofv3 PMC passes)."""
import sys
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'efficient-gaussian-process-on-graphs_amd'))
import torch
import bench
from grf_amd.engine import GRFEngine
from grf_amd import _lib as C
eng = GRFEngine('cuda:0')
n = int(sys.argv[1]); bw = int(sys.argv[2]); reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
A = bench.er_graph_exact_edges(n, n * 10, 0)
G = eng.laplacian(A)
slots = eng.walk(G, 128, 0.1, 8, rng=C.RNG_PHILOX, seed=42)
phi = eng.compact(eng.features(slots, bench.diffusion_modulator(8)), want64=False)
del slots
tr = eng.transpose_banded(phi, bw)
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
for _ in range(reps):
    eng.gram_sparse(phi, tr, out=K)
torch.cuda.synchronize()
print("nnz", phi.nnz)
