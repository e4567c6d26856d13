"""GPU CG vs the oracle, iteration by iteration (max_iter = 1..N): where do they part?"""
import sys
import numpy as np
import torch
sys.path[:0] = ["tests", ".", "efficient-gaussian-process-on-graphs_amd"]
from test_gpu_cg import _graph, _phi32, _system  # noqa: E402
from oracle import cg as OCG  # noqa: E402
from grf_amd.engine import GRFEngine  # noqa: E402

eng = GRFEngine("cuda:0")
A = _graph(3000, 8, 5)
G = eng.laplacian(A)
phi = eng.compact(eng.walk_phi(G, 16, 0.2, 4, [1.0, -0.5, 0.25, -0.125], seed=3))
for S, seed, noise in [(64, 64, 0.1), (5, 5, 0.1), (64, 7, 2.0)]:
    P, tr, B, mm = _system(phi, 1800, S, seed, noise)
    Bd = B.astype(np.float64)
    for mi in list(range(1, 13)) + [16, 20, 30]:
        X, it = eng.cg_solve(phi, torch.from_numpy(Bd).cuda(), noise, torch.from_numpy(tr), max_iter=mi)
        Xo, ito = OCG.linear_cg(mm, Bd, max_iter=mi)
        X = X.cpu().numpy()
        print(f"S={S} noise={noise} max_iter={mi}: it {it} vs {ito}  rel {np.linalg.norm(X - Xo) / np.linalg.norm(Xo):.3e}",
              flush=True)
