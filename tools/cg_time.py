"""Time the pathwise-conditioning stages at C4 scale (N=100k, m=128, L=8; 60/20 split, S=64)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator, er_graph_exact_edges  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402

S = int(os.environ.get("S", "64"))
dt = torch.float64 if os.environ.get("DT", "f64") == "f64" else torch.float32
eng = GRFEngine("cuda:0")
n = 100_000
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, 0), eng.device)
G = eng.laplacian(A)
phi = eng.compact(eng.walk_phi(G, 128, 0.1, 8, diffusion_modulator(8), seed=42), want64=False)
r = np.random.default_rng(0)
perm = torch.from_numpy(r.permutation(n))
tr, te = perm[:60000].cuda(), perm[60000:80000].cuda()
y = torch.randn(60000, device="cuda")
e1 = torch.randn(S, n, device="cuda")
e2 = 0.1 * torch.randn(S, 60000, device="cuda")


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


ms, pt = timed(lambda: eng.csr_transpose(phi, tr))
print(f"nnz(phi)={phi.nnz} nnz(phi_tr)={pt.nnz}  csr_transpose {ms:.2f} ms", flush=True)
P = torch.randn(60000, S, device="cuda", dtype=dt)
W = torch.randn(n, S, device="cuda", dtype=dt)
ms1, _ = timed(lambda: eng.spmm(pt, P))
ms2, _ = timed(lambda: eng.spmm(phi, W, tr))
gb = pt.nnz * (8 + S * P.element_size()) / 1e9
print(f"spmm Phi_tr^T P {ms1:.3f} ms, Phi_tr W {ms2:.3f} ms; gather {gb:.2f} GB each -> "
      f"{gb / ms1:.2f} / {gb / ms2:.2f} TB/s", flush=True)
B = torch.randn(60000, S, device="cuda", dtype=dt)
for mi in (11, 50):
    ms, (X, it) = timed(lambda: eng.cg_solve(phi, B, 0.1, tr, pt, max_iter=mi, tolerance=0.0), reps=3)
    print(f"cg max_iter={mi}: {ms:.2f} ms ({it} its, {ms / it:.3f} ms/it)", flush=True)
ms, (out, it) = timed(lambda: eng.pathwise_predict(phi, tr, te, y, 0.1, e1, e2, dtype=dt), reps=3)
print(f"pathwise_predict S={S}: {ms:.2f} ms, {it} CG iterations", flush=True)
