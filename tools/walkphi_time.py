"""C4: time walk (slots) vs phi_fused (from slots) vs fused walk_phi."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator, er_graph_exact_edges  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402

eng = GRFEngine("cuda:0")
n = 100_000
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, 0), eng.device)
G = eng.laplacian(A)
f = diffusion_modulator(8)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


ms_w, slots = timed(lambda: eng.walk(G, 128, 0.1, 8, seed=42))
ms_p, _ = timed(lambda: eng.phi_fused(slots, f))
ms_f, _ = timed(lambda: eng.walk_phi(G, 128, 0.1, 8, f, seed=42))
print(f"walk {ms_w:.2f} ms, phi_fused(slots) {ms_p:.2f} ms, walk_phi {ms_f:.2f} ms")
