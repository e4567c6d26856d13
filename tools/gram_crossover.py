"""Dense (MFMA) vs sparse (banded transpose + symmetric Gustavson Gram) K = Phi Phi^T by graph size:
the crossover that sets engine.DENSE_GRAM_MAX_N (gram(method="auto")).  ER graphs of mean degree 10,
m = 128, L = 8, p = 0.1 (C2's shape); one JSON line per n with the HIP-event ms of each path (each
path from Phi to K, the same K tolerance)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator, er_graph_exact_edges  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402

eng = GRFEngine("cuda:0")
sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [2000, 4000, 6000, 8000, 10000, 12000,
                                                                                  16000, 20000]
reps = 5


def timed(fn):
    fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


for n in sizes:
    A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 5 * n, 0), eng.device)
    G = eng.laplacian(A)
    phi = eng.compact(eng.walk_phi(G, 128, 0.1, 8, diffusion_modulator(8), seed=42, want64=False), want64=False)
    dense_ms = timed(lambda: eng.gram(phi, "dense"))
    sparse_ms = timed(lambda: eng.gram(phi, "sparse"))
    print(json.dumps({"n": n, "nnz_phi": phi.nnz, "dense_ms": round(dense_ms, 4), "sparse_ms": round(sparse_ms, 4),
                      "faster": "dense" if dense_ms < sparse_ms else "sparse"}), flush=True)
