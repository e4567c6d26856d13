"""Timing experiment (C3 / C2 dense path): one whole serial step (dense Laplacian -> walks -> dense Phi -> split
Gram) captured in a HIP graph and replayed, against the same step launched eagerly.  Prints one JSON line
with both ms per step and whether the replayed K equals the eager K bit for bit.
usage: python tools/dense_graph_exp.py [c3|c2] [steps]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import dense_workload, diffusion_modulator  # noqa: E402
from grf_amd import _lib as C  # noqa: E402
from grf_amd.engine import GRFEngine  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c3"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
eng = GRFEngine("cuda:0")
W, _, _ = dense_workload(wl)
n, m, L, p = W.shape[0], 128, 8, 0.1
f = diffusion_modulator(L, 1.0)
Wt = torch.from_numpy(W).to(eng.device)
s = torch.cuda.Stream(eng.device)


def step():
    G = eng.walk_matrix_dense(Wt, C.LAP_NUMPY)
    dense = eng.densify_padded(eng.walk_phi(G, m, p, L, f, seed=42, norm=C.NORM_DIV, want64=False))
    return eng.gram_dense(dense, n)


def timed(fn, k):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(k):
        fn()
    ev[1].record()
    ev[1].synchronize()
    return ev[0].elapsed_time(ev[1]) / k


with torch.cuda.stream(s):
    for _ in range(3):
        K_eager = step()
    torch.cuda.synchronize()
    eager_ms = timed(step, steps)
    K_eager = step().clone()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        K_graph = step()
    g.replay()
    torch.cuda.synchronize()
    same = bool(torch.equal(K_graph, K_eager))
    graph_ms = timed(g.replay, steps)
print(json.dumps({"workload": wl, "eager_ms": eager_ms, "graph_ms": graph_ms, "bits_equal": same}), flush=True)
