"""Pipelined C4 step timeline from HIP events (rocprofv3 serialises the two streams, events do not):
after the Gram tiles, the mirror on `main` and the next front (the bench's own stages, grf_amd.pipeline.front
in symmetric mode) on `side`; prints when each stage ends, relative to the tiles' end, next to the same
pieces run alone.  usage: overlap_events.py [mirror_wgs]   (one JSON line per configuration)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator  # noqa: E402
from grf_amd.engine import DEFAULT_BAND_WIDTH, DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import er_graph_exact_edges  # noqa: E402

wgs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
eng = GRFEngine("cuda:0")
n, m, L = 100_000, 128, 8
cap = min(m * L, n)
f = diffusion_modulator(L)
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, 0), eng.device)
bw = DEFAULT_BAND_WIDTH
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
STAGES = ("laplacian", "walk", "compact", "transpose")


def front(ev=None):
    def mark(k):
        if ev is not None:
            ev[k].record()
    G = eng.laplacian(A)
    mark("laplacian")
    rows = eng.walk_phi(G, m, 0.1, L, f, seed=42, want64=False)
    mark("walk")
    phi = eng.compact(rows, want64=False, want32=True, sync_free=True)
    mark("compact")
    tr = eng.transpose_banded(phi, bw, nnz_bound=n * cap)
    mark("transpose")
    return phi, tr


phi, tr = front()
out = {"mirror_wgs": wgs, "pipelined": []}
for rep in range(4):
    eng.gram_sparse_upper(phi, tr, K)
    t0 = E()
    t0.record(main)
    ev = {k: E() for k in STAGES}
    side.wait_event(t0)
    mirror_end = E()
    eng.gram_mirror(K, n, wgs)
    mirror_end.record(main)
    with torch.cuda.stream(side):
        front(ev)
    torch.cuda.synchronize()
    if rep:
        out["pipelined"].append({"mirror_end": round(t0.elapsed_time(mirror_end), 3),
                                 **{k: round(t0.elapsed_time(ev[k]), 3) for k in STAGES}})
# each alone
a, b = E(), E()
torch.cuda.synchronize()
a.record()
eng.gram_mirror(K, n, wgs)
b.record()
torch.cuda.synchronize()
out["mirror_alone"] = round(a.elapsed_time(b), 3)
for rep in range(3):
    a = E()
    ev = {k: E() for k in STAGES}
    a.record()
    front(ev)
    torch.cuda.synchronize()
    out["front_alone"] = {k: round(a.elapsed_time(ev[k]), 3) for k in STAGES}
print(json.dumps(out), flush=True)
