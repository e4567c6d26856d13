"""Time the fused walk -> Phi kernel (with bucket counting) on C4 or C5; prints JSON."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import er_graph_exact_edges, powerlaw_graph  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
eng = GRFEngine("cuda:0")
if cfg == "c4":
    n, m, bw = 100_000, 128, 4096
    A = er_graph_exact_edges(n, 1_000_000, 0)
else:
    n, m, bw = 1_000_000, 64, 8192
    A = powerlaw_graph(n, 10.0, 2.5, 0)
G = eng.laplacian(DeviceCSR.from_scipy(A, eng.device))
f = diffusion_modulator(8)
tws = eng.transpose_workspace(n, n, bw)


modes = sys.argv[2].split(",") if len(sys.argv) > 2 else ["count"]
fns = {
    "count": lambda: eng.walk_phi(G, m, 0.1, 8, f, seed=42, count_ws=tws, band_width=bw),  # (the bench's call)
    "nocount": lambda: eng.walk_phi(G, m, 0.1, 8, f, seed=42),
    "noaug": lambda: eng.walk_phi(G, m, 0.1, 8, f, seed=42, count_ws=tws, band_width=bw, use_aug=False),
    "walk": lambda: eng.walk(G, m, 0.1, 8, rng=1, seed=42),  # slots only (no sort, no Phi)
}
out = {"cfg": cfg}
for mode in modes:
    run = fns[mode]
    rows = run()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 5
    ev[0].record()
    for _ in range(reps):
        rows = run()
    ev[1].record()
    torch.cuda.synchronize()
    out[mode + "_ms"] = ev[0].elapsed_time(ev[1]) / reps
    if mode == "count":
        out["nnz"] = int(rows.cnt.sum().item())
        out["idx_sum"] = int(rows.idx.view(-1)[:1000].sum().item())
    print(json.dumps({mode: out[mode + "_ms"]}), flush=True)
print(json.dumps(out), flush=True)
