"""Time the staged transpose fill of an alternative library build (timing experiments only)."""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "efficient-gaussian-process-on-graphs_amd")]
import torch  # noqa: E402
from grf_amd import _lib  # noqa: E402
if len(sys.argv) > 1:
    _lib.LIB_PATH = os.path.abspath(sys.argv[1])
import bench  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402

eng = GRFEngine("cuda:0")
n = 100_000
G = eng.laplacian(DeviceCSR.from_scipy(bench.er_graph_exact_edges(n, 1_000_000, 0), eng.device))
phi = eng.compact(eng.walk_phi(G, 128, 0.1, 8, bench.diffusion_modulator(8), seed=42), want64=False)
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    eng.transpose_banded(phi)
    e1.record()
    e1.synchronize()
    ts.append(e0.elapsed_time(e1))
print(json.dumps({"lib": sys.argv[1] if len(sys.argv) > 1 else "default", "ms": [round(t, 3) for t in ts[1:]]}))
