"""Time grf_walk_phi of an alternative build of the library (timing experiments only)."""
import json, os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'efficient-gaussian-process-on-graphs_amd'))
import torch
from grf_amd import _lib
_lib.LIB_PATH = os.path.abspath(sys.argv[1])
import bench
from grf_amd.engine import GRFEngine
eng = GRFEngine('cuda:0')
n = 100000
A = bench.er_graph_exact_edges(n, n * 10, 0)
G = eng.laplacian(A)
f = bench.diffusion_modulator(8)
ts = []
for _ in range(4):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); eng.walk_phi(G, 128, 0.1, 8, f, seed=42); e1.record(); e1.synchronize()
    ts.append(e0.elapsed_time(e1))
print(json.dumps({"lib": sys.argv[1], "ms": ts[1:]}))
