"""Gram-kernel sweep on the C4 workload: band widths, one process (interleaved rounds)."""
import sys, time, json
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'efficient-gaussian-process-on-graphs_amd'))
import numpy as np, torch
import bench
from grf_amd.engine import GRFEngine, DeviceCSR
from grf_amd import _lib as C
eng = GRFEngine('cuda:0')
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
A = bench.er_graph_exact_edges(n, n * 10, 0)
f = bench.diffusion_modulator(8)
G = eng.laplacian(A)
slots = eng.walk(G, 128, 0.1, 8, rng=C.RNG_PHILOX, seed=42)
phi = eng.compact(eng.features(slots, f), want64=False)
del slots
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
res = {}
bws = [int(x) for x in (sys.argv[2].split(',') if len(sys.argv) > 2 else ['4096', '8192', '16384'])]
trs = {bw: eng.transpose_banded(phi, bw) for bw in bws}
for rnd in range(3):
    for bw in bws:
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); eng.gram_sparse(phi, trs[bw], out=K); e1.record(); e1.synchronize()
        res.setdefault(bw, []).append(e0.elapsed_time(e1))
print(json.dumps({str(k): v for k, v in res.items()}))
