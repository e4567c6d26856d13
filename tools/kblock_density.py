"""Density of the C5 K block (bench.py --workload c5: N = 1M Chung-Lu power-law, m = 64, the column
block K[:, 0:8192]): the share of nonzero entries and of 128-byte lines (32 floats of a row) holding
any nonzero -- what a write-out that skips all-zero lines (a zeroed buffer + line-sparse stores) could
save.  Prints one JSON line.  usage: python tools/kblock_density.py [n] [k_rows]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator  # noqa: E402
from grf_amd import pipeline as P  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import powerlaw_graph  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
kr = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
eng = GRFEngine("cuda:0")
A = powerlaw_graph(n, 10.0, 2.5, seed=0)
A_dev = DeviceCSR.from_scipy(A, eng.device)
pl = P.plan_step(n, 64, 8, 0.1, diffusion_modulator(8), seed=42, k_rows=kr)
K = P.alloc_k(eng, pl)
fr = P.front(eng, A_dev, pl)
P.k_assembly(eng, fr, pl, K)
torch.cuda.synchronize()
blk = K[:, :kr]
nz = 0
lines_nz = 0
for r0 in range(0, n, 65536):
    x = blk[r0:r0 + 65536] != 0
    nz += int(x.sum())
    lines_nz += int(x.view(x.shape[0], kr // 32, 32).any(dim=2).sum())
out = {"n": n, "k_rows": kr, "entries": n * kr, "nonzero_share": nz / (n * kr),
       "lines": n * kr // 32, "nonzero_line_share": lines_nz / (n * kr // 32)}
print(json.dumps(out), flush=True)
