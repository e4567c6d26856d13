"""C4 Gram kernel: timing per band width + bitwise equality across band widths + oracle rows."""
import json, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, 'efficient-gaussian-process-on-graphs_amd'))
import numpy as np, torch
import bench
from grf_amd.engine import GRFEngine
from grf_amd import _lib as C
from oracle import oracle as O
eng = GRFEngine('cuda:0')
n = int(sys.argv[1]); bws = [int(x) for x in sys.argv[2].split(',')]
A = bench.er_graph_exact_edges(n, n * 10, 0)
G = eng.laplacian(A)
slots = eng.walk(G, 128, 0.1, 8, rng=C.RNG_PHILOX, seed=42)
phi = eng.compact(eng.features(slots, bench.diffusion_modulator(8)), want64=False)
del slots
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
rows = np.r_[0:8, n // 2:n // 2 + 8, n - 8:n]
ps = phi.to_scipy().astype(np.float64).tocsr()
ref = np.concatenate([O.gram_rows(ps, int(a), int(a) + 8) for a in (0, n // 2, n - 8)])
base = None
out = {}
for bw in bws:
    tr = eng.transpose_banded(phi, bw)
    K.zero_()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); eng.gram_sparse(phi, tr, out=K); e1.record(); e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    Ks = K[torch.from_numpy(rows).to(eng.device), :n].cpu().numpy()
    err = float(np.abs(Ks - ref).max() / np.abs(ref).max())
    h = K[:, :n].sum(dim=1, dtype=torch.float64).cpu().numpy()
    same = None if base is None else bool(np.array_equal(h, base))
    if base is None: base = h
    out[bw] = {"ms": ts, "rel_err_rows": err, "rowsum_equal_first": same}
    print(bw, out[bw], flush=True)
    del tr
print(json.dumps(out))
