import sys, os
R='/root/repo'; sys.path.insert(0,R); sys.path.insert(0, R+'/efficient-gaussian-process-on-graphs_amd'); sys.path.insert(0, R+'/tests')
import numpy as np, scipy.sparse as sp
from grf_amd.engine import GRFEngine
from oracle import oracle as O
from test_gpu_parity import er_graph
eng = GRFEngine('cuda:0')
A = er_graph(300, 6, 1)
G = eng.laplacian(A)
for m, L in [(16, 4), (128, 8), (32, 8)]:
    slots = eng.walk(G, m, 0.1, L, rng=1, seed=3)
    f = [(-0.5) ** l for l in range(L)]
    got = eng.compact(eng.phi_fused(slots, f)).to_scipy()
    node, load = slots.node.cpu().numpy(), slots.load.cpu().numpy()
    ref = O.phi_sparse(O.reduce_steps(node, np.where(node >= 0, load, 0.0), 1), f)
    d = (got != ref)
    print(m, L, 'nnz', got.nnz, ref.nnz, 'diff entries', d.nnz)
    if d.nnz:
        r, c = d.nonzero()
        for i in range(min(5, len(r))):
            print('  row', r[i], 'col', c[i], got[r[i], c[i]], ref[r[i], c[i]])
        print('  row0 got', got[r[0]].indices[:12], '\n  row0 ref', ref[r[0]].indices[:12])
