"""Share of the row-stationary Gram's gathered records that the h densest Phi columns account for
(C5 column block, C4, Enron): records = sum_k c_k * c_k^block, c_k = nnz of Phi column k."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "efficient-gaussian-process-on-graphs_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from grf_amd.dist import setup_phi
from grf_amd.engine import DeviceCSR, GRFEngine
from grf_amd.graphs import powerlaw_graph
import bench

eng = GRFEngine("cuda:0")
def share(name, A, m, L, blk):
    f = bench.diffusion_modulator(L, 1.0)
    phi = setup_phi(eng, DeviceCSR.from_scipy(A, eng.device), m, 0.1, L, f, seed=42)
    n = A.shape[0]
    idx = phi.idx[:phi.nnz].long()
    c = torch.bincount(idx, minlength=n).double()
    e_blk = int(phi.ptr[blk])
    cb = torch.bincount(idx[:e_blk], minlength=n).double()
    rec = c * cb
    tot = rec.sum().item()
    order = torch.argsort(rec, descending=True)
    cs = torch.cumsum(rec[order], 0) / tot
    out = [f"{name}: n={n} nnz(Phi)={phi.nnz} block rows={blk} records={tot:.3e}"]
    for h in (16, 64, 256, 1024):
        k = order[:h]
        dense_mac = n * blk * h
        out.append(f"  top {h:5d} columns: {cs[h-1].item():.3f} of the records (c_k of the {h}th: {c[order[h-1]].item():.0f}); "
                   f"dense MACs {dense_mac:.2e} vs their sparse records {rec[k].sum().item():.2e}")
    print("\n".join(out), flush=True)

from grf_amd.graphs import er_graph_exact_edges, snap_graph
share("C5 power-law N=1M m=64 (block = first 8192 rows)", powerlaw_graph(1_000_000, 10.0, 2.5, seed=0), 64, 8, 8192)
share("Enron m=128 (whole K)", snap_graph("enron"), 128, 8, 36692)
share("Facebook m=128 (whole K)", snap_graph("facebook"), 128, 8, 22470)
share("C4 ER N=100k m=128 (whole K)", er_graph_exact_edges(100_000, 1_000_000, seed=0), 128, 8, 100_000)
