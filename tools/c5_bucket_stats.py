"""C5 column-block Gram lookups: the share finding an empty slot and the bucket entries per row (K block = Phi rows 0..8191).
-> profiles/r06_c5_bucket_stats.json (usage: python tools/c5_bucket_stats.py)"""
import os, sys, json
import torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
import bench
from grf_amd import pipeline as P
from grf_amd.engine import DeviceCSR, GRFEngine
from grf_amd.graphs import powerlaw_graph
eng = GRFEngine("cuda:0")
n, m, L, p = 1_000_000, 64, 8, 0.1
f = bench.diffusion_modulator(L, 1.0)
A = DeviceCSR.from_scipy(powerlaw_graph(n, 10.0, 2.5, seed=0), eng.device)
pl = P.plan_step(n, m, L, p, f, k_rows=8192)
fr = P.front(eng, A, pl)
phi = P.phi_csr(fr.phi)
ptr, idx = phi.ptr.long(), phi.idx.long()
blk = idx[: int(ptr[8192].item())]
cnt = torch.bincount(blk, minlength=n)
per = cnt[idx]                       # the bucket size each lookup finds
lookups = idx.numel()
empty = int((per == 0).sum().item())
inl = torch.clamp(per, max=4)        # entries in the slot's inline pairs (2 pairs = 4 entries)
out = {"lookups": lookups, "empty_frac": empty / lookups, "entries": int(per.sum().item()),
       "entries_per_row": float(per.sum().item()) / n, "lookups_gt4_frac": float((per > 4).float().mean().item()),
       "nonempty_buckets": int((cnt > 0).sum().item())}
print(json.dumps(out), flush=True)
