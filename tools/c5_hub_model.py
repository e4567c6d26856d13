"""Byte / flop model of a hub-column panel for the C5 column block, from the real Phi.

C5: N = 1M Chung-Lu power-law graph, m = 64, L = 8, block K[:, 0:8192].  The sparse Gram tile of row i
(1 x 8192 int64 accumulators) visits every nonzero k of Phi[i] and gathers the bucket (band, k) = the
entries of column k among the block's rows.  So column k costs c_k slot visits (c_k = its entries in all
of Phi) and c_k * b_k gathered records (b_k = its entries among the block's rows).  A panel of the H
columns with the most records would take those records out of the sparse tiles, at the price of an MFMA
product 2 * N * 8192 * H flops plus a way to add it into the fixed-point tile (the tiles write fp32 K
once; a separate panel pass costs the 32 GB block written and read back, the round-3 measurement).
Prints, for H in a sweep, the share of records and slot visits the panel removes and the panel's costs.
usage (GPU box): python tools/c5_hub_model.py [--n 1000000] [--rows 8192]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd"))
sys.path.insert(0, ROOT)
from grf_amd.dist import setup_phi  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import powerlaw_graph  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--rows", type=int, default=8192)
args = ap.parse_args()
eng = GRFEngine("cuda:0")
A = powerlaw_graph(args.n, 10.0, 2.5, seed=0)
L, m, p = 8, 64, 0.1
f = [1.0]
for l in range(1, L):
    f.append(f[-1] * (-1.0) / (2.0 * l))  # diffusion modulator, beta = 1 (bench.diffusion_modulator)
phi = setup_phi(eng, DeviceCSR.from_scipy(A, eng.device), m, p, L, f, seed=42)
n = args.n
nnz = int(phi.ptr[-1])
idx = phi.idx[:nnz].long()
c = torch.bincount(idx, minlength=n).double()
b = torch.bincount(idx[:int(phi.ptr[args.rows])], minlength=n).double()
rec = c * b
order = torch.argsort(rec, descending=True)
rec_s, c_s = rec[order], c[order]
tot_rec, tot_vis = float(rec.sum()), float(c.sum())
peak_tf = 157.3
out = {"n": n, "block_rows": args.rows, "nnz_phi": nnz, "records_total": tot_rec, "slot_visits_total": tot_vis,
       "mean_bucket": tot_rec / tot_vis, "max_c": float(c.max()), "rows": []}
for H in [0, 1, 4, 16, 64, 256, 1024, 4096]:
    r = float(rec_s[:H].sum()) if H else 0.0
    v = float(c_s[:H].sum()) if H else 0.0
    out["rows"].append({"H": H, "record_share": r / tot_rec, "visit_share": v / tot_vis,
                        "min_c_in_panel": float(c_s[H - 1]) if H else None,
                        "panel_tflop": 2.0 * n * args.rows * H / 1e12,
                        "panel_ms_at_peak": 2.0 * n * args.rows * H / (peak_tf * 1e12) * 1e3})
print(json.dumps(out))
for row in out["rows"]:
    print(f"H={row['H']:5d} records {row['record_share']:.4f} visits {row['visit_share']:.5f} "
          f"min c {row['min_c_in_panel']} panel {row['panel_ms_at_peak']:.2f} ms at the fp32 MFMA peak")
