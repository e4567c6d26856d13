"""Column tiers of a real graph's Phi (a mid-degree-column tier for Enron / Facebook).

The whole-K symmetric sparse Gram visits, for every row i and every nonzero k of Phi[i], the buckets
(band, k) of the bands at or after band(i): column k costs c_k slot visits per band pass and about
c_k^2 / 2 gathered records (c_k = column k's entries).  The hub panel (bench --hubs auto) takes the
columns with c_k >= 0.13 N to an MFMA panel of N^2 / 2 multiply-adds each.  This prints, per tier of
columns ranked by c_k, the share of records and visits and what the tier would cost as an MFMA panel
(N^2 / 2 multiply-adds per column at the fp32 MFMA peak) or as a row-compressed panel (only the rows
holding a tier column: |R|^2 / 2 multiply-adds per column, plus a read-modify-write of those |R|^2 K
entries).  Phi from the C oracle (Philox stream, the bench's seed), CPU only.
usage: python tools/hub_tiers.py enron|facebook [--walks 128] [--length 8]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd"))
from grf_amd.graphs import snap_graph  # noqa: E402
from oracle import oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("graph")
ap.add_argument("--walks", type=int, default=128)
ap.add_argument("--length", type=int, default=8)
ap.add_argument("--p-halt", type=float, default=0.1)
args = ap.parse_args()
A = snap_graph(args.graph)
n = A.shape[0]
Ls, _ = O.laplacian_sparse(A)
ip, ix, dx = O._csr_arrays(Ls)
node, load = O.walk_slots(ip, ix, dx, args.walks, args.p_halt, args.length, rng=O.RNG_PHILOX, seed=42, begin=0, end=n)
f = [1.0]
for l in range(1, args.length):
    f.append(f[-1] * (-1.0) / (2.0 * l))
phi = O.phi_sparse(O.reduce_steps(node, np.where(node >= 0, load, 0.0), 1), f)
c = np.bincount(phi.indices, minlength=n).astype(np.float64)
order = np.argsort(-c)
cs = c[order]
rec = cs * cs / 2.0
tot_rec, tot_vis = rec.sum(), cs.sum()
peak = 157.3e12
rows_of = phi.tocsc()
out = {"graph": args.graph, "n": n, "nnz_phi": int(phi.nnz), "records_total": tot_rec, "tiers": []}
edges = [0, 16, 32, 64, 96, 128, 256, 512, 1024, 2048, 4096]
for a, b in zip(edges[:-1], edges[1:]):
    cols = order[a:b]
    R = np.unique(rows_of[:, cols].indices) if len(cols) else np.array([], np.int64)
    panel_ms = (b - a) * n * n / 2 * 2 / peak * 1e3
    comp_ms = (b - a) * len(R) ** 2 / 2 * 2 / peak * 1e3
    out["tiers"].append({"cols": [a, b], "c_range": [float(cs[b - 1]), float(cs[a])],
                         "c_over_n": [float(cs[b - 1]) / n, float(cs[a]) / n],
                         "record_share": float(rec[a:b].sum() / tot_rec), "visit_share": float(cs[a:b].sum() / tot_vis),
                         "rows_touched": int(len(R)), "panel_ms_at_peak": panel_ms,
                         "compressed_panel_ms_at_peak": comp_ms,
                         "compressed_rmw_gb": 2 * 4 * len(R) ** 2 / 2 / 1e9})
print(json.dumps(out))
for t in out["tiers"]:
    print(f"cols {t['cols'][0]:5d}-{t['cols'][1]:5d}  c/N {t['c_over_n'][0]:.3f}-{t['c_over_n'][1]:.3f}  "
          f"records {t['record_share']:.3f}  visits {t['visit_share']:.4f}  rows {t['rows_touched']:6d}  "
          f"panel {t['panel_ms_at_peak']:.3f} ms  compressed {t['compressed_panel_ms_at_peak']:.3f} ms "
          f"+ RMW {t['compressed_rmw_gb']:.2f} GB")
