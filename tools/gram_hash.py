"""Bit-level fingerprints of K from the bench's own K assembly (grf_amd.pipeline) for a few shapes, so
that two library builds or two knob settings (e.g. GRF_GRAM_PERSIST=0 / 1) can be compared run against
run: identical lines = identical K bits.  Shapes: C4 (whole symmetric K), an odd-n ER graph (ragged last
band, n % 4 != 0), a power-law graph's symmetric K and its 8192-row column block in the slot layout
(the C5 path at 200k nodes), and the row mode.  usage: gram_hash.py  (one JSON line per shape)"""
import json
import math
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from grf_amd import pipeline as P  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import er_graph_exact_edges, powerlaw_graph  # noqa: E402


def fingerprint(Kv):
    """(xor-free) position-weighted int64 sums of K's bit patterns over row chunks, and an fp64 sum."""
    h, s = 0, 0.0
    w = None
    for r0 in range(0, Kv.shape[0], 4096):
        blk = Kv[r0:r0 + 4096].contiguous()
        bits = blk.view(torch.int32).to(torch.int64)
        if w is None or w.shape[0] != bits.shape[1]:
            w = (torch.arange(bits.shape[1], device=bits.device, dtype=torch.int64) * 2654435761) % 1000003 + 1
        rows = torch.arange(r0, r0 + bits.shape[0], device=bits.device, dtype=torch.int64)[:, None] % 997 + 1
        h = (h * 1000003 + int((bits * w * rows).sum())) % (1 << 61)
        s += float(blk.double().sum())
    return h, s


def diffusion(L):
    return np.array([(-1.0) ** l / (2.0 ** l * math.factorial(l)) for l in range(L)])


def main():
    eng = GRFEngine("cuda:0")
    cases = [
        ("c4", er_graph_exact_edges(100_000, 1_000_000, 0), 128, 8, {}),
        ("er_odd", er_graph_exact_edges(30_001, 200_000, 3), 32, 6, {}),
        ("powerlaw_sym", powerlaw_graph(60_000, 10.0, 2.5, seed=1), 32, 8, {}),
        ("powerlaw_c5_block", powerlaw_graph(200_000, 10.0, 2.5, seed=2), 64, 8, {"k_rows": 8192}),
        ("er_rows", er_graph_exact_edges(30_001, 200_000, 3), 32, 6, {"no_sym": True}),
    ]
    for name, A, m, L, kw in cases:
        n = A.shape[0]
        pl = P.plan_step(n, m, L, 0.1, diffusion(L), **kw)
        K, fr = P.kernel_step(eng, DeviceCSR.from_scipy(A, eng.device), pl)
        torch.cuda.synchronize()
        h, s = fingerprint(P.k_view(K, pl))
        print(json.dumps({"case": name, "mode": pl.mode, "rec_unit": int(fr.tr.rec_unit), "n": n,
                          "hash": h, "sum": s}), flush=True)
        del K, fr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
