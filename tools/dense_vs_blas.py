"""The dense MFMA Gram (grf_gram_dense: tiles on and above the diagonal + split-K combine / mirror) against
the vendor library's fp32 GEMM of the same product (torch.matmul -> hipBLASLt / rocBLAS, A A^T in full, and
torch's fp32 SYRK-free path), HIP events, same operands; the max |difference| between the two K's is printed.
usage: python tools/dense_vs_blas.py [n ...]  (one JSON line per n)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd"))
from grf_amd.engine import GRFEngine  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
eng = GRFEngine("cuda:0")


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    out = None
    for a, b in ev:
        a.record()
        out = fn()
        b.record()
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in ev) / reps, out


for n in [int(a) for a in sys.argv[1:]] or [2708, 4096, 10000]:
    lda = -(-n // 64) * 64
    A = torch.zeros((n, lda), dtype=torch.float32, device=eng.device)
    g = torch.Generator(device=eng.device).manual_seed(n)
    A[:, :n] = torch.rand((n, n), device=eng.device, generator=g) * (torch.rand((n, n), device=eng.device, generator=g) < 0.05)
    An = A[:, :n].contiguous()
    ms_ours, K = timed(lambda: eng.gram_dense(A, n))
    ms_blas, Kb = timed(lambda: torch.matmul(An, An.t()))
    unique = n * (n + 1) * float(n)  # the unique entries' flops (what the MFMA Gram computes)
    full = 2.0 * n * n * float(n)
    print(json.dumps({"n": n, "ours_ms": round(ms_ours, 4), "blas_ms": round(ms_blas, 4),
                      "ours_TFs_unique": round(unique / ms_ours / 1e9, 1), "blas_TFs_full": round(full / ms_blas / 1e9, 1),
                      "max_abs_diff": float((K[:, :n] - Kb).abs().max())}), flush=True)
