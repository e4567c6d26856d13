"""MFMA dense Gram throughput (grf_gram_dense incl. its mirror) at several n: N (N + 1) k flops over
HIP-event time, and a digest of K (knob A/Bs that keep the MFMA order must agree bit for bit).
usage: python tools/dense_sweep.py [n ...]  (GRF_DENSE_TILE / GRF_DENSE_BK / GRF_DENSE_DB knobs)."""
import hashlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd"))
from grf_amd.engine import GRFEngine  # noqa: E402

eng = GRFEngine("cuda:0")
for n in [int(a) for a in sys.argv[1:]] or [2708, 4096, 10000]:
    lda = -(-n // 64) * 64
    A = torch.zeros((n, lda), dtype=torch.float32, device=eng.device)
    g = torch.Generator(device=eng.device).manual_seed(n)
    A[:, :n] = torch.rand((n, n), device=eng.device, generator=g) * (torch.rand((n, n), device=eng.device, generator=g) < 0.05)
    for _ in range(3):
        eng.gram_dense(A, n)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record()
        K = eng.gram_dense(A, n)
        b.record()
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
    flops = n * (n + 1) * float(n)
    ref = (A[:, :n].double() @ A[:, :n].double().t())
    err = ((K.double() - ref).abs().max() / ref.abs().max()).item()
    print(f"n={n} tile={os.environ.get('GRF_DENSE_TILE', 'auto')} bk={os.environ.get('GRF_DENSE_BK', 'auto')} "
          f"db={os.environ.get('GRF_DENSE_DB', 'auto')} {ms:.4f} ms {flops / ms / 1e9:.1f} TF/s frac={flops / ms / 1e9 / 157.3:.3f} "
          f"relerr={err:.2e} digest={hashlib.sha256(K.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]}", flush=True)
