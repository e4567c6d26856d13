"""Dense MFMA Gram A/B harness: time grf_gram_dense_ws (HIP events, `reps` launches back to back) at
several n on random sparse-ish fp32 operands, check it against fp64 (|dK| <= 1e-5 (|A||A|^T)), exact
symmetry and run-to-run bit identity, and print one JSON line per n.  Knobs are the library's env
variables (GRF_DENSE_SK, GRF_DENSE_SPLIT, GRF_DENSE_TAIL), read once per process: run one process per arm.
usage: python tools/dense_ab.py [--label L] [--zeros-frac F] n [n ...]"""
import argparse
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd"))
from grf_amd.engine import GRFEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("n", type=int, nargs="*", default=[2708, 4096, 10000])
ap.add_argument("--label", default="")
ap.add_argument("--density", type=float, default=0.05)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--k", type=int, default=0, help="k_dim (default n)")
args = ap.parse_args()
eng = GRFEngine("cuda:0")
for n in args.n:
    k = args.k or n
    lda = -(-k // 64) * 64
    A = torch.zeros((n, lda), dtype=torch.float32, device=eng.device)
    g = torch.Generator(device=eng.device).manual_seed(n)
    A[:, :k] = torch.rand((n, k), device=eng.device, generator=g) * (
        torch.rand((n, k), device=eng.device, generator=g) < args.density)
    K = eng.gram_dense(A, k)
    torch.cuda.synchronize()
    d0 = hashlib.sha256(K.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]
    for _ in range(3):
        eng.gram_dense(A, k)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(args.reps):
        K = eng.gram_dense(A, k)
    ev[1].record()
    ev[1].synchronize()
    ms = ev[0].elapsed_time(ev[1]) / args.reps
    d1 = hashlib.sha256(K.contiguous().cpu().numpy().tobytes()).hexdigest()[:12]
    Ad = A[:, :k].double()
    ref = Ad @ Ad.t()
    bound = 1e-5 * (Ad.abs() @ Ad.abs().t()) + 1e-30
    ratio = float(((K.double() - ref).abs() / bound).max())
    sym = bool(torch.equal(K, K.t()))
    flops = n * (n + 1) * float(k)
    print(json.dumps({"label": args.label, "n": n, "k": k, "ms": round(ms, 4), "TFs": round(flops / ms / 1e9, 1),
                      "frac": round(flops / ms / 1e9 / 157.3, 3), "err_ratio": round(ratio, 4), "sym": sym,
                      "repeat_identical": d0 == d1, "digest": d1,
                      "env": {e: os.environ[e] for e in os.environ if e.startswith("GRF_DENSE")}}), flush=True)
    del A, K, Ad, ref, bound
    torch.cuda.empty_cache()
