"""Error of the dense Gram against fp64, fp32 MFMA path vs the bf16 three-plane split path (grf_gram_dense_split).

Operands: C3's dense Phi (Cora through the bench's dense front), the C2-dense size (n = k = 10 000, Phi-like
random entries, sampled rows) and a signed operand.  Error of an entry = |K - K64| / (|Phi| |Phi|^T)_ij (the
scale the parity tests bound); printed: max and rms over the entries, and the ratio split / fp32.
usage (GPU): python3 tools/split_gram_error.py > profiles/r05_split_gram_error.txt
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd"))

from grf_amd import _lib as C  # noqa: E402
from grf_amd.engine import GRFEngine  # noqa: E402


def errors(eng, A, k, rows=None):
    P = A[:, :k].double()
    Pr = P if rows is None else P[rows]
    ref = Pr @ P.t()
    scale = Pr.abs() @ P.abs().t() + 1e-300
    out = {}
    for prec in ("fp32", "split"):
        K = eng.gram_dense(A, k, precision=prec)
        Kr = (K if rows is None else K[rows]).double()
        e = ((Kr - ref).abs() / scale)
        out[prec] = (float(e.max()), float(e.pow(2).mean().sqrt()))
        del K
    return out


def main():
    eng = GRFEngine("cuda:0")
    cases = []
    from bench import cora_adjacency, diffusion_modulator
    W = cora_adjacency()
    n = W.shape[0]
    G = eng.walk_matrix_dense(torch.from_numpy(W).to(eng.device), C.LAP_NUMPY)
    dense = eng.densify_padded(eng.walk_phi(G, 128, 0.1, 8, diffusion_modulator(8, 1.0), seed=42, norm=C.NORM_DIV,
                                            want64=False))
    cases.append(("C3 Cora dense Phi (n = k = 2708)", dense, n, None))
    g = torch.Generator(device=eng.device).manual_seed(1)
    for nn, signed in ((10000, False), (4096, True)):
        lda = -(-nn // 64) * 64
        A = torch.zeros((nn, lda), dtype=torch.float32, device=eng.device)
        v = torch.rand((nn, nn), device=eng.device, generator=g) * 10.0 ** (
            torch.rand((nn, nn), device=eng.device, generator=g) * 4 - 3)
        v *= torch.rand((nn, nn), device=eng.device, generator=g) < 0.05
        if signed:
            v *= torch.sign(torch.randn((nn, nn), device=eng.device, generator=g))
        A[:, :nn] = v
        rows = torch.arange(0, nn, 37, device=eng.device)
        cases.append((f"{'signed' if signed else 'Phi-like'} random n = k = {nn} (4 decades, 5 % dense; every 37th row)",
                      A, nn, rows))
    print("# dense Gram error against fp64: |K - K64| / (|Phi| |Phi|^T), fp32 MFMA vs bf16 three-plane split")
    for name, A, k, rows in cases:
        e = errors(eng, A, k, rows)
        f, s = e["fp32"], e["split"]
        print(f"{name}\n    fp32  max {f[0]:.3e}  rms {f[1]:.3e}\n    split max {s[0]:.3e}  rms {s[1]:.3e}"
              f"   (split / fp32: max {s[0] / max(f[0], 1e-300):.2f}, rms {s[1] / max(f[1], 1e-300):.2f})", flush=True)


if __name__ == "__main__":
    main()
