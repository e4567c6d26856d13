"""C4 K assembly timing: symmetric Gram tiles + mirror, the mirror alone, the full (row-mode) Gram.
Prints one JSON line with the HIP-event times (ms, mean of reps) and a checksum of K (knob A/B runs
must agree bit for bit: the Gram's fixed-point sum is order independent)."""
import hashlib
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator, er_graph_exact_edges  # noqa: E402
from grf_amd.engine import DEFAULT_BAND_WIDTH, DeviceCSR, GRFEngine  # noqa: E402

eng = GRFEngine("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["sym", "mirror", "rows"]
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 10 * n, 0), eng.device)
G = eng.laplacian(A)
bw = int(os.environ.get("GRF_BW", DEFAULT_BAND_WIDTH))
phi = eng.compact(eng.walk_phi(G, 128, 0.1, 8, diffusion_modulator(8), seed=42), want64=False, sync_free=True)
ru = int(os.environ["GRF_REC_UNIT"]) if "GRF_REC_UNIT" in os.environ else None
# the bench's transpose (self-counting, sub-band split for the symmetric diagonal tiles)
tr = eng.transpose_banded(phi, bw, nnz_bound=phi.nnz_bound, rec_unit=ru, split=os.environ.get("GRF_SPLIT", "0") == "1")
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
out = {"n": n, "bw": bw, "rec_unit": tr.rec_unit, "t_rec_MB": tr.t_rec.numel() / 1e6,
       "split": os.environ.get("GRF_GRAM_SPLIT", "1")}


def timed(fn):
    fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def digest():
    h = hashlib.sha256()
    h.update(K[:, :n].contiguous().cpu().numpy().tobytes())
    return h.hexdigest()[:16]


for mode in modes:
    if mode == "sym":
        out["sym_ms"] = timed(lambda: eng.gram_sparse_sym(phi, tr, out=K))
        out["sym_digest"] = digest()
    elif mode == "upper":  # the Gram tiles alone (the mirror's input)
        out["upper_ms"] = timed(lambda: eng.gram_sparse_upper(phi, tr, K))
    elif mode == "mirror":
        out["mirror_ms"] = timed(lambda: eng.gram_mirror(K, n))
    elif mode == "rows":
        out["rows_ms"] = timed(lambda: eng.gram_sparse(phi, tr, out=K))
        out["rows_digest"] = digest()
print(json.dumps(out), flush=True)
