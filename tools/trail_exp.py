"""C4 K assembly with a trailing mirror (pipeline.k_assembly_trailing) against tiles + one mirror pass
(the bench's K assembly), HIP events on one box, both interleaved; the trailing K is compared with the
reference K bit for bit.  usage: trail_exp.py [chunk_rows,... [mirror_wgs,... [tile_streams,...]]]  (JSON lines;
tile_streams: streams the tile chunks are dealt to, 1 = the caller's alone)"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator  # noqa: E402
from grf_amd import pipeline as P  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import er_graph_exact_edges  # noqa: E402

chunks = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [4096, 8192, 16384]
wgs_list = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
ts_list = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1]
eng = GRFEngine("cuda:0")
n, m, L = 100_000, 128, 8
pl = P.plan_step(n, m, L, 0.1, diffusion_modulator(L))
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, 0), eng.device)
fr = P.front(eng, A, pl)
K = P.alloc_k(eng, pl)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
extra = [torch.cuda.Stream() for _ in range(3)]
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731


def base():
    s, t, e = E(), E(), E()
    s.record()
    eng.gram_sparse_upper(fr.phi, fr.tr, out=K, cuts=getattr(fr, "cuts", None))
    t.record()
    eng.gram_mirror(K, n, 0)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(t), t.elapsed_time(e), s.elapsed_time(e)


def trail(c, w, ts):
    s, e = E(), E()
    s.record()
    P.k_assembly_trailing(eng, fr, pl, K, side, chunk_rows=c, mirror_workgroups=w, tile_streams=extra[:ts - 1])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e)


base()
torch.cuda.synchronize()
Kref = K.clone()
for c, w, ts in [(c, w, ts) for c in chunks for w in wgs_list for ts in ts_list]:
        K.fill_(float("nan"))
        trail(c, w, ts)
        same = bool(torch.equal(K[:, :n], Kref[:, :n]))
        tb, tt = [], []
        for _ in range(4):
            tb.append(base())
            tt.append(trail(c, w, ts))
        print(json.dumps({"chunk_rows": c, "mirror_wgs": w, "tile_streams": ts, "lib": os.environ.get("GRF_AMD_LIB", "default"),
                          "bit_identical": same,
                          "base_tiles_mirror_total_ms": [[round(x, 3) for x in b] for b in tb],
                          "trailing_ms": [round(x, 3) for x in tt]}), flush=True)
