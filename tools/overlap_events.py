"""Pipelined C4 step timeline from HIP events (rocprofv3 serialises the two streams, events do not):
after the Gram tiles, the mirror on `main` and the next front on `side`; prints when each ends,
relative to the tiles' end, next to the same pieces run alone.  usage: overlap_events.py [mirror_wgs]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator  # noqa: E402
from grf_amd.engine import DEFAULT_BAND_WIDTH, DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import er_graph_exact_edges  # noqa: E402

wgs = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
eng = GRFEngine("cuda:0")
n, m, L = 100_000, 128, 8
f = diffusion_modulator(L)
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, 0), eng.device)
bw = DEFAULT_BAND_WIDTH
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731


def front(ev=None):
    G = eng.laplacian(A)
    tws = eng.transpose_workspace(n, n, bw)
    if ev is not None:
        ev["lap"].record()
    phi = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=42, count_ws=tws, band_width=bw), want64=False,
                      sync_free=True)
    if ev is not None:
        ev["walk"].record()
    tr = eng.transpose_banded(phi, bw, counted_ws=tws, nnz_bound=n * m * L)
    if ev is not None:
        ev["front"].record()
    return phi, tr


phi, tr = front()
for rep in range(3):
    eng.gram_sparse_upper(phi, tr, K)
    t0 = E()
    t0.record(main)
    ev = {k: E() for k in ("lap", "walk", "front")}
    side.wait_event(t0)
    mirror_end = E()
    eng.gram_mirror(K, n, wgs)
    mirror_end.record(main)
    with torch.cuda.stream(side):
        front(ev)
    torch.cuda.synchronize()
    print(f"[{wgs} WGs] pipelined: mirror ends {t0.elapsed_time(mirror_end):.2f} ms, front: lap {t0.elapsed_time(ev['lap']):.2f}"
          f" walk+compact {t0.elapsed_time(ev['walk']):.2f} transpose {t0.elapsed_time(ev['front']):.2f} ms", flush=True)
# alone
a, b = E(), E()
a.record()
eng.gram_mirror(K, n, wgs)
b.record()
torch.cuda.synchronize()
print(f"mirror alone {a.elapsed_time(b):.2f} ms", flush=True)
ev = {k: E() for k in ("lap", "walk", "front")}
a.record()
front(ev)
torch.cuda.synchronize()
print(f"front alone: lap {a.elapsed_time(ev['lap']):.2f} walk+compact {a.elapsed_time(ev['walk']):.2f} "
      f"transpose {a.elapsed_time(ev['front']):.2f} ms", flush=True)
