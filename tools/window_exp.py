"""Where the pipelined window goes (timing-only experiment, C4): the mirror on `main` beside
variants of the next front on `side`, HIP events.  Variants (the last two are NOT valid steps --
they reuse step 0's bucket counts -- they only bound what removing a piece could gain):
  full      : the bench's front (Laplacian, walk_phi with bucket-count atomics, compaction, transpose)
  nocount   : walk_phi without the count atomics, the transpose planned from step 0's counts
  walkonly  : Laplacian + walk_phi (+ counts), nothing after
  none      : the mirror alone"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
from bench import diffusion_modulator  # noqa: E402
from grf_amd.engine import DEFAULT_BAND_WIDTH, DeviceCSR, GRFEngine  # noqa: E402
from grf_amd.graphs import er_graph_exact_edges  # noqa: E402

eng = GRFEngine("cuda:0")
n, m, L = 100_000, 128, 8
f = diffusion_modulator(L)
A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, 0), eng.device)
bw = DEFAULT_BAND_WIDTH
K = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
side_hi = torch.cuda.Stream(priority=-1)  # (ROCm: lower number = higher priority)
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
saved = {}


def front(variant):
    G = eng.laplacian(A)
    if variant == "nocount":
        rows = eng.walk_phi(G, m, 0.1, L, f, seed=42, want64=False)
        phi = eng.compact(rows, want64=False, sync_free=True)
        return phi, eng.transpose_banded(phi, bw, counted_ws=saved["tws"].clone(), nnz_bound=n * m * L)
    tws = eng.transpose_workspace(n, n, bw)
    rows = eng.walk_phi(G, m, 0.1, L, f, seed=42, count_ws=tws, band_width=bw, want64=False)
    if variant == "walkonly":
        return None
    phi = eng.compact(rows, want64=False, sync_free=True)
    if "tws" not in saved:
        saved["tws"] = tws.clone()
    return phi, eng.transpose_banded(phi, bw, counted_ws=tws, nnz_bound=n * m * L)


phi, tr = front("full")
eng.gram_sparse_upper(phi, tr, K)
torch.cuda.synchronize()
configs = [(v, 1024, "normal") for v in ("none", "full", "nocount", "walkonly")]
configs += [(v, w, pr) for w in (0, 512, 768, 2048) for pr in ("normal", "high") for v in ("none", "full")]
for variant, wgs, prio in configs + configs[:2]:
    sd = side_hi if prio == "high" else side
    ts = []
    for rep in range(3):
        t0 = E()
        t0.record(main)
        sd.wait_event(t0)
        eng.gram_mirror(K, n, wgs)  # (issued first, as in the bench)
        if variant != "none":
            with torch.cuda.stream(sd):
                front(variant)
        t1 = E()
        side_done = E()
        side_done.record(sd)
        main.wait_event(side_done)
        t1.record(main)
        torch.cuda.synchronize()
        ts.append(t0.elapsed_time(t1))
    a, b = E(), E()
    a.record()
    if variant != "none":
        front(variant)
    b.record()
    torch.cuda.synchronize()
    print(f"{variant:9s} mirror_wgs={wgs:5d} front_prio={prio:6s} window {min(ts):.2f} / {sum(ts) / len(ts):.2f} ms (min / mean), front alone {a.elapsed_time(b):.2f} ms",
          flush=True)
