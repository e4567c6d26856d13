"""Timing-only experiment (C4): step s's mirror pass beside step s+1's Gram tiles, on two HIP streams
with two resident K buffers (80 GB), against the two kernels back to back.  HIP events; the Gram
writes K_b while the mirror completes K_a, so both results stay valid."""
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
ld = eng.leading_dim(n)
Ka = torch.empty((n, ld), dtype=torch.float32, device=eng.device)
Kb = torch.empty((n, ld), dtype=torch.float32, device=eng.device)
main = torch.cuda.current_stream()
side = torch.cuda.Stream()
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731

G = eng.laplacian(A)
tws = eng.transpose_workspace(n, n, bw)
rows = eng.walk_phi(G, m, 0.1, L, f, seed=42, count_ws=tws, band_width=bw, want64=False)
phi = eng.compact(rows, want64=False, sync_free=True)
tr = eng.transpose_banded(phi, bw, counted_ws=tws, nnz_bound=n * m * L)
eng.gram_sparse_upper(phi, tr, Ka)
eng.gram_mirror(Ka, n)
torch.cuda.synchronize()


def timed(fn, reps=3):
    ts = []
    for _ in range(reps):
        t0, t1 = E(), E()
        t0.record(main)
        fn()
        t1.record(main)
        torch.cuda.synchronize()
        ts.append(t0.elapsed_time(t1))
    return min(ts), sum(ts) / len(ts)


def both(wgs, mirror_first):
    def run():
        start = E()
        start.record(main)
        side.wait_event(start)
        if mirror_first:
            with torch.cuda.stream(side):
                eng.gram_mirror(Ka, n, wgs)
            eng.gram_sparse_upper(phi, tr, Kb)
        else:
            eng.gram_sparse_upper(phi, tr, Kb)
            with torch.cuda.stream(side):
                eng.gram_mirror(Ka, n, wgs)
        done = E()
        done.record(side)
        main.wait_event(done)
    return run


print("gram alone      %.2f / %.2f ms" % timed(lambda: eng.gram_sparse_upper(phi, tr, Kb)), flush=True)
for wgs in (0, 1024):
    print("mirror alone wgs=%5d %.2f / %.2f ms" % ((wgs,) + timed(lambda: eng.gram_mirror(Ka, n, wgs))), flush=True)
print("serial (gram then mirror) %.2f / %.2f ms" % timed(lambda: (eng.gram_sparse_upper(phi, tr, Kb), eng.gram_mirror(Ka, n, 1024))),
      flush=True)
for wgs in (256, 512, 1024, 0):
    for mf in (True, False):
        print("overlap wgs=%5d mirror_first=%d %.2f / %.2f ms" % ((wgs, mf) + timed(both(wgs, mf))), flush=True)


# the whole step: front F (Laplacian, walk + Phi, compaction, transpose), Gram G, mirror M
def front():
    G_ = eng.laplacian(A)
    tws_ = eng.transpose_workspace(n, n, bw)
    rows_ = eng.walk_phi(G_, m, 0.1, L, f, seed=43, count_ws=tws_, band_width=bw, want64=False)
    phi_ = eng.compact(rows_, want64=False, sync_free=True)
    return phi_, eng.transpose_banded(phi_, bw, counted_ws=tws_, nnz_bound=n * m * L)


def current(wgs=1024):
    # one K buffer: G(s) then M(s) on main beside F(s+1) on side (the bench's pipelined period)
    def run():
        eng.gram_sparse_upper(phi, tr, Kb)
        start = E()
        start.record(main)
        side.wait_event(start)
        eng.gram_mirror(Kb, n, wgs)
        with torch.cuda.stream(side):
            front()
        done = E()
        done.record(side)
        main.wait_event(done)
    return run


def option_b(wgs=1024):
    # two K buffers: M(s) on side beside F(s+1) then G(s+1) on main
    def run():
        start = E()
        start.record(main)
        side.wait_event(start)
        with torch.cuda.stream(side):
            eng.gram_mirror(Ka, n, wgs)
        front()
        eng.gram_sparse_upper(phi, tr, Kb)
        done = E()
        done.record(side)
        main.wait_event(done)
    return run


def option_a(wgs=1024):
    # two K buffers: G(s+1) on main beside M(s) then F(s+2) on side
    def run():
        start = E()
        start.record(main)
        side.wait_event(start)
        with torch.cuda.stream(side):
            eng.gram_mirror(Ka, n, wgs)
            front()
        eng.gram_sparse_upper(phi, tr, Kb)
        done = E()
        done.record(side)
        main.wait_event(done)
    return run


print("front alone %.2f / %.2f ms" % timed(front), flush=True)
for wgs in (1024, 768, 512):
    print("period current  wgs=%5d %.2f / %.2f ms" % ((wgs,) + timed(current(wgs))), flush=True)
    print("period option B wgs=%5d %.2f / %.2f ms" % ((wgs,) + timed(option_b(wgs))), flush=True)
    print("period option A wgs=%5d %.2f / %.2f ms" % ((wgs,) + timed(option_a(wgs))), flush=True)
