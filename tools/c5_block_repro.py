"""Single-process replay of every rank's C5 column-block step (bench.py --workload c5 --gpus W --k-rows R) on one
GPU, step by step with a synchronise and a progress line after each: the un-sharded Phi stands in for the
gathered one (bit-identical: Philox keying), each rank's front walks its own sources, transposes its first R
rows and runs the column-block Gram, the in-run K check and the fingerprint.  usage: c5_block_repro.py W R"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "efficient-gaussian-process-on-graphs_amd")]
import bench  # noqa: E402
from grf_amd import pipeline as P  # noqa: E402
from grf_amd.dist import setup_phi, shard_range  # noqa: E402
from grf_amd.engine import DeviceCSR, GRFEngine, cols_band_width  # noqa: E402
from grf_amd.graphs import powerlaw_graph  # noqa: E402
from tools.gram_hash import fingerprint  # noqa: E402


def say(*a):
    torch.cuda.synchronize()
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    world, kr = int(sys.argv[1]), int(sys.argv[2])
    eng = GRFEngine("cuda:0")
    n, m, L, p = 1_000_000, 64, 8, 0.1
    f = bench.diffusion_modulator(L, 1.0)
    A = DeviceCSR.from_scipy(powerlaw_graph(n, 10.0, 2.5, seed=0), eng.device)
    phi = setup_phi(eng, A, m, p, L, f, seed=42)
    shifts = eng.phi_row_shifts(phi)
    say("setup phi", int(phi.ptr[-1]))
    K = torch.empty((n, eng.leading_dim(kr)), dtype=torch.float32, device=eng.device)
    G = eng.laplacian(A)
    for r in range(world):
        b, e = shard_range(n, r, world)
        pl = P.plan_step(n, m, L, p, f, world=world, rank=r, mode="cols", k_rows=kr, collective=True)
        local = eng.compact(eng.walk_phi(G, m, p, L, f, seed=42, src_begin=b, src_end=e, want64=False),
                            want64=False, want32=True, sync_free=True)
        say(r, "walk", b, e, "bw", pl.band_width)
        blk = DeviceCSR(pl.block_rows, n, local.ptr[:pl.block_rows + 1], local.idx, None, local.val32)
        tr = eng.transpose_banded(blk, pl.band_width, nnz_bound=pl.block_rows * pl.rows_cap, slots=True)
        say(r, "transpose unit", int(tr.rec_unit), "t_rec", tr.t_rec.numel())
        fr = P.Front(phi, tr, local, shifts)
        P.k_assembly(eng, fr, pl, K)
        say(r, "gram")
        chk = P.k_block_check(eng, fr, pl, K)
        say(r, "check", chk["max_ratio"])
        print(r, fingerprint(P.k_view(K, pl)), flush=True)
        del local, blk, tr, fr


if __name__ == "__main__":
    main()
