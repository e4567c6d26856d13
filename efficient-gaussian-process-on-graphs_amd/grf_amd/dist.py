"""Multi-GPU sharding of the GRF kernel matrix (one process per GPU, RCCL over xGMI).

Walks are independent per source node, so rank r owns the contiguous source
range ``shard_range(n, r, world)``: it runs the walks and builds its Phi rows
locally (Philox is keyed by (seed, source, walk), so the result does not depend
on the number of GPUs).  The one real exchange is Phi itself: K[i, :] needs
every row of Phi, so the ranks all-gather their Phi rows (CSR; ~0.35-0.7 GB at
N = 100k) and each computes its row block K[R_r, :] = Phi[R_r] Phi^T.  K stays
row-sharded; no reduction over the 40 GB K is ever needed (an
all-reduce of K would move ~70 GB per GPU through the xGMI ring).

``mode="allreduce"`` is the north star's literal alternative, kept as an option
so both can be measured: after the same Phi all-gather, rank r computes the
partial Gram over its slice of the inner dimension, K_r = sum over k in C_r of
Phi[:, k] Phi[:, k]^T (all n rows), and the ranks sum the K_r with an all-reduce
in fixed-size buckets.  Every rank ends with the whole K (replicated).

The reference has no distributed code; its only parallelism is a fork pool over
source chunks (sparse_sampler.py:90-114), which this replaces.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.distributed as dist


def _host_staged(group=None) -> bool:
    """gloo has no all-gather for device tensors, so it moves them through host memory (this is how
    the multi-process path is rehearsed with several ranks on one GPU: GRF_DIST_BACKEND=gloo in
    bench.py).  RCCL ("nccl") works on the device tensors directly."""
    return dist.get_backend(group) == "gloo"


def _all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None):
    if out.is_cuda and _host_staged(group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _all_gather_list(outs, inp: torch.Tensor, group=None):
    if inp.is_cuda and _host_staged(group):
        o = [x.cpu() for x in outs]
        dist.all_gather(o, inp.cpu(), group=group)
        for x, y in zip(outs, o):
            x.copy_(y)
    else:
        dist.all_gather(outs, inp, group=group)


def all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None):
    """In-place all-reduce of a device (or host) tensor; host-staged under gloo."""
    if t.is_cuda and _host_staged(group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous source range of ``rank`` (np.array_split boundaries)."""
    base, extra = divmod(n, world)
    b = rank * base + min(rank, extra)
    return b, b + base + (1 if rank < extra else 0)


def allgather_csr_rows(ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, group=None):
    """All-gather row-sharded CSR pieces (rank order) into the full CSR on every rank.

    ``ptr`` is the local int64 row pointer (n_local + 1, starting at 0), ``idx``
    int32 columns, ``val`` values.  Works with RCCL (device tensors) and gloo
    (CPU tensors).  Returns (ptr, idx, val) of the concatenation.
    """
    world = dist.get_world_size(group)
    dev = ptr.device
    n_local = ptr.numel() - 1
    nnz_local = int(ptr[-1].item()) if n_local >= 0 else 0
    sizes = torch.tensor([n_local, nnz_local], dtype=torch.int64, device=dev)
    all_sizes = [torch.empty_like(sizes) for _ in range(world)]
    _all_gather_list(all_sizes, sizes, group=group)
    all_sizes = torch.stack(all_sizes).cpu()
    n_max, nnz_max = int(all_sizes[:, 0].max()), int(all_sizes[:, 1].max())

    counts = torch.zeros(n_max, dtype=torch.int64, device=dev)
    counts[:n_local] = ptr[1:] - ptr[:-1]
    idx_pad = torch.zeros(max(nnz_max, 1), dtype=idx.dtype, device=dev)
    idx_pad[:nnz_local] = idx[:nnz_local]
    val_pad = torch.zeros(max(nnz_max, 1), dtype=val.dtype, device=dev)
    val_pad[:nnz_local] = val[:nnz_local]

    # flat outputs (gloo requires world * numel; RCCL accepts either)
    z = max(nnz_max, 1)
    g_counts = torch.empty(world * n_max, dtype=torch.int64, device=dev)
    g_idx = torch.empty(world * z, dtype=idx.dtype, device=dev)
    g_val = torch.empty(world * z, dtype=val.dtype, device=dev)
    _all_gather_into(g_counts, counts, group=group)
    _all_gather_into(g_idx, idx_pad, group=group)
    _all_gather_into(g_val, val_pad, group=group)
    g_counts, g_idx, g_val = g_counts.view(world, n_max), g_idx.view(world, z), g_val.view(world, z)

    parts_c, parts_i, parts_v = [], [], []
    for r in range(world):
        nr, zr = int(all_sizes[r, 0]), int(all_sizes[r, 1])
        parts_c.append(g_counts[r, :nr])
        parts_i.append(g_idx[r, :zr])
        parts_v.append(g_val[r, :zr])
    cnt = torch.cat(parts_c)
    full_ptr = torch.zeros(cnt.numel() + 1, dtype=torch.int64, device=dev)
    full_ptr[1:] = torch.cumsum(cnt, 0)
    return full_ptr, torch.cat(parts_i), torch.cat(parts_v)


def gather_phi(engine, local, count_ws=None, group=None, band_width=None):
    """All ranks' Phi rows (CSR, float32) from this rank's compacted rows ``local``.

    count_ws: this rank's transpose workspace in which ``walk_phi`` counted the banded transpose's
    buckets for its own rows (global band ids, bands of ``band_width``).  The per-rank counts are
    summed in place with one all-reduce (n_bands * n int32, 5-10 MB at N = 100k), so the caller's
    ``transpose_banded(..., counted_ws=count_ws)`` skips the counting pass over the gathered Phi --
    the same workspace a single GPU's fused count leaves."""
    from .engine import DEFAULT_BAND_WIDTH, DeviceCSR

    n = local.n_cols
    if count_ws is not None and dist.get_world_size(group) > 1:
        nbk = -(-n // (band_width or DEFAULT_BAND_WIDTH)) * n
        all_reduce(count_ws[:4 * nbk].view(torch.int32), group=group)
    if dist.get_world_size(group) == 1:
        return local
    ptr, idx, val32 = allgather_csr_rows(local.ptr, local.idx, local.val32, group)
    return DeviceCSR(n, n, ptr, idx, None, val32, int(idx.numel()))


def allreduce_buckets(t: torch.Tensor, bucket_bytes: int = 1 << 30, group=None) -> torch.Tensor:
    """In-place sum of a (possibly row-padded, row-strided) 2-D tensor over the ranks, one
    contiguous row bucket of at most ``bucket_bytes`` per collective (bounds RCCL's staging)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return t
    rows_per = max(1, bucket_bytes // max(1, t.stride(0) * t.element_size()))
    base = t.as_strided((t.shape[0], t.stride(0)), (t.stride(0), 1)) if t.dim() == 2 else t.view(-1, 1)
    for r0 in range(0, base.shape[0], rows_per):
        all_reduce(base[r0:r0 + rows_per], group=group)
    return t


def sharded_kernel_matrix(engine, A, f, walks_per_node, p_halt, max_walk_length, *, seed=42, group=None,
                          rng=None, mode: str = "rows"):
    """This rank's row block of K = Phi Phi^T (float32, on the engine's device), and its row range.

    ``mode="cols"``: this rank's column block K[:, b:e] (n x (e - b)) instead -- the same numbers
    as the row block (K is symmetric; entry for entry the row mode's K[i, b + j], except that for
    world <= 4 the square K[b:e, b:e] is computed on and above its diagonal and mirrored), from a
    transpose of the rank's own Phi rows only (no replicated transpose, no bucket-count all-reduce).
    ``mode="allreduce"``: every rank returns the whole K (row range (0, n)), assembled as the
    all-reduced sum of per-rank partial Grams over inner-dimension slices."""
    if mode not in ("rows", "cols", "allreduce"):
        raise ValueError(f"mode must be 'rows', 'cols' or 'allreduce', got {mode!r}")
    from . import _lib as C
    from .engine import DeviceCSR

    rng = C.RNG_PHILOX if rng is None else rng
    if rng != C.RNG_PHILOX:
        raise NotImplementedError("sharded walks use Philox (shard-invariant); PCG64 replay is single-GPU")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    from .engine import ROWS_BAND_WIDTH

    G = engine.laplacian(A)
    n = G.n_rows
    b, e = shard_range(n, rank, world)
    bw = ROWS_BAND_WIDTH  # (row-mode Grams: the wide bands)
    if mode == "cols":
        from .engine import cols_band_width
        return _cols_block(engine, G, f, walks_per_node, p_halt, max_walk_length, seed, rng, b, e, group,
                           cols_band_width(e - b)), (b, e)
    tws = None
    if walks_per_node * max_walk_length <= 4096:
        # fused walk -> Phi, counting this rank's buckets of the banded transpose on the way
        tws = engine.transpose_workspace(n, n, bw)
        rows = engine.walk_phi(G, walks_per_node, p_halt, max_walk_length, f, seed=seed, src_begin=b, src_end=e,
                               count_ws=tws, band_width=bw, want64=False)
    else:
        rows = engine.features(engine.walk(G, walks_per_node, p_halt, max_walk_length, rng=rng, seed=seed,
                                           src_begin=b, src_end=e), f)
    local = engine.compact(rows, want64=False, want32=True)
    phi = gather_phi(engine, local, tws, group, band_width=bw) if world > 1 else \
        DeviceCSR(n, n, local.ptr, local.idx, None, local.val32, local.nnz)
    tr = engine.transpose_banded(phi, bw, counted_ws=tws)
    if mode == "allreduce":
        K = engine.gram_sparse_kslice(phi, tr, b, e)
        allreduce_buckets(K, group=group)
        return K, (0, n)
    return engine.gram_sparse(phi, tr, b, e), (b, e)


def _cols_block(engine, G, f, m, p_halt, L, seed, rng, b, e, group, wl):
    """K[:, b:e] from this rank's rows: walks -> Phi rows (counting the local transpose's buckets)
    -> Phi all-gather -> transpose of the local rows -> column-block Gram with all rows' shifts."""
    from .engine import DeviceCSR

    n = G.n_rows
    tws = None
    if m * L <= 4096:
        tws = engine.transpose_workspace(e - b, n, wl)
        rows = engine.walk_phi(G, m, p_halt, L, f, seed=seed, src_begin=b, src_end=e, count_ws=tws, band_width=wl,
                               count_origin=b, want64=False)
    else:
        rows = engine.features(engine.walk(G, m, p_halt, L, rng=rng, seed=seed, src_begin=b, src_end=e), f)
    local = engine.compact(rows, want64=False, want32=True)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    phi = gather_phi(engine, local, None, group) if world > 1 else \
        DeviceCSR(n, n, local.ptr, local.idx, None, local.val32, local.nnz)
    tr = engine.transpose_banded(local, wl, counted_ws=tws)
    # the square K[b:e, b:e] on and above its diagonal, then mirrored, when it is a large enough share
    # of the block to pay for the mirror (N <= 4)
    sym = 4 * (e - b) >= n
    return engine.gram_sparse_cols(phi, engine.phi_row_shifts(phi), tr, sym_row0=b if sym else None)

