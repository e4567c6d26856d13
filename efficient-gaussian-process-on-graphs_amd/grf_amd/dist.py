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
in fixed-size buckets.  Every rank ends with the whole K (replicated).  Unlike the row and column
modes, whose entries are the exact fixed-point sums rounded once (bit-identical for any GPU count),
this mode adds the ranks' rounded fp32 partials in the collective's order: K depends on the rank
count and on the reduction order, within the fp32 K tolerance (tests/test_gpu_parity.py).

The reference has no distributed code; its only parallelism is a fork pool over
source chunks (sparse_sampler.py:90-114), which this replaces.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

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


def shard_bounds(weights, world: int) -> List[Tuple[int, int]]:
    """Contiguous ranges of rows with (as nearly as row granularity allows) equal total weight:
    rank r ends at the first row whose inclusive prefix weight reaches (r + 1) / world of the total.
    Every rank gets at least one row when there are at least ``world`` rows."""
    import numpy as np

    w = np.asarray(weights, dtype=np.float64).ravel()
    n = w.size
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * (world - 1)
    cum = np.cumsum(w)
    total = cum[-1]
    if total <= 0:
        return [shard_range(n, r, world) for r in range(world)]
    ends = []
    prev = 0
    for r in range(world - 1):
        e = int(np.searchsorted(cum, total * (r + 1) / world, side="left")) + 1
        e = max(e, prev + (1 if n - prev > world - 1 - r else 0))  # a row for everyone left, if possible
        e = min(e, n - (world - 1 - r) if n >= world else n)
        ends.append(e)
        prev = e
    ends.append(n)
    starts = [0] + ends[:-1]
    return list(zip(starts, ends))


# per-row cost model of one step (C4 measurements): the K block row's write
# (4 n bytes at ~6.3 TB/s) and the Gram's record gathers (g_j records of 6 B with ~1.8x line
# amplification at ~7.3 TB/s, g_j = sum over Phi[j, k] != 0 of the column count of k)
_K_WRITE_NS_PER_ENTRY = 4.0 / 6.3
_GATHER_NS_PER_RECORD = 6.0 * 1.8 / 7.3


def row_costs(engine, phi) -> torch.Tensor:
    """Estimated step time of every row of Phi (device float64 [n]): its K row's write plus its
    Gram tiles' record gathers.  A row's gathers are g_j = sum_{k in row j} c_k, c_k = nnz of
    column k -- rows whose walks reach hubs cost more than their Phi nnz alone says."""
    n_rows, n_cols = phi.n_rows, phi.n_cols
    nnz = phi.nnz
    idx = phi.idx[:nnz].long()
    col_cnt = torch.bincount(idx, minlength=n_cols).to(torch.float64)
    per_entry = col_cnt[idx]
    csum = torch.zeros(nnz + 1, dtype=torch.float64, device=per_entry.device)
    csum[1:] = torch.cumsum(per_entry, 0)
    g = csum[phi.ptr[1:]] - csum[phi.ptr[:-1]]
    return _K_WRITE_NS_PER_ENTRY * n_cols + _GATHER_NS_PER_RECORD * g


def setup_phi(engine, A, m: int, p_halt: float, L: int, f, *, seed: int = 42):
    """Phi of ALL sources from one setup walk (float32 CSR on the engine's device).  Philox is keyed
    by (seed, source, walk), so every rank computes the identical Phi without a collective, and it
    is the Phi every step with this seed produces.  Run once, outside the timed steps."""
    G = engine.laplacian(A)
    return engine.compact(engine.walk_phi(G, m, p_halt, L, f, seed=seed, want64=False), want64=False)


def balanced_shards(engine, A, m: int, p_halt: float, L: int, f, world: int, *, seed: int = 42,
                    policy: str = "phi", phi=None) -> List[Tuple[int, int]]:
    """Source shards of equal estimated step time.  policy "phi": the setup walk's Phi (``setup_phi``,
    or ``phi`` when the caller already has it) gives each row's cost (``row_costs``), and the ranks
    get contiguous ranges of equal total cost.  policy "nodes": equal node counts.
    Run once per (graph, m, L, seed), outside the timed steps."""
    if policy == "nodes":
        n = A.n_rows if hasattr(A, "n_rows") else A.shape[0]
        return [shard_range(n, r, world) for r in range(world)]
    if policy != "phi":
        raise ValueError(f"policy must be 'phi' or 'nodes', got {policy!r}")
    if phi is None:
        phi = setup_phi(engine, A, m, p_halt, L, f, seed=seed)
    return shard_bounds(row_costs(engine, phi).cpu().numpy(), world)


def shard_entries(phi, shards: Sequence[Tuple[int, int]]) -> List[int]:
    """Phi entries of every shard's rows (one host read of the row pointer; setup only).  With the
    step's seed these are exactly the entries each rank's compaction produces every step, so their
    maximum is a tight ``entries_bound`` for the sync-free Phi all-gather (``gather_phi``)."""
    ptr = phi.ptr.cpu()
    return [int(ptr[e] - ptr[b]) for b, e in shards]


_GATHER_OVERFLOW = {}  # device -> int32 flag: a bounded all-gather met a rank with more entries than its bound
_ROW0 = {}             # (device, rows per rank) -> int64 first global row of every rank, on the device

# Collective instrumentation (bench.py --gpus N): when a list, every Phi all-gather appends
# (start event, end event, bytes sent by this rank, bytes received) -- HIP events on the issuing stream around
# the collectives (RCCL runs them on its own stream, which the issuing stream then waits for: the
# interval covers the transfer and the wait for the slowest rank).  None: no events recorded.
GATHER_STATS: Optional[list] = None


def _gather_timer():
    if GATHER_STATS is None or not torch.cuda.is_available():
        return None
    ev = torch.cuda.Event(enable_timing=True)
    ev.record()
    return ev


def _gather_record(start, sent: int, received: int):
    if start is None:
        return
    end = torch.cuda.Event(enable_timing=True)
    end.record()
    GATHER_STATS.append((start, end, int(sent), int(received)))


def _row0(rows_per_rank: Sequence[int], dev) -> torch.Tensor:
    """First global row of every rank as a device tensor, made once per shard layout (a pageable
    host-to-device copy per step would synchronise the issuing stream inside the pipelined front)."""
    key = (str(dev), tuple(int(r) for r in rows_per_rank))
    t = _ROW0.get(key)
    if t is None:
        starts = [0]
        for r in rows_per_rank[:-1]:
            starts.append(starts[-1] + int(r))
        t = _ROW0[key] = torch.tensor(starts, dtype=torch.int64, device=dev)
    return t


def check_gather_overflow(device) -> None:
    """Raise if any bounded Phi all-gather on ``device`` since the last check met a rank whose
    entries exceeded the bound (that rank's rows were gathered empty, so K is wrong).  One host read;
    call it after the timed steps."""
    flag = _GATHER_OVERFLOW.get(torch.device(device))
    if flag is not None and int(flag.item()):
        flag.zero_()
        raise RuntimeError("bounded Phi all-gather: a rank's Phi entries exceeded entries_bound "
                           "(the gathered Phi is incomplete; size the bound from this step's seed)")


def allgather_csr_rows_bounded(ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor,
                               rows_per_rank: Sequence[int], entries_bound: int, group=None):
    """All-gather of row-sharded CSR pieces with NO host round trip: every rank sends its first
    ``entries_bound`` column / value entries (the capacity its sync-free compaction allocated,
    rows x the padded row capacity; entries past its nnz are ignored) and its row pointers padded
    to the largest shard; the full row pointers come from the gathered counts on the device, and
    ``grf_concat_segments`` packs each rank's entries to its final offset.  The row counts are the
    host-known shard sizes.  A tighter ``entries_bound`` (``shard_entries`` of the setup walk) moves
    only the entries that exist; a rank above it is gathered empty and flagged
    (``check_gather_overflow``).  Returns (ptr, idx, val) of the concatenation (nnz = ptr[-1], read
    lazily; idx / val are sized world x entries_bound)."""
    from . import _lib as C
    from .engine import _p, get_engine

    world = dist.get_world_size(group)
    dev = ptr.device
    n_max = max(rows_per_rank)
    B = max(int(entries_bound), 1)
    t0 = _gather_timer()
    lp = torch.empty(n_max + 1, dtype=torch.int64, device=dev)
    n_loc = ptr.numel() - 1
    lp[:n_loc + 1] = ptr
    lp[n_loc + 1:] = ptr[-1]
    g_ptr = torch.empty(world * (n_max + 1), dtype=torch.int64, device=dev)
    _all_gather_into(g_ptr, lp, group=group)
    g_ptr = g_ptr.view(world, n_max + 1)
    send_i = idx[:B] if idx.numel() >= B else torch.cat([idx, idx.new_zeros(B - idx.numel())])
    send_v = val[:B] if val.numel() >= B else torch.cat([val, val.new_zeros(B - val.numel())])
    g_idx = torch.empty(world * B, dtype=idx.dtype, device=dev)
    g_val = torch.empty(world * B, dtype=val.dtype, device=dev)
    _all_gather_into(g_idx, send_i.contiguous(), group=group)
    _all_gather_into(g_val, send_v.contiguous(), group=group)
    # a rank whose entries exceed the bound sent a truncated segment: its rows are gathered empty
    # (every read and write stays inside the buffers) and the overflow flag is raised on the device
    seg_len = torch.stack([g_ptr[r, n_r] for r, n_r in enumerate(rows_per_rank)]).contiguous()
    fits = seg_len <= B
    flag = _GATHER_OVERFLOW.setdefault(dev, torch.zeros((), dtype=torch.int32, device=dev))
    flag.bitwise_or_((~fits.all()).to(torch.int32))
    seg_len = seg_len * fits
    counts = torch.cat([(g_ptr[r, 1:n_r + 1] - g_ptr[r, :n_r]) * fits[r] for r, n_r in enumerate(rows_per_rank)])
    full_ptr = torch.zeros(counts.numel() + 1, dtype=torch.int64, device=dev)
    full_ptr[1:] = torch.cumsum(counts, 0)
    dst_off = full_ptr[_row0(rows_per_rank, dev)].contiguous()
    out_i = torch.empty(world * B, dtype=idx.dtype, device=dev)
    out_v = torch.empty(world * B, dtype=val.dtype, device=dev)
    if dev.type == "cuda":
        eng = get_engine(dev)
        for src, dst in ((g_idx, out_i), (g_val, out_v)):
            if src.element_size() != 4:
                raise ValueError("allgather_csr_rows_bounded: 4-byte column and value entries expected")
            C.check(eng.lib.grf_concat_segments(world, B, _p(src), _p(seg_len), _p(dst_off), _p(dst), eng.stream),
                    "grf_concat_segments")
    else:  # (CPU tensors: the host-side test harness; sizes are host-readable there)
        for r in range(world):
            o, n_e = int(dst_off[r]), int(seg_len[r])
            out_i[o:o + n_e] = g_idx[r * B:r * B + n_e]
            out_v[o:o + n_e] = g_val[r * B:r * B + n_e]
    sent = (n_max + 1) * 8 + B * (idx.element_size() + val.element_size())
    _gather_record(t0, sent, world * sent)
    return full_ptr, out_i, out_v


def allgather_csr_rows(ptr: torch.Tensor, idx: torch.Tensor, val: torch.Tensor, group=None):
    """All-gather row-sharded CSR pieces (rank order) into the full CSR on every rank, exactly sized.

    ``ptr`` is the local int64 row pointer (n_local + 1, starting at 0), ``idx``
    int32 columns, ``val`` values.  Works with RCCL (device tensors) and gloo
    (CPU tensors).  Returns (ptr, idx, val) of the concatenation.  One host read of the
    gathered (rows, nnz) pairs sizes the transfer; ``allgather_csr_rows_bounded`` avoids it.
    """
    world = dist.get_world_size(group)
    dev = ptr.device
    n_local = ptr.numel() - 1
    sizes = torch.stack([torch.tensor(n_local, dtype=torch.int64, device=dev), ptr[-1].to(torch.int64)])
    all_sizes = [torch.empty_like(sizes) for _ in range(world)]
    _all_gather_list(all_sizes, sizes, group=group)
    all_sizes = torch.stack(all_sizes).cpu()
    nnz_local = int(all_sizes[dist.get_rank(group), 1])
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


def gather_phi(engine, local, count_ws=None, group=None, band_width=None, shards=None, entries_bound=None,
               row_cap=None, always=False):
    """All ranks' Phi rows (CSR, float32) from this rank's compacted rows ``local``.

    shards: every rank's (begin, end) source range.  When given and ``local`` came from a
    sync-free compaction (``nnz_bound`` = rows x row capacity), the gather reads nothing back to
    the host (``allgather_csr_rows_bounded``); otherwise one host read sizes it exactly.
    entries_bound: the per-rank entry bound of that gather (default: rows x the row capacity, which
    no rank can exceed; ``shard_entries`` of the setup walk gives the exact, ~2.4x smaller one at C4).
    row_cap: the padded row capacity of every rank's compaction (global: min(m L, n)); default: this
    rank's nnz_bound / rows.  The bounded / exact choice depends on global information only, so every
    rank issues the same collectives (an empty shard included).

    count_ws: this rank's transpose workspace in which ``walk_phi`` counted the banded transpose's
    buckets for its own rows (global band ids, bands of ``band_width``).  The per-rank counts are
    summed in place with one all-reduce (n_bands * n int32, 5-10 MB at N = 100k), so the caller's
    ``transpose_banded(..., counted_ws=count_ws)`` skips the counting pass over the gathered Phi --
    the same workspace a single GPU's fused count leaves.

    always: gather even with one rank (the pipeline's planned collective step: one rank rehearses the
    RCCL all-gather); otherwise one rank returns ``local`` as it is."""
    from .engine import DEFAULT_BAND_WIDTH, DeviceCSR

    n = local.n_cols
    if count_ws is not None and dist.get_world_size(group) > 1:
        nbk = -(-n // (band_width or DEFAULT_BAND_WIDTH)) * n
        all_reduce(count_ws[:4 * nbk].view(torch.int32), group=group)
    if dist.get_world_size(group) == 1 and not always:
        return local
    bound = getattr(local, "nnz_bound", None)
    if shards is not None and (bound is not None or row_cap is not None) and (row_cap or entries_bound
                                                                          or local.n_rows > 0):
        cap = int(row_cap) if row_cap else -(-bound // max(local.n_rows, 1))
        rows = [e - b for b, e in shards]
        B = int(entries_bound) if entries_bound else max(rows) * cap
        ptr, idx, val32 = allgather_csr_rows_bounded(local.ptr, local.idx, local.val32, rows, B, group)
        out = DeviceCSR(n, n, ptr, idx, None, val32, None)
        out.nnz_bound = int(idx.numel())
        return out
    t0 = _gather_timer()
    ptr, idx, val32 = allgather_csr_rows(local.ptr, local.idx, local.val32, group)
    _gather_record(t0, (local.n_rows + 1) * 8 + 8 * local.nnz, 8 * int(idx.numel()) + 8 * (n + 1))
    return DeviceCSR(n, n, ptr, idx, None, val32, int(idx.numel()))


# (bench.py --mode allreduce): when a list, every bucketed K all-reduce appends (start event, end event, bytes
# reduced by this rank) -- HIP events on the issuing stream around the whole bucket loop
ALLREDUCE_STATS: Optional[list] = None


def allreduce_buckets(t: torch.Tensor, bucket_bytes: int = 1 << 30, group=None) -> torch.Tensor:
    """In-place sum of a (possibly row-padded, row-strided) 2-D tensor over the ranks, one
    contiguous row bucket of at most ``bucket_bytes`` per collective (bounds RCCL's staging)."""
    if not dist.is_initialized():
        return t  # (one rank in an initialised group still runs the collectives: the RCCL rehearsal)
    rows_per = max(1, bucket_bytes // max(1, t.stride(0) * t.element_size()))
    base = t.as_strided((t.shape[0], t.stride(0)), (t.stride(0), 1)) if t.dim() == 2 else t.view(-1, 1)
    start = None
    if ALLREDUCE_STATS is not None and torch.cuda.is_available() and t.is_cuda:
        start = torch.cuda.Event(enable_timing=True)
        start.record()
    for r0 in range(0, base.shape[0], rows_per):
        all_reduce(base[r0:r0 + rows_per], group=group)
    if start is not None:
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        ALLREDUCE_STATS.append((start, end, int(base.numel() * base.element_size())))
    return t


def sharded_kernel_matrix(engine, A, f, walks_per_node, p_halt, max_walk_length, *, seed=42, group=None,
                          rng=None, mode: str = "rows", shards: Optional[Sequence[Tuple[int, int]]] = None):
    """This rank's row block of K = Phi Phi^T (float32, on the engine's device), and its row range.

    ``mode="cols"``: this rank's column block K[:, b:e] (n x (e - b)) instead -- the same numbers
    as the row block (K is symmetric; entry for entry the row mode's K[i, b + j], except that for
    world <= 4 the square K[b:e, b:e] is computed on and above its diagonal and mirrored), from a
    transpose of the rank's own Phi rows only (no replicated transpose, no bucket-count all-reduce).
    ``mode="allreduce"``: every rank returns the whole K (row range (0, n)), assembled as the
    all-reduced sum of per-rank partial Grams over inner-dimension slices.
    ``shards``: every rank's source range (default: equal node counts; ``balanced_shards`` for
    equal estimated work)."""
    if mode not in ("rows", "cols", "allreduce"):
        raise ValueError(f"mode must be 'rows', 'cols' or 'allreduce', got {mode!r}")
    from . import _lib as C
    from .engine import SELF_COUNT_TRANSPOSE, DeviceCSR  # noqa: F401

    rng = C.RNG_PHILOX if rng is None else rng
    if rng != C.RNG_PHILOX:
        raise NotImplementedError("sharded walks use Philox (shard-invariant); PCG64 replay is single-GPU")
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    from .engine import ROWS_BAND_WIDTH

    G = engine.laplacian(A)
    n = G.n_rows
    shards = list(shards) if shards is not None else [shard_range(n, r, world) for r in range(world)]
    b, e = shards[rank]
    bw = ROWS_BAND_WIDTH  # (row-mode Grams: the wide bands)
    if mode == "cols":
        from .engine import cols_band_width
        return _cols_block(engine, G, f, walks_per_node, p_halt, max_walk_length, seed, rng, b, e, group,
                           cols_band_width(e - b), shards), (b, e)
    tws = None
    if walks_per_node * max_walk_length <= 4096:
        # fused walk -> Phi (counting this rank's buckets of the banded transpose on the way when the
        # transpose does not count them itself, GRF_TRANSPOSE_SELF=0)
        tws = None if SELF_COUNT_TRANSPOSE else engine.transpose_workspace(n, n, bw)
        rows = engine.walk_phi(G, walks_per_node, p_halt, max_walk_length, f, seed=seed, src_begin=b, src_end=e,
                               count_ws=tws, band_width=bw if tws is not None else 0, want64=False)
    else:
        rows = engine.features(engine.walk(G, walks_per_node, p_halt, max_walk_length, rng=rng, seed=seed,
                                           src_begin=b, src_end=e), f)
    local = engine.compact(rows, want64=False, want32=True, sync_free=True)
    phi = gather_phi(engine, local, tws, group, band_width=bw, shards=shards,
                     row_cap=max(1, min(walks_per_node * max_walk_length, n))) if world > 1 else local
    tr = engine.transpose_banded(phi, bw, counted_ws=tws, nnz_bound=phi.nnz_bound)
    if mode == "allreduce":
        K = engine.gram_sparse_kslice(phi, tr, b, e)
        allreduce_buckets(K, group=group)
        return K, (0, n)
    return engine.gram_sparse(phi, tr, b, e), (b, e)


def _cols_block(engine, G, f, m, p_halt, L, seed, rng, b, e, group, wl, shards=None):
    """K[:, b:e] from this rank's rows: walks -> Phi rows -> Phi all-gather -> transpose of the local
    rows -> column-block Gram with all rows' shifts."""
    from .engine import SELF_COUNT_TRANSPOSE

    n = G.n_rows
    tws = None
    if m * L <= 4096:
        tws = None if SELF_COUNT_TRANSPOSE else engine.transpose_workspace(e - b, n, wl)
        rows = engine.walk_phi(G, m, p_halt, L, f, seed=seed, src_begin=b, src_end=e, count_ws=tws,
                               band_width=wl if tws is not None else 0, count_origin=b, want64=False)
    else:
        rows = engine.features(engine.walk(G, m, p_halt, L, rng=rng, seed=seed, src_begin=b, src_end=e), f)
    local = engine.compact(rows, want64=False, want32=True, sync_free=True)
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    phi = gather_phi(engine, local, None, group, shards=shards, row_cap=max(1, min(m * L, n))) if world > 1 else local
    tr = engine.transpose_banded(local, wl, counted_ws=tws, nnz_bound=local.nnz_bound)
    # the square K[b:e, b:e] on and above its diagonal, then mirrored, when it is a large enough share
    # of the block to pay for the mirror (N <= 4)
    sym = 4 * (e - b) >= n
    return engine.gram_sparse_cols(phi, engine.phi_row_shifts(phi), tr, sym_row0=b if sym else None)

