"""The timed hot path of ``bench.py`` as library functions, so that the parity tests run exactly it.

One step (CSR adjacency resident in HBM -> full dense fp32 K resident in HBM) is
a *front* and a *K assembly*:

* front: normalised Laplacian (a1, ``graph_utils.py:5-30``) -> fused Philox walks straight to
  Phi rows, counting the banded transpose's buckets on the way (a7 + a9's
  ``Phi = sum_l f_l M_l``, ``sparse_sampler.py:26-56`` and ``fast_grf_kernel_general.py:47-52``)
  -> sync-free compaction -> [Phi all-gather, N > 1] -> banded transpose of Phi (or of this rank's
  own rows for column blocks).
* K assembly (a9's ``Phi @ Phi.T``, ``fast_grf_kernel_general.py:55``): one GPU, whole K: the
  Gram tiles on and above the diagonal band + the mirror pass; row blocks; column blocks
  ``K[:, R_r]`` (= the rank's rows: K is symmetric); or the north star's literal partial K over
  an inner slice + all-reduce.

``plan_step`` fixes every size and mode up front, so the front reads nothing back to the host.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch

from . import _lib as C
from .engine import (DEFAULT_BAND_WIDTH, ROWS_BAND_WIDTH, SELF_COUNT_TRANSPOSE, DeviceCSR, GRFEngine, PaddedRows,
                     cols_band_width)

# column blocks with sparse buckets take the GRF_REC_SLOT transpose (GRF_REC_SLOTS=0: packed pairs, A/B)
SLOTS_DEFAULT = os.environ.get("GRF_REC_SLOTS", "1") == "1"
# one GPU, column blocks: the compaction leaves the rows' Gram shift statistics (GRF_COMPACT_STATS=0: a
# separate pass over Phi's values, A/B)
COMPACT_STATS = os.environ.get("GRF_COMPACT_STATS", "1") == "1"
# one GPU, column blocks (C5): Phi stays the walk's padded rows -- the column-block Gram and the row shifts read
# them directly and only the block's own rows are compacted for its transpose (GRF_PADDED_PHI=0: the whole
# compaction, A/B)
PADDED_PHI = os.environ.get("GRF_PADDED_PHI", "1") == "1"
# pipelined whole K with the hub-column split: the next front starts beside the hub panel's MFMA Gram,
# not at the mirror (Enron 8.66-8.68 -> 8.13-8.23 ms per K, profiles/r03_hub_early_front_ab.txt;
# GRF_HUB_EARLY_FRONT=0: at the mirror)
HUB_EARLY_FRONT = os.environ.get("GRF_HUB_EARLY_FRONT", "1") == "1"


@dataclass
class StepPlan:
    """Sizes and modes of one step on one rank."""

    n: int
    m: int
    L: int
    p_halt: float
    f: np.ndarray
    seed: int = 42
    world: int = 1
    rank: int = 0
    src: Tuple[int, int] = (0, 0)  # this rank's walk sources [b, e) (= its K rows / columns)
    shards: Optional[List[Tuple[int, int]]] = None  # every rank's [b, e) (N > 1)
    k_rows: int = 0                # 0: all of the rank's rows; R: only [b, b + R)
    mode: str = "sym"              # "sym" (one GPU, whole K), "rows", "cols", "allreduce"
    band_width: int = DEFAULT_BAND_WIDTH
    cols_sym: bool = False         # column blocks: the square K[b:e, b:e] by the symmetric enumeration
    hubs: int = 0                  # "sym": Phi's densest columns as a dense MFMA panel (hub-column split)
    skewed: bool = False           # "sym": Phi's column counts are skewed -> pair-balanced wave shares (row_cuts)
    group: object = None           # torch.distributed group (N > 1)
    collective: bool = False       # the Phi all-gather runs (N > 1; or one rank, to rehearse RCCL on one GPU)
    gather_bound: int = 0          # N > 1: per-rank Phi entries moved by the all-gather (0: rows x rows_cap;
    #                                dist.shard_entries of the setup walk: exact, checked by check_gather_overflow)
    extra: dict = field(default_factory=dict)

    @property
    def b(self) -> int:
        return self.src[0]

    @property
    def e(self) -> int:
        return self.src[1]

    @property
    def kr_end(self) -> int:
        return min(self.e, self.b + self.k_rows) if self.k_rows else self.e

    @property
    def block_rows(self) -> int:
        """Rows of K this rank writes (all n for the all-reduce mode)."""
        return self.n if self.mode == "allreduce" else self.kr_end - self.b

    @property
    def rows_cap(self) -> int:
        """walk_phi's padded row capacity (the bound that sizes everything downstream)."""
        return max(1, min(self.m * self.L, self.n))


def plan_step(n: int, m: int, L: int, p_halt: float, f, *, seed: int = 42, world: int = 1, rank: int = 0,
              mode: str = "cols", k_rows: int = 0, band_width: int = 0, no_sym: bool = False,
              shards: Optional[List[Tuple[int, int]]] = None, group=None,
              collective: Optional[bool] = None) -> StepPlan:
    """The bench's mode rules: one GPU whole K -> symmetric mode; N > 1 or K-row workloads -> column
    blocks (``mode="cols"``), row blocks (``"rows"``) or the all-reduce option (``"allreduce"``).
    shards: every rank's source range (default: equal node counts; dist.balanced_shards for equal
    estimated work).  collective (default: world > 1): plan the multi-GPU step -- column / row
    blocks after a Phi all-gather -- even for one rank (bench.py's GRF_DIST_FORCE=1 runs RCCL's
    collectives on a one-GPU box through exactly the N > 1 code)."""
    from .dist import shard_range

    if mode not in ("cols", "rows", "allreduce"):
        raise ValueError(f"mode must be 'cols', 'rows' or 'allreduce', got {mode!r}")
    if k_rows and mode == "allreduce":
        raise ValueError("k_rows applies to the row / column modes only")
    shards = list(shards) if shards is not None else [shard_range(n, r, world) for r in range(world)]
    if len(shards) != world or shards[0][0] != 0 or shards[-1][1] != n or \
            any(shards[r][1] != shards[r + 1][0] for r in range(world - 1)):
        raise ValueError("shards must be contiguous ranges covering [0, n) in rank order")
    b, e = shards[rank]
    pl = StepPlan(n, int(m), int(L), float(p_halt), np.asarray(f, np.float64), int(seed), world, rank, (b, e),
                  shards, int(k_rows), mode, group=group)
    pl.collective = world > 1 if collective is None else bool(collective)
    if mode == "cols" and (pl.collective or k_rows):
        pl.mode = "cols"
        pl.band_width = band_width or cols_band_width(pl.block_rows)
        pl.cols_sym = not no_sym and 4 * pl.block_rows >= n
    elif mode == "allreduce":
        pl.band_width = band_width or ROWS_BAND_WIDTH
    elif not pl.collective and not no_sym and not k_rows:
        pl.mode = "sym"
        pl.band_width = band_width or DEFAULT_BAND_WIDTH
    else:
        pl.mode = "rows"
        pl.band_width = band_width or ROWS_BAND_WIDTH
    return pl


@dataclass
class Front:
    phi: DeviceCSR                 # all rows of Phi (float32 values)
    tr: object                     # Banded transpose (of all rows, or of this rank's block for "cols")
    local: DeviceCSR               # this rank's own rows
    row_shift: Optional[torch.Tensor] = None  # "cols": every row's fixed-point shift


class PaddedPhi:
    """Phi as the walk's padded rows (``rows``: row r's entries at r * cap, no compaction), for the K assembly
    of one GPU's column block; every other attribute is the compacted CSR's, built on first use (checks and
    tests, outside the timed steps)."""

    def __init__(self, eng: GRFEngine, rows: PaddedRows):
        self.eng, self.rows, self._csr = eng, rows, None

    @property
    def csr(self) -> DeviceCSR:
        if self._csr is None:
            self._csr = self.eng.compact(self.rows, want64=False, want32=True)
        return self._csr

    def __getattr__(self, name):
        if name in ("eng", "rows", "_csr"):
            raise AttributeError(name)
        return getattr(self.csr, name)


def phi_csr(phi) -> DeviceCSR:
    """A front's Phi as a CSR (compacting padded rows on first use)."""
    return phi.csr if isinstance(phi, PaddedPhi) else phi


def alloc_k(eng: GRFEngine, pl: StepPlan) -> torch.Tensor:
    """The resident K buffer of one step (reused across steps)."""
    if pl.mode == "cols":
        return torch.empty((pl.n, eng.leading_dim(pl.block_rows)), dtype=torch.float32, device=eng.device)
    return torch.empty((pl.block_rows, eng.leading_dim(pl.n)), dtype=torch.float32, device=eng.device)


def front(eng: GRFEngine, A_dev: DeviceCSR, pl: StepPlan) -> Front:
    """Laplacian -> fused walk/Phi (+ bucket counts) -> compaction -> [gather] -> banded transpose."""
    from .dist import gather_phi

    n, b, e = pl.n, pl.b, pl.e
    G = eng.laplacian(A_dev)
    if pl.mode == "cols":
        # the transpose of the block's rows alone (no count all-reduce, a 1/N-size transpose); the
        # walk counts its buckets when the block is all of the rank's rows
        fused = pl.kr_end == e and not SELF_COUNT_TRANSPOSE
        if PADDED_PHI and not pl.collective and b == 0 and not fused and not pl.cols_sym and SLOTS_DEFAULT:
            # one GPU: Phi stays the walk's padded rows (no compaction of all of Phi; the row shifts from one
            # pass over them); the block's rows [0, block_rows) compacted for their transpose
            rows = eng.walk_phi(G, pl.m, pl.p_halt, pl.L, pl.f, seed=pl.seed, src_begin=b, src_end=e, want64=False)
            head = PaddedRows(rows.cnt[:pl.block_rows], rows.idx, None, rows.val32, rows.cap, rows.n_cols)
            blk = eng.compact(head, want64=False, want32=True, sync_free=True)
            tr = eng.transpose_banded(blk, pl.band_width, nnz_bound=pl.block_rows * pl.rows_cap, slots=True)
            # (the padded Gram reads slot buckets; denser blocks take line buckets and the compacted Phi)
            phi = PaddedPhi(eng, rows) if tr.rec_unit == C.REC_SLOT else \
                eng.compact(rows, want64=False, want32=True, sync_free=True)
            return Front(phi, tr, phi, eng.phi_row_shifts(rows))
        tws = eng.transpose_workspace(pl.block_rows, n, pl.band_width) if fused else None
        local = eng.compact(eng.walk_phi(G, pl.m, pl.p_halt, pl.L, pl.f, seed=pl.seed, src_begin=b, src_end=e,
                                         count_ws=tws, band_width=pl.band_width if fused else 0, count_origin=b,
                                         want64=False),
                            want64=False, want32=True, sync_free=True, stats=COMPACT_STATS and not pl.collective)
        phi = gather_phi(eng, local, group=pl.group, shards=pl.shards, entries_bound=pl.gather_bound or None,
                         row_cap=pl.rows_cap, always=True) if pl.collective else local
        blk = local if fused else DeviceCSR(pl.block_rows, n, local.ptr[:pl.block_rows + 1], local.idx, None,
                                            local.val32)
        # (sparse buckets: the slot layout -- one line per small bucket in the Gram)
        tr = eng.transpose_banded(blk, pl.band_width, counted_ws=tws, nnz_bound=pl.block_rows * pl.rows_cap,
                                  slots=SLOTS_DEFAULT and tws is None)
        return Front(phi, tr, local, eng.phi_row_shifts(phi))
    return front_transpose(eng, pl, front_walk(eng, A_dev, pl, G))


def front_walk(eng: GRFEngine, A_dev: DeviceCSR, pl: StepPlan, G: Optional[DeviceCSR] = None) -> Front:
    """The first part of a row / symmetric-mode front: Laplacian -> fused walks -> compaction -> [gather]
    (``Front.tr`` is None until ``front_transpose``)."""
    from .dist import gather_phi

    n, b, e = pl.n, pl.b, pl.e
    G = eng.laplacian(A_dev) if G is None else G
    # (the transpose counts its own buckets unless GRF_TRANSPOSE_SELF=0: then the walk counts them)
    tws = None if SELF_COUNT_TRANSPOSE else eng.transpose_workspace(n, n, pl.band_width)
    local = eng.compact(eng.walk_phi(G, pl.m, pl.p_halt, pl.L, pl.f, seed=pl.seed, src_begin=b, src_end=e,
                                     count_ws=tws, band_width=pl.band_width if tws is not None else 0,
                                     want64=False),
                        want64=False, want32=True, sync_free=True)
    phi = gather_phi(eng, local, tws, group=pl.group, band_width=pl.band_width, shards=pl.shards,
                     entries_bound=pl.gather_bound or None, row_cap=pl.rows_cap, always=True) if pl.collective else local
    fr = Front(phi, None, local)
    fr.tws = tws
    return fr


def front_transpose(eng: GRFEngine, pl: StepPlan, fr: Front) -> Front:
    """The second part: the banded transpose of the (gathered) Phi, sized from bounds (n x the padded
    row capacity): no host round trip.  (No sub-band split: the symmetric diagonal tiles' skip saves
    records, not lines, and measured no faster: profiles/r03_split_ab.txt.)"""
    fr.tr = eng.transpose_banded(fr.phi, pl.band_width, counted_ws=getattr(fr, "tws", None),
                                 nnz_bound=pl.n * pl.rows_cap)
    # the whole-K tiles' pair-balanced wave shares (policy: engine.ROW_CUTS; the hub split makes its own
    # after dropping the hub columns)
    fr.cuts = eng.row_cuts(fr.phi, fr.tr, pl.skewed) if pl.mode == "sym" and pl.hubs == 0 else None
    return fr


def k_assembly(eng: GRFEngine, fr: Front, pl: StepPlan, K: torch.Tensor, *,
               after_tiles: Optional[Callable[[torch.cuda.Event], None]] = None, mirror_workgroups: int = 0,
               front_at: float = 1.0):
    """The K assembly of one step from its front.  Symmetric mode: ``after_tiles(event)`` is called
    between the Gram tiles and the mirror (the pipelined bench issues the next front there, beside
    the HBM-bound mirror; ``mirror_workgroups`` then bounds the mirror's grid, 1024 measured best);
    front_at < 1 issues it after that share of the tiles instead."""
    from .dist import allreduce_buckets

    if pl.mode == "cols":
        phi = fr.phi.rows if isinstance(fr.phi, PaddedPhi) else fr.phi
        eng.gram_sparse_cols(phi, fr.row_shift, fr.tr, out=K, sym_row0=pl.b if pl.cols_sym else None)
    elif pl.mode == "allreduce":
        eng.gram_sparse_kslice(fr.phi, fr.tr, pl.b, pl.e, out=K)  # all rows, inner slice [b, e)
        allreduce_buckets(K[:, :pl.n], group=pl.group)
    elif pl.mode == "sym" and pl.hubs > 0:
        eng.gram_sparse_sym_hubs(fr.phi, fr.tr, pl.hubs, out=K, mirror_workgroups=mirror_workgroups,
                                 after_tiles=after_tiles, skewed=pl.skewed,
                                 early_front=HUB_EARLY_FRONT or front_at < 1.0)
    elif pl.mode == "sym":
        main = torch.cuda.current_stream(eng.device)
        tiles_done = None
        if after_tiles is not None and front_at < 1.0:
            cut = int(round(front_at * 1000))
            eng.gram_sparse_upper(fr.phi, fr.tr, out=K, parts=(0, cut, 1000), cuts=getattr(fr, "cuts", None))
            tiles_done = torch.cuda.Event()
            tiles_done.record(main)
            eng.gram_sparse_upper(fr.phi, fr.tr, out=K, parts=(cut, 1000, 1000), cuts=getattr(fr, "cuts", None))
        else:
            eng.gram_sparse_upper(fr.phi, fr.tr, out=K, cuts=getattr(fr, "cuts", None))
            if after_tiles is not None:
                tiles_done = torch.cuda.Event()
                tiles_done.record(main)
        eng.gram_mirror(K, pl.n, mirror_workgroups)
        if after_tiles is not None:
            after_tiles(tiles_done)  # (issued after the mirror: the host's launch time does not delay it)
    else:
        eng.gram_sparse(fr.phi, fr.tr, pl.b, pl.kr_end, out=K)
    return K


def kernel_step(eng: GRFEngine, A_dev: DeviceCSR, pl: StepPlan, K: Optional[torch.Tensor] = None,
                mirror_workgroups: int = 0) -> Tuple[torch.Tensor, Front]:
    """One whole un-pipelined step (front + K assembly); returns (K buffer, front)."""
    K = alloc_k(eng, pl) if K is None else K
    fr = front(eng, A_dev, pl)
    k_assembly(eng, fr, pl, K, mirror_workgroups=mirror_workgroups)
    return K, fr


def k_view(K: torch.Tensor, pl: StepPlan) -> torch.Tensor:
    """The logical block of the K buffer: (rows x n) for row modes, (n x block_rows) for columns."""
    if pl.mode == "cols":
        return K[:, :pl.block_rows]
    return K[:, :pl.n]


def _abs_csr(A: DeviceCSR) -> DeviceCSR:
    return DeviceCSR(A.n_rows, A.n_cols, A.ptr, A.idx, None, A.val32.abs(), A._nnz)


def k_block_check(eng: GRFEngine, fr: Front, pl: StepPlan, K: torch.Tensor, seed: int = 7,
                  chunk: int = 2048) -> dict:
    """Size-independent check of this rank's K block against the Phi the step gathered (the bench's
    in-run parity, on the device; tests/test_gpu_headline.py's matvec checks).  With the block
    K_blk = Phi_A Phi_B^T (rows A, columns B of K) and random +-1 vectors u (over B) and v (over A):
        K_blk u   against  Phi_A (Phi_B^T u)      and      K_blk^T v  against  Phi_B (Phi_A^T v),
    both sides summed in fp64, each entry within the summed elementwise K tolerance
        3e-5 |Phi_A| (|Phi_B|^T |u|) + 1e-12 max|Phi| max_i max_k |Phi_ik| sum|u| + 1e-7 |want|.
    Returns {"max_ratio": max |got - want| / bound (<= 1 passes), ...}.  Reads K once (chunked)."""
    n = pl.n
    phi = phi_csr(fr.phi)
    if pl.mode == "cols":
        A_rows, B_rows = None, torch.arange(pl.b, pl.kr_end, device=eng.device)
        Kv = K[:, :pl.block_rows]                      # n x |B|
    elif pl.mode == "allreduce":
        A_rows, B_rows = None, None
        Kv = K[:, :n]
    else:  # sym (all rows) / rows (this rank's rows)
        A_rows = None if (pl.b, pl.kr_end) == (0, n) else torch.arange(pl.b, pl.kr_end, device=eng.device)
        B_rows = None
        Kv = K[:, :n][:pl.block_rows]
    gen = torch.Generator(device=eng.device).manual_seed(seed)
    u = (torch.randint(0, 2, (Kv.shape[1],), generator=gen, device=eng.device) * 2 - 1).to(torch.float64)
    v = (torch.randint(0, 2, (Kv.shape[0],), generator=gen, device=eng.device) * 2 - 1).to(torch.float64)
    Ku = torch.empty(Kv.shape[0], dtype=torch.float64, device=eng.device)
    Ktv = torch.zeros(Kv.shape[1], dtype=torch.float64, device=eng.device)
    for r0 in range(0, Kv.shape[0], chunk):
        blk = Kv[r0:r0 + chunk].double()
        Ku[r0:r0 + chunk] = blk @ u
        Ktv += blk.t() @ v[r0:r0 + chunk]
    aphi = _abs_csr(phi)

    def prod(P, rows_out, rows_in, w):
        """P[rows_out] (P[rows_in]^T w) in fp64 on the device (two CSR SpMMs)."""
        Pt = eng.csr_transpose(P, rows_in)
        return eng.spmm(P, eng.spmm(Pt, w[:, None].contiguous()), rows_out)[:, 0]

    amax = float(phi.val32[:phi.nnz].abs().max().item()) if phi.nnz else 0.0
    ratios = []
    for got, w, out_rows, in_rows in ((Ku, u, A_rows, B_rows), (Ktv, v, B_rows, A_rows)):
        want = prod(phi, out_rows, in_rows, w)
        bound = 3e-5 * prod(aphi, out_rows, in_rows, w.abs()) + 1e-12 * amax * amax * float(w.abs().sum()) \
            + 1e-7 * want.abs() + 1e-300
        ratios.append(float(((got - want).abs() / bound).max().item()))
    return {"max_ratio": max(ratios), "ok": max(ratios) <= 1.0,
            "checks": "K_blk u and K_blk^T v (fp64, random +-1 vectors) vs Phi_A (Phi_B^T u) and Phi_B (Phi_A^T v) "
                      "from this step's gathered Phi, elementwise-summed K tolerance"}
