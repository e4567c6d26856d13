"""Device-resident GRF pipeline on one MI355X: thin Python over the C ABI.

Every stage is one call into ``libgrf_amd.so`` on the current torch stream of
the engine's device; buffers are torch tensors (device memory plumbing only).
Nothing here computes on the host: the only host reads are sizes
(``DeviceCSR.nnz``) needed to allocate an output exactly.

Pipeline (re-designed for gfx950)::

    A (CSR) --laplacian--> L (CSR) --walk--> visit slots [n][L][m]
      --steps--> per-step rows (sampler API)   --phi--> Phi rows
      --phi_fused (m*L <= 4096)-----------------------> Phi rows
      --compact--> Phi CSR --transpose_banded--> Phi^T buckets --gram_sparse--> K (fp32)
                           --densify--> dense Phi --gram_dense (MFMA)-----------> K (fp32)
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib as C

DEFAULT_BAND_WIDTH = 4096  # transpose band = one Gram tile (32 KB int64 LDS accumulator per workgroup)
# row-mode Grams (row blocks: multi-GPU, K row ranges) are 6 % faster on 8192-wide bands with 8-wave
# tiles (C4: 25.9 vs 27.5 ms); the symmetric whole-K mode stays at 4096 (21.9 vs 22.7 ms: with 13
# bands the diagonal band tiles' lower halves cost more than the wider buckets save)
ROWS_BAND_WIDTH = 8192
# hub-column split: columns in at least this share of Phi's rows go to the dense MFMA panel (hub_count)
HUB_SHARE = 0.13
# ... and once a graph has such columns, with the split panel (bf16 products: 3/8 of the fp32 MFMA's cost per
# multiply-add) the columns down to this share as well: Enron 96 -> 192 columns, 7.52 -> 7.38 ms per K; 128 /
# 256 columns 7.47 / 7.50 (profiles/r05_hub_sweep_split.txt); Facebook's 20 columns above 0.13 stay unsplit
HUB_EXTEND_SHARE = 0.105
# gram(method="auto"): the dense MFMA path up to this many rows, the sparse path above
DENSE_GRAM_MAX_N = 4500  # measured crossover, profiles/r03_gram_crossover.txt (split Gram: r05_gram_crossover.txt)
# the banded transpose counts its buckets itself (grf_transpose_banded_self: no count atomics in the
# walk, no scan over every bucket); GRF_TRANSPOSE_SELF=0 restores the walk-counted plan (A/B)
SELF_COUNT_TRANSPOSE = os.environ.get("GRF_TRANSPOSE_SELF", "1") != "0"
# the whole-K Gram's waves take shares of about equal record pairs (grf_gram_row_cuts) instead of equal
# nonzero counts: "auto" (default) when Phi's column counts are skewed (column_stats), "1" always, "0" never
ROW_CUTS = os.environ.get("GRF_GRAM_CUTS", "auto")
# skewed: the densest column of Phi holds at least this many times the mean column's entries (C4's
# Erdos-Renyi Phi: ~1.2; Facebook / Enron: > 20)
SKEW_RATIO = 4.0


def _p(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


@dataclass
class DeviceCSR:
    """CSR matrix in device memory (int64 row pointers, int32 columns)."""

    n_rows: int
    n_cols: int
    ptr: torch.Tensor
    idx: torch.Tensor
    val: Optional[torch.Tensor] = None    # float64
    val32: Optional[torch.Tensor] = None  # float32
    _nnz: Optional[int] = None
    nnz_bound: Optional[int] = None  # an upper bound of nnz known without a host read (buffers sized by it)
    row_bound: Optional[int] = None  # an upper bound of the entries of any one row

    @property
    def nnz(self) -> int:
        if self._nnz is None:
            self._nnz = int(self.ptr[-1].item())
        return self._nnz

    # a row selection's entry buffers are sized by rows x row_bound only while that stays within this factor
    # of the matrix's own entries (repeats allowed) or ROWS_BOUND_FLOOR entries; past it (a hub row makes
    # row_bound ~ n_cols) the exact count is read back instead
    ROWS_BOUND_FACTOR = 4
    ROWS_BOUND_FLOOR = 1 << 22

    def rows_entry_bound(self, n_sel: int) -> Optional[int]:
        """An upper bound of the entries of n_sel selected rows that is known without a host read and
        not wasteful (None: count them exactly)."""
        if self.row_bound is None:
            return None
        bound = n_sel * self.row_bound
        total = self.nnz_or_bound() if (self._nnz is not None or self.nnz_bound is not None) else None
        if total is None:
            return None
        reps = -(-max(n_sel, 1) // max(self.n_rows, 1))  # (a selection longer than the matrix repeats rows)
        return bound if bound <= max(self.ROWS_BOUND_FACTOR * reps * total, self.ROWS_BOUND_FLOOR) else None

    def nnz_or_bound(self) -> int:
        """nnz when it is known on the host, else the bound (no device->host read), else nnz (read)."""
        if self._nnz is not None:
            return self._nnz
        return self.nnz_bound if self.nnz_bound is not None else self.nnz

    @classmethod
    def from_scipy(cls, A, device) -> "DeviceCSR":
        A = sp.csr_matrix(A)
        if A.shape[0] > 0x7FFFFFFF or A.shape[1] > 0x7FFFFFFF:
            raise ValueError("graphs with more than 2^31-1 nodes are not supported")
        ptr = torch.from_numpy(np.asarray(A.indptr, dtype=np.int64)).to(device)
        idx = torch.from_numpy(np.asarray(A.indices, dtype=np.int32)).to(device)
        val = torch.from_numpy(np.asarray(A.data, dtype=np.float64)).to(device)
        return cls(A.shape[0], A.shape[1], ptr, idx, val, None, int(A.nnz))

    def to_scipy(self) -> sp.csr_matrix:
        nnz = self.nnz
        ptr = self.ptr.cpu().numpy()
        idx = self.idx[:nnz].cpu().numpy()
        val = (self.val if self.val is not None else self.val32)[:nnz].cpu().numpy()
        if ptr[-1] <= np.iinfo(np.int32).max:
            ptr = ptr.astype(np.int32)
        return sp.csr_matrix((val, idx, ptr), shape=(self.n_rows, self.n_cols))


@dataclass
class Slots:
    node: torch.Tensor  # int32 [n_src, L, m], -1 = no visit
    load: torch.Tensor  # float64 [n_src, L, m]
    src_begin: int
    n: int              # nodes of the graph (columns)

    @property
    def n_src(self):
        return self.node.shape[0]

    @property
    def L(self):
        return self.node.shape[1]

    @property
    def m(self):
        return self.node.shape[2]


@dataclass
class StepRows:
    cnt: torch.Tensor  # int32 [n_src * L]
    idx: torch.Tensor  # int32 [n_src * L * m]
    val: torch.Tensor  # float64 [n_src * L * m]
    n_src: int
    L: int
    m: int
    n: int


@dataclass
class PaddedRows:
    cnt: torch.Tensor             # int32 [n_rows]
    idx: torch.Tensor             # int32 [n_rows * cap]
    val: torch.Tensor             # float64 [n_rows * cap]
    val32: Optional[torch.Tensor]  # float32 [n_rows * cap]
    cap: int
    n_cols: int

    @property
    def n_rows(self):
        return self.cnt.shape[0]


@dataclass
class Banded:
    t_desc: torch.Tensor  # int32 [2 * (n_bands * n_cols + 1)]: per bucket {first unit, pairs}
    t_rec: torch.Tensor   # uint8 [units * rec_unit]: 12-byte record pairs {u16 j0 | u16 j1, f32 v0, f32 v1}
    t_maxabs: torch.Tensor  # float32 [1], max |Phi|
    t_rowshift: torch.Tensor  # int32 [n_rows], Gram fixed-point scale exponent per row
    band_width: int
    n_rows: int
    n_cols: int
    rec_unit: int = C.REC_LINE  # bucket alignment: 128-byte lines or packed 12-byte pairs
    # per bucket 8 uint16 entry offsets of its sub-bands (buckets laid out by sub-band; the symmetric
    # Gram's diagonal tiles start there), or None (records in arbitrary order within a bucket)
    t_split: Optional[torch.Tensor] = None


def cols_band_width(rows: int, max_width: int = ROWS_BAND_WIDTH) -> int:
    """Band width of a rank's own-rows transpose (column-block Gram): the rows in the fewest bands
    of at most ``max_width``, split evenly and rounded up to a multiple of 64."""
    nb = max(1, -(-rows // max_width))
    return max(64, -(-(-(-rows // nb)) // 64) * 64)


def choose_rec_unit(nnz: int, n_rows: int, n_cols: int, band_width: int) -> int:
    """Line-aligned buckets when a bucket averages >= 8 entries (C4: ~18 at W = 4096), packed
    pairs below that (C5: ~1.4 at W = 8192, where a 128-byte line per bucket would be ~15x
    the records' bytes)."""
    per_bucket = nnz / max(1, n_rows) * band_width / max(1, n_cols)
    return C.REC_LINE if per_bucket >= 8.0 else C.REC_PACKED


class DensePlanes:
    """The dense Phi as the split Gram's three bf16 planes (include/grf.h grf_split_planes): ``P`` uint8
    [n x row bytes] on the device, ``n`` rows, ``k_dim`` columns."""

    def __init__(self, P: torch.Tensor, n: int, k_dim: int):
        self.P, self.n, self.k_dim = P, int(n), int(k_dim)

    @property
    def shape(self):
        return (self.n, self.k_dim)

    def record_stream(self, stream):
        self.P.record_stream(stream)


class GRFEngine:
    """All device work for one GPU.  ``device`` is a torch device (``cuda:N``)."""

    def __init__(self, device=None):
        if not torch.cuda.is_available():
            raise RuntimeError("grf_amd needs a ROCm GPU (MI355X / gfx950); none is visible")
        self.lib = C.load()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        C.check(self.lib.grf_set_device(self.device.index), "grf_set_device")
        # the Gram kernels' tile work counter (calls on this engine's stream are ordered)
        self._gram_ws = self._ws(self.lib.grf_gram_workspace_bytes())
        # the dense Gram's arithmetic (gram_dense): the exact three-plane bf16 'split' on the bf16 matrix
        # cores (fp32-class error, 1.3-1.4x faster: profiles/r05_split_gram_error.txt, AB_LOG "split Gram") or
        # the 'fp32' matrix instruction
        self.dense_precision = os.environ.get("GRF_GRAM_DENSE_PRECISION", "split")
        if self.dense_precision not in ("split", "fp32"):
            raise ValueError(f"GRF_GRAM_DENSE_PRECISION must be 'split' or 'fp32', got {self.dense_precision!r}")

    # ------------------------------------------------------------ utilities
    @property
    def stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _empty(self, n, dtype):
        return torch.empty(int(max(n, 0)), dtype=dtype, device=self.device)

    def _ws(self, nbytes: int) -> torch.Tensor:
        return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.device)

    def _set_device(self):
        C.check(self.lib.grf_set_device(self.device.index), "grf_set_device")

    def to_device(self, A) -> DeviceCSR:
        return A if isinstance(A, DeviceCSR) else DeviceCSR.from_scipy(A, self.device)

    # ----------------------------------------------------------- Laplacians
    def laplacian(self, A) -> DeviceCSR:
        """scipy-semantics normalised Laplacian (utils_sparse/graph_utils.py:5-30)."""
        A = self.to_device(A)
        if A.n_rows != A.n_cols:
            raise ValueError("Adjacency matrix must be square.")
        n = A.n_rows
        cap = A.nnz + n
        lp, li, lv = self._empty(n + 1, torch.int64), self._empty(cap, torch.int32), self._empty(cap, torch.float64)
        deg, dinv = self._empty(n, torch.float64), self._empty(n, torch.float64)
        ws = self._ws(self.lib.grf_laplacian_csr_workspace_bytes(n))
        C.check(self.lib.grf_laplacian_csr(n, _p(A.ptr), _p(A.idx), _p(A.val), C.LAP_SCIPY, _p(lp), _p(li), _p(lv),
                                           cap, _p(deg), _p(dinv), _p(ws), ws.numel(), self.stream),
                "grf_laplacian_csr")
        G = DeviceCSR(n, n, lp, li, lv)
        G.nnz_bound = cap  # (sizes the augmented walk matrix without reading nnz back)
        return G

    def walk_matrix_dense(self, W, mode: int, nnz_w: Optional[int] = None) -> DeviceCSR:
        """Dense-input walk matrix (numpy Laplacian variants or the matrix itself) as CSR.

        Its capacity (and the augmented walk matrix sized from it, cached on the result) is nnz(W) + n
        (the Laplacian adds at most the diagonal).  nnz(W) is counted on the host for a host W, taken
        from ``nnz_w`` when the caller knows it (the bench counts its resident W once, at setup), else
        bounded by n^2 while that is small (<= 2^26 entries: 0.8 GB of CSR) or counted on the device
        (a torch reduction and a host round trip: 0.64 ms of C2's front, profiles/r05_c2_kernel_alone.txt)."""
        host = not torch.is_tensor(W)
        Wn = np.ascontiguousarray(W, dtype=np.float64) if host else None
        Wt = torch.as_tensor(Wn) if host else W
        Wt = Wt.to(self.device, torch.float64).contiguous()
        n = Wt.shape[0]
        if Wt.dim() != 2 or Wt.shape[1] != n:
            raise ValueError("Adjacency matrix must be square.")
        if nnz_w is not None:
            cap = min(int(nnz_w) + n, n * n)
        elif host:
            cap = int(np.count_nonzero(Wn)) + n
        elif n * n <= (1 << 26):
            cap = n * n
        else:
            cap = int(torch.count_nonzero(Wt).item()) + n
        cap = max(cap, 1)
        lp, li, lv = self._empty(n + 1, torch.int64), self._empty(cap, torch.int32), self._empty(cap, torch.float64)
        deg = self._empty(n, torch.float64)
        ws = self._ws(self.lib.grf_laplacian_dense_workspace_bytes(n))
        C.check(self.lib.grf_laplacian_dense(n, _p(Wt), mode, _p(lp), _p(li), _p(lv), cap, _p(deg), _p(ws),
                                             ws.numel(), self.stream), "grf_laplacian_dense")
        G = DeviceCSR(n, n, lp, li, lv)
        G.nnz_bound = cap
        return G

    # ---------------------------------------------------------------- walks
    def walk(self, G: DeviceCSR, walks_per_node: int, p_halt: float, max_walk_length: int, *, rng: int = C.RNG_PHILOX,
             seed: int = 42, n_chunks: int = 1, load_rule: int = C.LOAD_CUMULATIVE, src_begin: int = 0,
             src_end: Optional[int] = None, use_aug: bool = True) -> Slots:
        """Visit slots of the walks from sources [src_begin, src_end).  use_aug: step through the
        augmented walk matrix (one dependent round trip per step; the same slots bit for bit)."""
        n = G.n_rows
        src_end = n if src_end is None else src_end
        m, L = int(walks_per_node), int(max_walk_length)
        if m < 1 or L < 1:
            raise ValueError("walks_per_node and max_walk_length must be >= 1")
        ns = src_end - src_begin
        node = torch.empty((ns, L, m), dtype=torch.int32, device=self.device)
        load = torch.empty((ns, L, m), dtype=torch.float64, device=self.device)
        prm = C.GrfWalkParams(m, float(p_halt), L, int(load_rule), int(rng), 0, int(n_chunks),
                              int(seed) & 0xFFFFFFFFFFFFFFFF)
        aug = self.walk_aug(G) if use_aug else None
        C.check(self.lib.grf_walk_ex(n, _p(G.ptr), _p(G.idx), _p(G.val), _p(aug), ctypes.byref(prm), src_begin,
                                     src_end, _p(node), _p(load), self.stream), "grf_walk_ex")
        return Slots(node, load, src_begin, n)

    def chunk_bounds(self, n: int, n_chunks: int) -> list[int]:
        return [int(self.lib.grf_chunk_bounds(n, n_chunks, c)) for c in range(n_chunks)] + [n]

    # ----------------------------------------------------- steps / features
    def steps(self, slots: Slots, norm: int = C.NORM_MUL_RECIP) -> StepRows:
        ns, L, m = slots.n_src, slots.L, slots.m
        cnt = self._empty(ns * L, torch.int32)
        idx = self._empty(ns * L * m, torch.int32)
        val = self._empty(ns * L * m, torch.float64)
        C.check(self.lib.grf_steps(ns, m, L, norm, _p(slots.node), _p(slots.load), _p(cnt), _p(idx), _p(val),
                                   self.stream), "grf_steps")
        return StepRows(cnt, idx, val, ns, L, m, slots.n)

    def _f(self, f) -> torch.Tensor:
        """The modulator on the device.  Host values are uploaded once per distinct vector (a pageable
        host-to-device copy per call stalled the issuing thread ~0.2 ms inside every pipelined step)."""
        if torch.is_tensor(f):
            return f.to(self.device, torch.float64).reshape(-1)
        host = np.asarray(f, dtype=np.float64).reshape(-1)
        key = host.tobytes()
        cache = self.__dict__.setdefault("_f_cache", {})
        t = cache.get(key)
        if t is None:
            if len(cache) > 64:
                cache.clear()
            t = cache[key] = torch.from_numpy(host.copy()).to(self.device)
        return t

    def phi(self, st: StepRows, f, want32: bool = True) -> PaddedRows:
        ft = self._f(f)
        cap = max(1, min(st.m * st.L, st.n))
        cnt = self._empty(st.n_src, torch.int32)
        idx = self._empty(st.n_src * cap, torch.int32)
        val = self._empty(st.n_src * cap, torch.float64)
        v32 = self._empty(st.n_src * cap, torch.float32) if want32 else None
        C.check(self.lib.grf_phi(st.n_src, st.m, st.L, _p(st.cnt), _p(st.idx), _p(st.val), _p(ft), ft.numel(), cap,
                                 _p(cnt), _p(idx), _p(val), _p(v32), self.stream), "grf_phi")
        return PaddedRows(cnt, idx, val, v32, cap, st.n)

    def phi_fused(self, slots: Slots, f, norm: int = C.NORM_MUL_RECIP, want32: bool = True) -> PaddedRows:
        ft = self._f(f)
        ns, L, m = slots.n_src, slots.L, slots.m
        cap = max(1, min(m * L, slots.n))
        cnt = self._empty(ns, torch.int32)
        idx = self._empty(ns * cap, torch.int32)
        val = self._empty(ns * cap, torch.float64)
        v32 = self._empty(ns * cap, torch.float32) if want32 else None
        C.check(self.lib.grf_phi_fused(ns, m, L, norm, _p(slots.node), _p(slots.load), _p(ft), ft.numel(), cap,
                                       _p(cnt), _p(idx), _p(val), _p(v32), self.stream), "grf_phi_fused")
        return PaddedRows(cnt, idx, val, v32, cap, slots.n)

    def walk_phi(self, G: DeviceCSR, walks_per_node: int, p_halt: float, max_walk_length: int, f, *,
                 seed: int = 42, load_rule: int = C.LOAD_CUMULATIVE, norm: int = C.NORM_MUL_RECIP,
                 src_begin: int = 0, src_end: Optional[int] = None, want32: bool = True,
                 count_ws: Optional[torch.Tensor] = None, band_width: int = 0, use_aug: bool = True,
                 count_origin: int = 0, want64: bool = True) -> PaddedRows:
        """Philox walks straight to Phi rows (one kernel; identical to walk + features).

        count_ws: a zeroed transpose workspace (``transpose_workspace``) in which the kernel also
        counts the banded transpose's buckets, for ``transpose_banded(..., counted_ws=...)``;
        count_origin: the transposed matrix's first row (0: all of Phi; src_begin: these rows alone)."""
        n = G.n_rows
        src_end = n if src_end is None else src_end
        m, L = int(walks_per_node), int(max_walk_length)
        if m < 1 or L < 1:
            raise ValueError("walks_per_node and max_walk_length must be >= 1")
        ft = self._f(f)
        ns = src_end - src_begin
        cap = max(1, min(m * L, n))
        cnt = self._empty(ns, torch.int32)
        idx = self._empty(ns * cap, torch.int32)
        if not (want64 or want32):
            raise ValueError("walk_phi: want64 or want32")
        val = self._empty(ns * cap, torch.float64) if want64 else None  # (want64=False: f32 values only)
        v32 = self._empty(ns * cap, torch.float32) if want32 else None
        prm = C.GrfWalkParams(m, float(p_halt), L, int(load_rule), C.RNG_PHILOX, 0, 1, int(seed) & 0xFFFFFFFFFFFFFFFF)
        aug = self.walk_aug(G) if use_aug else None
        C.check(self.lib.grf_walk_phi(n, _p(G.ptr), _p(G.idx), _p(G.val), _p(aug), ctypes.byref(prm), src_begin,
                                      src_end,
                                      norm, _p(ft), ft.numel(), cap, _p(cnt), _p(idx), _p(val), _p(v32),
                                      _p(count_ws), int(band_width), int(count_origin), self.stream),
                "grf_walk_phi")
        return PaddedRows(cnt, idx, val, v32, cap, n)

    def walk_aug(self, G: DeviceCSR) -> Optional[torch.Tensor]:
        """The augmented walk matrix of G (grf_walk_aug), built once per DeviceCSR; None when
        nnz >= 2^32 (the walk then reads the row bounds per step)."""
        aug = getattr(G, "_aug", None)
        if aug is not None:
            return aug
        nnz = G.nnz_bound if getattr(G, "nnz_bound", None) is not None else G.nnz
        if nnz >= 2 ** 32:
            return None
        aug = torch.empty(max(int(self.lib.grf_walk_aug_bytes(nnz)), 32), dtype=torch.uint8, device=self.device)
        C.check(self.lib.grf_walk_aug(G.n_rows, _p(G.ptr), _p(G.idx), _p(G.val), _p(aug), self.stream), "grf_walk_aug")
        G._aug = aug
        return aug

    def features(self, slots: Slots, f, norm: int = C.NORM_MUL_RECIP) -> PaddedRows:
        """Phi rows; the fused kernel when m*L fits LDS, else steps + merge (bit-identical)."""
        if slots.m * slots.L <= 4096:
            return self.phi_fused(slots, f, norm)
        return self.phi(self.steps(slots, norm), f)

    # ------------------------------------------------------ sparse utilities
    def compact(self, rows: PaddedRows, want64: bool = True, want32: bool = True,
                sync_free: bool = False, stats: bool = False) -> DeviceCSR:
        """Compact CSR of padded rows.  sync_free: size the outputs by the padded capacity instead of
        reading nnz back (no host synchronisation; nnz is read lazily if asked for).  stats: also keep
        the rows' Gram shift statistics (``phi_row_shifts`` then skips its pass over the values)."""
        n = rows.n_rows
        ptr = self._empty(n + 1, torch.int64)
        ws = self._ws(self.lib.grf_scan_workspace_bytes(n))
        C.check(self.lib.grf_scan_counts(n, _p(rows.cnt), _p(ptr), _p(ws), ws.numel(), self.stream),
                "grf_scan_counts")
        nnz = n * rows.cap if sync_free else int(ptr[-1].item())
        idx = self._empty(nnz, torch.int32)
        v64 = self._empty(nnz, torch.float64) if want64 else None
        v32 = self._empty(nnz, torch.float32) if (want32 and rows.val32 is not None) else None
        st = None
        if stats and v32 is not None:
            st = torch.empty(int(self.lib.grf_phi_row_shifts_workspace_bytes(n)), dtype=torch.uint8,
                             device=self.device)
            C.check(self.lib.grf_compact_rows_stats(n, rows.cap, _p(rows.cnt), _p(ptr), _p(rows.idx),
                                                    _p(rows.val if want64 else None), _p(rows.val32), _p(idx),
                                                    _p(v64), _p(v32), _p(st), st.numel(), self.stream),
                    "grf_compact_rows_stats")
        else:
            C.check(self.lib.grf_compact_rows(n, rows.cap, _p(rows.cnt), _p(ptr), _p(rows.idx),
                                              _p(rows.val if want64 else None),
                                              _p(rows.val32 if v32 is not None else None), _p(idx), _p(v64),
                                              _p(v32), self.stream), "grf_compact_rows")
        out = DeviceCSR(n, rows.n_cols, ptr, idx, v64, v32, None if sync_free else nnz)
        out.row_stats = st
        out.nnz_bound = nnz
        return out

    def dense_to_scipy_csr(self, K: torch.Tensor):
        """K (dense fp32, on the device) as the scipy CSR the reference's sparse entry point returns
        (``Phi @ Phi.T``: float64 values, sorted int32 columns, exact zeros absent), built on the device
        (``grf_dense_to_csr_count`` / ``_fill``) and copied to the host once: indptr, indices, data."""
        import scipy.sparse as sp
        n_rows, n_cols = K.shape
        if K.dtype != torch.float32 or K.device != self.device or K.stride(1) != 1:
            raise ValueError("dense_to_scipy_csr: K must be a row-major float32 tensor on the engine's device")
        cnt = self._empty(n_rows, torch.int32)
        C.check(self.lib.grf_dense_to_csr_count(n_rows, n_cols, _p(K), K.stride(0), _p(cnt), self.stream),
                "grf_dense_to_csr_count")
        ptr = self._empty(n_rows + 1, torch.int64)
        ws = self._ws(self.lib.grf_scan_workspace_bytes(n_rows))
        C.check(self.lib.grf_scan_counts(n_rows, _p(cnt), _p(ptr), _p(ws), ws.numel(), self.stream),
                "grf_scan_counts")
        nnz = int(ptr[-1].item())
        idx, val = self._empty(nnz, torch.int32), self._empty(nnz, torch.float64)
        if nnz:
            C.check(self.lib.grf_dense_to_csr_fill(n_rows, n_cols, _p(K), K.stride(0), _p(ptr), _p(idx), _p(val),
                                                   self.stream), "grf_dense_to_csr_fill")
        out = sp.csr_matrix((val.cpu().numpy(), idx.cpu().numpy(), ptr.cpu().numpy()), shape=(n_rows, n_cols),
                            copy=False)
        out.has_sorted_indices = True  # (columns ascending within every row by construction)
        return out

    def step_matrices(self, st: StepRows) -> list[DeviceCSR]:
        """Per-step CSR matrices (rows = the sources of this step block)."""
        out = []
        cnt2 = st.cnt.view(st.n_src, st.L)
        for l in range(st.L):
            rows = PaddedRows(cnt2[:, l].contiguous(), st.idx[l * st.m:], st.val[l * st.m:], None, st.L * st.m, st.n)
            out.append(self.compact(rows, want64=True, want32=False))
        return out

    def steps_dense(self, st: StepRows, n_cols: Optional[int] = None) -> torch.Tensor:
        n_cols = st.n if n_cols is None else n_cols
        out = torch.zeros((st.n_src, n_cols, st.L), dtype=torch.float64, device=self.device)
        C.check(self.lib.grf_steps_densify(st.n_src, st.m, st.L, n_cols, _p(st.cnt), _p(st.idx), _p(st.val), _p(out),
                                           self.stream), "grf_steps_densify")
        return out

    def transpose_workspace(self, n_rows: int, n_cols: int, band_width: int = DEFAULT_BAND_WIDTH) -> torch.Tensor:
        """Zeroed workspace of ``transpose_banded`` (its first n_bands * n_cols int32 are bucket counts)."""
        nbk = -(-n_rows // band_width) * n_cols
        ws = self._ws(self.lib.grf_transpose_workspace_bytes(nbk))
        ws.zero_()
        return ws

    def transpose_banded(self, phi: DeviceCSR, band_width: int = DEFAULT_BAND_WIDTH,
                         counted_ws: Optional[torch.Tensor] = None, staged: Optional[bool] = None,
                         nnz_bound: Optional[int] = None, rec_unit: Optional[int] = None,
                         self_count: Optional[bool] = None, split: bool = False, slots: bool = False) -> Banded:
        """Banded transpose of Phi.  counted_ws: workspace whose bucket counts ``walk_phi`` filled.
        staged: two-pass binned fill (default when band_width % 64 == 0) or the atomic fill.
        self_count: the staged fill without a plan (grf_transpose_banded_self; default unless
        counted_ws is given or GRF_TRANSPOSE_SELF=0): buckets in per-region slabs.
        nnz_bound: an upper bound of nnz(Phi) (e.g. ``compact(..., sync_free=True)``'s): the record
        buffer is then sized from bounds and no size is read back (no host synchronisation).
        split: (self-count transpose) lay every bucket out by sub-band and return the offsets
        (``Banded.t_split``) for the symmetric Gram's diagonal-tile skip -- measured no faster (a skip
        saves records inside lines the tile fetches anyway: profiles/r03_split_ab.txt), so off by default.
        slots: (self-count transpose) where the buckets are sparse enough for packed pairs and the bands
        wider than 4096 (8-wave Gram tiles), the GRF_REC_SLOT layout instead: each bucket's header and
        first two pairs in one 32-byte slot, so the Gram reads a small bucket with one line (the column
        blocks over power-law graphs, C5).  Not for the hub-column split (which edits descriptors)."""
        n_rows, n_cols = phi.n_rows, phi.n_cols
        nb = -(-n_rows // band_width)
        nbk = nb * n_cols
        t_desc = self._empty(2 * (nbk + 1), torch.int32)
        t_max = self._empty(1, torch.float32)
        t_shift = self._empty(max(n_rows, 1), torch.int32)
        if staged is None:
            staged = band_width % 64 == 0 and os.environ.get("GRF_TRANSPOSE_STAGED", "1") != "0"
        if self_count is None:
            self_count = SELF_COUNT_TRANSPOSE and counted_ws is None and staged
        if self_count:
            if counted_ws is not None or not staged:
                raise ValueError("self_count: the staged transpose counts its own buckets (no counted_ws)")
            if slots and not split and rec_unit is None and band_width > 4096:
                u0 = choose_rec_unit(phi.nnz if phi._nnz is not None or nnz_bound is None else nnz_bound,
                                     n_rows, n_cols, band_width)
                rec_unit = C.REC_SLOT if u0 == C.REC_PACKED else u0
            return self._transpose_self(phi, band_width, nnz_bound, rec_unit, t_desc, t_max, t_shift, split)
        ws = counted_ws if counted_ws is not None else self._ws(self.lib.grf_transpose_workspace_bytes(nbk))
        if rec_unit is None:
            rec_unit = choose_rec_unit(phi.nnz if phi._nnz is not None or nnz_bound is None else nnz_bound,
                                       n_rows, n_cols, band_width)
        u = int(rec_unit)
        C.check(self.lib.grf_transpose_banded_plan(n_rows, n_cols, band_width, u, _p(phi.ptr), _p(phi.idx),
                                                   _p(t_desc), int(counted_ws is not None), _p(ws), ws.numel(),
                                                   self.stream), "grf_transpose_banded_plan")
        # the Gram kernel addresses a band's records with 32-bit byte offsets.  A bucket of c entries
        # takes ceil(12 ceil(c / 2) / u) units: lines (u = 128) <= 0.047 c + 1.1, pairs (u = 12)
        # <= c, so a band of rows with at most `row_cap` entries each holds < 6 bw row_cap +
        # 141 n_cols bytes (lines) or 12 bw row_cap bytes (pairs).
        row_cap = min(n_cols, max(1, -(-(nnz_bound or 0) // max(n_rows, 1)))) if nnz_bound is not None else None
        band_bytes = (None if row_cap is None else
                      6 * band_width * row_cap + 141 * n_cols if u == C.REC_LINE else 12 * band_width * row_cap)
        if nnz_bound is not None and nb and band_bytes < 2 ** 31:
            # bound: no read-back
            units = int(0.047 * nnz_bound + 1.1 * nbk) + 1 if u == C.REC_LINE else int(nnz_bound) + 1
        else:
            # band starts (first unit of bucket (band, 0)) and the total, read back
            starts = torch.cat([t_desc[0:2 * nbk:2 * n_cols], t_desc[2 * nbk:2 * nbk + 1]]).cpu().numpy()
            starts = starts.view(np.uint32).astype(np.int64)
            tail = t_desc[2 * nbk:].cpu().numpy().view(np.uint32).astype(np.int64)
            units = int(tail[0] + (tail[1] << 32))
            starts[-1] = units
            if nb and int(np.diff(starts).max(initial=0)) * u >= 2 ** 31:
                raise NotImplementedError("a transpose band holds >= 2 GiB of records; use a smaller band_width")
        # (+128 B: a masked Gram lane reads the first pair of an empty last band)
        t_rec = self._empty(max(units, 1) * u + 128, torch.uint8)  # torch allocations are 256-B aligned
        if staged:
            nnz = nnz_bound if nnz_bound is not None else phi.nnz
            sg = self._ws(self.lib.grf_transpose_staging_bytes(n_rows, n_cols, band_width, nnz))
            C.check(self.lib.grf_transpose_banded_fill_staged(
                n_rows, n_cols, band_width, u, _p(phi.ptr), _p(phi.idx), _p(phi.val32), _p(t_desc), _p(t_rec),
                t_rec.numel(), _p(t_max), _p(t_shift), _p(ws), ws.numel(), nnz, _p(sg), sg.numel(), self.stream),
                "grf_transpose_banded_fill_staged")
        else:
            C.check(self.lib.grf_transpose_banded_fill(n_rows, n_cols, band_width, u, _p(phi.ptr), _p(phi.idx),
                                                       _p(phi.val32), _p(t_desc), _p(t_rec), t_rec.numel(),
                                                       _p(t_max), _p(t_shift), _p(ws), ws.numel(), self.stream),
                    "grf_transpose_banded_fill")
        return Banded(t_desc, t_rec, t_max, t_shift, band_width, n_rows, n_cols, u)

    def _transpose_self(self, phi: DeviceCSR, band_width: int, nnz_bound: Optional[int], rec_unit: Optional[int],
                        t_desc, t_max, t_shift, split: bool = False) -> Banded:
        """The plan-free staged transpose (grf_transpose_banded_self): buckets counted by the placing
        workgroups themselves, no counts from the walk and no scan over every bucket."""
        n_rows, n_cols = phi.n_rows, phi.n_cols
        nnz = int(nnz_bound) if nnz_bound is not None else phi.nnz
        if rec_unit is None:
            rec_unit = choose_rec_unit(phi.nnz if phi._nnz is not None or nnz_bound is None else nnz_bound,
                                       n_rows, n_cols, band_width)
        u = int(rec_unit)
        # the Gram addresses a band's records with 32-bit byte offsets: bound one band's slabs
        row_cap = min(n_cols, max(1, -(-nnz // max(n_rows, 1))))
        band_units = self.lib.grf_transpose_self_units_bound(min(band_width, n_rows), n_cols, band_width, u,
                                                             min(nnz, band_width * row_cap))
        if n_rows and band_units * u >= 2 ** 31:
            raise NotImplementedError("a transpose band holds >= 2 GiB of records; use a smaller band_width")
        units = self.lib.grf_transpose_self_units_bound(n_rows, n_cols, band_width, u, nnz)
        if u == C.REC_SLOT and units * u >= 2 ** 30:
            # (slot offsets are counted from the first slot of all bands: fall back to packed pairs)
            return self._transpose_self(phi, band_width, nnz_bound, C.REC_PACKED, t_desc, t_max, t_shift, split)
        t_rec = self._empty(max(units, 1) * u + 128, torch.uint8)
        ws = self._ws(self.lib.grf_transpose_self_workspace_bytes(n_rows, n_cols, band_width))
        sg = self._ws(self.lib.grf_transpose_staging_bytes(n_rows, n_cols, band_width, nnz))
        nbk = -(-n_rows // band_width) * n_cols
        t_split = self._empty(8 * nbk, torch.int16) if split and band_width <= 8192 else None
        C.check(self.lib.grf_transpose_banded_self(n_rows, n_cols, band_width, u, _p(phi.ptr), _p(phi.idx),
                                                   _p(phi.val32), _p(t_desc), _p(t_split), _p(t_rec), t_rec.numel(),
                                                   _p(t_max), _p(t_shift), _p(ws), ws.numel(), nnz, _p(sg),
                                                   sg.numel(), self.stream), "grf_transpose_banded_self")
        return Banded(t_desc, t_rec, t_max, t_shift, band_width, n_rows, n_cols, u, t_split)

    # ----------------------------------------------------------------- Gram
    @staticmethod
    def leading_dim(n: int) -> int:
        return max(64, -(-n // 64) * 64)

    def gram_sparse(self, phi: DeviceCSR, tr: Banded, row_begin: int = 0, row_end: Optional[int] = None,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """K[row_begin:row_end, :] (float32) with leading dimension padded to 64."""
        n = tr.n_rows
        row_end = n if row_end is None else row_end
        ldk = self.leading_dim(n)
        if out is None:
            out = torch.empty((row_end - row_begin, ldk), dtype=torch.float32, device=self.device)
        C.check(self.lib.grf_gram_sparse(n, row_begin, row_end, _p(phi.ptr), _p(phi.idx), _p(phi.val32),
                                         tr.band_width, tr.rec_unit, _p(tr.t_desc), _p(tr.t_rec),
                                         _p(tr.t_rowshift), _p(out),
                                         out.stride(0), _p(self._gram_ws), self._gram_ws.numel(), self.stream),
                "grf_gram_sparse")
        return out[:, :n]

    def phi_row_shifts(self, phi: DeviceCSR) -> torch.Tensor:
        """The Gram fixed-point shifts of every row of Phi (int32 [n_rows]; grf_phi_row_shifts): the
        same values as ``transpose_banded(phi).t_rowshift``, for rows that are not in the transpose."""
        n = phi.n_rows
        shift = self._empty(max(n, 1), torch.int32)
        mx = self._empty(1, torch.float32)
        if isinstance(phi, PaddedRows):  # (the walk's rows, not compacted: grf_phi_row_shifts_padded)
            if phi.val32 is None:
                raise ValueError("phi_row_shifts: padded rows need their float32 values")
            ws = self._ws(self.lib.grf_phi_row_shifts_workspace_bytes(n))
            C.check(self.lib.grf_phi_row_shifts_padded(n, phi.cap, _p(phi.cnt), _p(phi.val32), _p(mx), _p(shift),
                                                       _p(ws), ws.numel(), self.stream), "grf_phi_row_shifts_padded")
            return shift
        st = getattr(phi, "row_stats", None)
        if st is not None:  # (left by compact(..., stats=True): same bits, no pass over the values)
            C.check(self.lib.grf_phi_row_shifts_stats(n, _p(st), _p(mx), _p(shift), self.stream),
                    "grf_phi_row_shifts_stats")
            return shift
        ws = self._ws(self.lib.grf_phi_row_shifts_workspace_bytes(n))
        C.check(self.lib.grf_phi_row_shifts(n, _p(phi.ptr), _p(phi.val32), _p(mx), _p(shift), _p(ws), ws.numel(),
                                            self.stream), "grf_phi_row_shifts")
        return shift

    def gram_sparse_cols(self, phi: DeviceCSR, row_shift: torch.Tensor, tr_b: Banded, row_begin: int = 0,
                         row_end: Optional[int] = None, out: Optional[torch.Tensor] = None,
                         sym_row0: Optional[int] = None) -> torch.Tensor:
        """Column block K[row_begin:row_end, B] = Phi[rows] Phi_B^T (float32) from the banded transpose
        ``tr_b`` of another row set Phi_B (grf_gram_sparse_cols); row_shift = ``phi_row_shifts(phi)``.
        With Phi_B = Phi[b:e] this is K[:, b:e], bit-identical to ``gram_sparse(...)[:, b:e]``;
        sym_row0 = b says so, and the square K[b:e, b:e] is then computed on and above its diagonal
        and mirrored (the symmetric mode's bits there)."""
        n = phi.n_rows
        row_end = n if row_end is None else row_end
        t_rows = tr_b.n_rows
        if out is None:
            out = torch.empty((row_end - row_begin, self.leading_dim(max(t_rows, 1))), dtype=torch.float32,
                              device=self.device)
        if isinstance(phi, PaddedRows):
            # Phi as the walk's padded rows (rows 0 .. n of Phi, not compacted): the pipelined kernel reads them
            if sym_row0 is not None or tr_b.rec_unit != C.REC_SLOT:
                raise ValueError("gram_sparse_cols: padded rows take a GRF_REC_SLOT transpose and no symmetric square")
            C.check(self.lib.grf_gram_sparse_cols_padded(phi.n_cols, row_begin, row_end, phi.cap, _p(phi.cnt),
                                                         _p(phi.idx), _p(phi.val32), _p(row_shift), t_rows,
                                                         tr_b.band_width, _p(tr_b.t_desc), _p(tr_b.t_rec), _p(out),
                                                         out.stride(0), self.stream), "grf_gram_sparse_cols_padded")
            return out[:, :t_rows]
        C.check(self.lib.grf_gram_sparse_cols(phi.n_cols, row_begin, row_end, _p(phi.ptr), _p(phi.idx),
                                              _p(phi.val32), _p(row_shift), t_rows,
                                              -1 if sym_row0 is None else int(sym_row0), tr_b.band_width, tr_b.rec_unit,
                                              _p(tr_b.t_desc), _p(tr_b.t_rec), _p(tr_b.t_split), _p(out), out.stride(0),
                                              _p(self._gram_ws), self._gram_ws.numel(), self.stream),
                "grf_gram_sparse_cols")
        return out[:, :t_rows]

    def gram_sparse_kslice(self, phi: DeviceCSR, tr: Banded, k_begin: int, k_end: int, row_begin: int = 0,
                           row_end: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Partial K[row_begin:row_end, :] over the inner-dimension slice [k_begin, k_end) (float32)."""
        n = tr.n_rows
        row_end = n if row_end is None else row_end
        ldk = self.leading_dim(n)
        if out is None:
            out = torch.empty((row_end - row_begin, ldk), dtype=torch.float32, device=self.device)
        C.check(self.lib.grf_gram_sparse_kslice(n, row_begin, row_end, k_begin, k_end, _p(phi.ptr), _p(phi.idx),
                                                _p(phi.val32), tr.band_width, tr.rec_unit, _p(tr.t_desc),
                                                _p(tr.t_rec),
                                                _p(tr.t_rowshift), _p(out), out.stride(0), _p(self._gram_ws),
                                                self._gram_ws.numel(), self.stream), "grf_gram_sparse_kslice")
        return out[:, :n]

    def gram_sparse_sym(self, phi: DeviceCSR, tr: Banded, out: Optional[torch.Tensor] = None,
                        skewed: bool = False) -> torch.Tensor:
        """Whole K (float32) on this device from the upper band tiles plus a mirror pass (skewed: see
        ``row_cuts``)."""
        n = tr.n_rows
        ldk = self.leading_dim(n)
        if out is None:
            out = torch.empty((n, ldk), dtype=torch.float32, device=self.device)
        cuts = self.row_cuts(phi, tr, skewed)
        if cuts is not None:  # (the waves' pair-balanced shares: same bits)
            self._gram_upper_cuts(phi, tr, out, cuts, (0, 1, 1), False)
            self.gram_mirror(out, n)
            return out[:, :n]
        C.check(self.lib.grf_gram_sparse_sym(n, _p(phi.ptr), _p(phi.idx), _p(phi.val32), tr.band_width,
                                             tr.rec_unit, _p(tr.t_desc), _p(tr.t_rec), _p(tr.t_split), _p(tr.t_rowshift),
                                             _p(out), out.stride(0),
                                             _p(self._gram_ws), self._gram_ws.numel(), self.stream),
                "grf_gram_sparse_sym")
        return out[:, :n]

    def row_cuts(self, phi: DeviceCSR, tr: Banded, skewed: bool = False) -> Optional[torch.Tensor]:
        """8 cuts per row of Phi splitting its nonzeros into shares of about equal record pairs (weights:
        every column's pairs over all bands of ``tr``), for the whole-K Gram's waves; None when the
        policy says no (GRF_GRAM_CUTS: auto = when ``skewed``, ``column_stats``) or the buckets are slots.
        Measured: Facebook 2.86-2.91 -> 2.75-2.79 ms per K; C4 (not skewed) would pay 0.5 ms for the
        cuts and gain nothing (profiles/r03_gram_balance_ab.txt)."""
        on = ROW_CUTS == "1" or (ROW_CUTS == "auto" and skewed)
        if not on or tr.rec_unit == C.REC_SLOT or phi.n_rows == 0:
            return None
        nb = -(-tr.n_rows // tr.band_width)
        col_w = torch.empty(max(1, tr.n_cols), dtype=torch.int32, device=self.device)
        cuts = torch.empty(8 * phi.n_rows, dtype=torch.int32, device=self.device)
        C.check(self.lib.grf_gram_row_cuts(phi.n_rows, _p(phi.ptr), _p(phi.idx), nb, tr.n_cols, _p(tr.t_desc),
                                           _p(col_w), _p(cuts), self.stream), "grf_gram_row_cuts")
        return cuts

    def _gram_upper_cuts(self, phi: DeviceCSR, tr: Banded, out: torch.Tensor, cuts: torch.Tensor, parts,
                         add_k: bool) -> None:
        C.check(self.lib.grf_gram_sparse_upper_ex(tr.n_rows, _p(phi.ptr), _p(phi.idx), _p(phi.val32), tr.band_width,
                                                  tr.rec_unit, _p(tr.t_desc), _p(tr.t_rec), _p(tr.t_split),
                                                  _p(tr.t_rowshift), _p(cuts), _p(out), out.stride(0), int(parts[0]),
                                                  int(parts[1]), int(parts[2]), int(add_k), self.stream),
                "grf_gram_sparse_upper_ex")

    def gram_sparse_upper(self, phi: DeviceCSR, tr: Banded, out: torch.Tensor, parts=(0, 1, 1),
                          cuts: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The Gram half of ``gram_sparse_sym`` (tiles K[i, band >= band(i)]); ``gram_mirror`` completes K.
        parts = (begin, end, n): only those parts of the band-major tile sequence cut into n.
        cuts: ``row_cuts(phi, tr)`` (the waves' pair-balanced shares; same bits)."""
        n = tr.n_rows
        if cuts is not None:
            self._gram_upper_cuts(phi, tr, out, cuts, parts, False)
            return out[:, :n]
        C.check(self.lib.grf_gram_sparse_upper(n, _p(phi.ptr), _p(phi.idx), _p(phi.val32), tr.band_width,
                                               tr.rec_unit, _p(tr.t_desc), _p(tr.t_rec), _p(tr.t_split),
                                               _p(tr.t_rowshift), _p(out),
                                               out.stride(0), int(parts[0]), int(parts[1]), int(parts[2]),
                                               _p(self._gram_ws), self._gram_ws.numel(), self.stream),
                "grf_gram_sparse_upper")
        return out[:, :n]

    def hub_split(self, phi: DeviceCSR, tr: Banded, hubs: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Split Phi's ``hubs`` densest columns off the banded transpose ``tr`` of Phi (modified in place:
        their buckets emptied in every band) into a dense fp32 panel P (n_rows x ldp, ldp a multiple of 32).
        The columns are ranked by their record pairs over all bands (the descriptors the transpose left:
        no host read), ties by column id; the panel holds them in ascending column order.
        Returns (P, cols).  Hub-heavy graphs: a column in a large share of the rows costs the sparse
        Gram one gathered record per multiply-add, the MFMA Gram of the panel ~60x less."""
        if tr.rec_unit == C.REC_SLOT:
            raise ValueError("hub_split: the GRF_REC_SLOT layout keeps no descriptor table to edit")
        n_rows, n = phi.n_rows, tr.n_cols
        h = max(0, min(int(hubs), n))
        nb = -(-tr.n_rows // tr.band_width)
        pairs = tr.t_desc[:2 * nb * n].view(nb, n, 2)[:, :, 1].sum(0, dtype=torch.int64)
        top = torch.sort(pairs, descending=True, stable=True).indices[:h]
        cols = torch.sort(top).values.to(torch.int32).contiguous()
        pos = torch.full((n,), -1, dtype=torch.int32, device=self.device)
        pos[cols.long()] = torch.arange(h, dtype=torch.int32, device=self.device)
        ldp = max(32, -(-h // 32) * 32)
        P = torch.zeros((n_rows, ldp), dtype=torch.float32, device=self.device)
        C.check(self.lib.grf_hub_panel(n_rows, _p(phi.ptr), _p(phi.idx), _p(phi.val32), _p(pos), _p(P), ldp,
                                       self.stream), "grf_hub_panel")
        C.check(self.lib.grf_transpose_drop_columns(nb, n, _p(tr.t_desc), _p(cols), h, self.stream),
                "grf_transpose_drop_columns")
        return P, cols

    def gram_sparse_sym_hubs(self, phi: DeviceCSR, tr: Banded, hubs: int, out: Optional[torch.Tensor] = None,
                             mirror_workgroups: int = 0, after_tiles=None, skewed: bool = False,
                             early_front: bool = False) -> torch.Tensor:
        """Whole K with the hub-column split: the panel of Phi's ``hubs`` densest columns through the
        MFMA Gram (tiles on and above the diagonal), the rest through the sparse Gram tiles adding to
        it, then the mirror.  ``tr`` is consumed (its hub buckets emptied).  Within the fp32 K
        tolerance of ``gram_sparse_sym`` (the hub part is an fp32 MFMA sum), exactly symmetric.
        ``after_tiles(event)``: called between the tiles and the mirror (the pipelined bench)."""
        n = tr.n_rows
        if out is None:
            out = torch.empty((n, self.leading_dim(n)), dtype=torch.float32, device=self.device)
        if int(hubs) <= 0:  # (no split: the plain symmetric Gram)
            self.gram_sparse_upper(phi, tr, out, cuts=self.row_cuts(phi, tr, skewed))
            ev = None
            if after_tiles is not None:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
            self.gram_mirror(out, n, mirror_workgroups)
            if after_tiles is not None:
                after_tiles(ev)
            return out[:, :n]
        P, cols = self.hub_split(phi, tr, hubs)
        h = int(cols.numel())
        if early_front and after_tiles is not None:
            # (the pipelined bench's next front beside the compute-bound MFMA panel, the tiles and the mirror)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            after_tiles(ev)
            after_tiles = None
        upper = self.lib.grf_gram_dense_split_upper if self.dense_precision == "split" else self.lib.grf_gram_dense_upper
        C.check(upper(n, h, _p(P), P.stride(0), _p(out), out.stride(0), self.stream), "grf_gram_dense_upper")
        cuts = self.row_cuts(phi, tr, skewed)  # (after the hub drop: the weights of the columns left)
        if cuts is not None:
            self._gram_upper_cuts(phi, tr, out, cuts, (0, 1, 1), True)
        else:
            C.check(self.lib.grf_gram_sparse_upper_add(n, _p(phi.ptr), _p(phi.idx), _p(phi.val32), tr.band_width,
                                                       tr.rec_unit, _p(tr.t_desc), _p(tr.t_rec), _p(tr.t_split),
                                                       _p(tr.t_rowshift), _p(out), out.stride(0), 0, 1, 1,
                                                       _p(self._gram_ws), self._gram_ws.numel(), self.stream),
                    "grf_gram_sparse_upper_add")
        ev = None
        if after_tiles is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
        self.gram_mirror(out, n, mirror_workgroups)
        if after_tiles is not None:
            after_tiles(ev)
        return out[:, :n]

    def gram_mirror(self, K: torch.Tensor, n: int, max_workgroups: int = 0) -> torch.Tensor:
        """K[j, i] = K[i, j] for every j > i (the second half of ``gram_sparse_sym``).
        max_workgroups > 0 bounds the grid (leaves CU slots to work on another stream)."""
        C.check(self.lib.grf_gram_mirror(n, _p(K), K.stride(0), int(max_workgroups), self.stream), "grf_gram_mirror")
        return K[:, :n]

    def densify(self, phi: DeviceCSR) -> torch.Tensor:
        lda = max(64, -(-phi.n_cols // 64) * 64)  # (zero-padded k: every k-tile width of the MFMA Gram divides it)
        out = torch.empty((phi.n_rows, lda), dtype=torch.float32, device=self.device)
        C.check(self.lib.grf_densify(phi.n_rows, _p(phi.ptr), _p(phi.idx), _p(phi.val32), _p(out), lda, self.stream),
                "grf_densify")
        return out

    def densify_padded(self, rows: PaddedRows, planes: bool = False):
        """The dense fp32 Phi (zero-padded lda, as ``densify``) straight from the walk's padded rows, no
        compaction (grf_densify_padded); rows too wide for one CU's LDS take compact + densify.
        planes: the split Gram's three bf16 planes instead (``DensePlanes``, grf_densify_padded_planes), for
        ``gram_dense``'s planes path."""
        n = rows.n_rows
        lda = max(64, -(-rows.n_cols // 64) * 64)
        if planes and rows.val32 is not None and -(-rows.n_cols // 16) * 64 <= 160 * 1024:
            ldp = int(self.lib.grf_planes_row_bytes(rows.n_cols))
            P = torch.empty((n, ldp), dtype=torch.uint8, device=self.device)
            C.check(self.lib.grf_densify_padded_planes(n, rows.cap, rows.n_cols, _p(rows.cnt), _p(rows.idx),
                                                       _p(rows.val32), _p(P), ldp, self.stream),
                    "grf_densify_padded_planes")
            return DensePlanes(P, n, rows.n_cols)
        if rows.val32 is None or lda * 4 > 160 * 1024:
            out = self.densify(self.compact(rows, want64=False, sync_free=True))
            return self.split_planes(out, rows.n_cols) if planes else out
        out = torch.empty((n, lda), dtype=torch.float32, device=self.device)
        C.check(self.lib.grf_densify_padded(n, rows.cap, rows.n_cols, _p(rows.cnt), _p(rows.idx), _p(rows.val32),
                                            _p(out), lda, self.stream), "grf_densify_padded")
        return self.split_planes(out, rows.n_cols) if planes else out

    @staticmethod
    def use_planes(n: int) -> bool:
        """The split Gram on pre-split bf16 planes (grf_gram_dense_planes) where the wide kernels run (from 64 tile
        rows on, n > 8064; GRF_DENSE_WIDE=0 turns it off with them): with the wide kernels' XCD-ordered whole-item
        rounds the staged k-tiles are L2 / Infinity-Cache hits, so staging the planes' 1.5x bytes costs less than
        the split's VALU -- C2 Gram 4.40 -> 4.01 ms (profiles/r06_dense_xcd_ab.txt; before those rounds the planes
        were staging-bound and slower, r06_dense_planes_ab.txt).  Below, the 128-tile kernel splits in registers:
        its planes twin (gram_planes_tile_kernel) measured equal at C3 (0.133 ms both: that Gram is bound by neither
        the split nor the staged bytes).  GRF_DENSE_PLANES (read per call): 1 always, 0 never.  Same K bits."""
        env = os.environ.get("GRF_DENSE_PLANES")
        if env in ("0", "1"):
            return env == "1"
        return -(-int(n) // 128) >= 64 and os.environ.get("GRF_DENSE_WIDE") != "0"

    def split_planes(self, dense_phi: torch.Tensor, k_dim: int) -> "DensePlanes":
        """The dense fp32 Phi's three bf16 planes, split once (grf_split_planes)."""
        n = dense_phi.shape[0]
        ldp = int(self.lib.grf_planes_row_bytes(k_dim))
        P = torch.empty((n, ldp), dtype=torch.uint8, device=self.device)
        C.check(self.lib.grf_split_planes(n, k_dim, _p(dense_phi), dense_phi.stride(0), _p(P), ldp, self.stream),
                "grf_split_planes")
        return DensePlanes(P, n, k_dim)

    def gram_dense(self, dense_phi: torch.Tensor, k_dim: int, precision: Optional[str] = None) -> torch.Tensor:
        """K = A A^T of the dense fp32 Phi on the MFMA.  precision 'fp32': the fp32 matrix instruction
        (grf_gram_dense_ws); 'split': the same product on the bf16 matrix cores from an exact three-plane
        split of A (grf_gram_dense_split, error bound the fp32 path's + (2^-23 + 2^-32) sum |a b|); None: the engine's
        ``dense_precision`` (GRF_GRAM_DENSE_PRECISION, default 'split')."""
        precision = precision or self.dense_precision
        if precision not in ("fp32", "split"):
            raise ValueError(f"unknown dense Gram precision {precision!r}")
        split = precision == "split"
        planes = isinstance(dense_phi, DensePlanes)
        if planes and not split:
            raise ValueError("gram_dense: the bf16 planes take precision 'split'")
        if split and not planes and self.use_planes(dense_phi.shape[0]):
            dense_phi = self.split_planes(dense_phi, k_dim)  # (the split once, then the planes' k-loop)
            planes = True
        n = dense_phi.shape[0]
        ldk = self.leading_dim(n)
        out = torch.empty((n, ldk), dtype=torch.float32, device=self.device)
        # split-K partial tiles (small n, or the last tiles of a large n) and their tickets: a cached
        # workspace per stream, ZEROED when allocated (the kernel leaves the tickets zero after every
        # launch; an uninitialised block gave round 4's NaN, profiles/AB_LOG.md "dense-Gram NaN"), dropped
        # after a failed call so that no ticket a broken launch may have left is read again.  The split
        # path sizes it for its own (wide-workgroup) slabs as well.
        need = int(self.lib.grf_gram_dense_split_workspace_bytes(n, k_dim) if split
                   else self.lib.grf_gram_dense_workspace_bytes(n, k_dim))
        stream = self.stream
        cache = self.__dict__.setdefault("_dense_ws", {})
        ws = cache.get(stream.value)
        if ws is None or ws.numel() < need:
            ws = cache[stream.value] = torch.zeros(max(need, 16), dtype=torch.uint8, device=self.device)
        fn = self.lib.grf_gram_dense_split if split else self.lib.grf_gram_dense_ws
        try:
            if planes:
                C.check(self.lib.grf_gram_dense_planes(n, k_dim, _p(dense_phi.P), dense_phi.P.stride(0), _p(out), ldk,
                                                       _p(ws), ws.numel(), stream), "grf_gram_dense_planes")
            else:
                C.check(fn(n, k_dim, _p(dense_phi), dense_phi.stride(0), _p(out), ldk, _p(ws), ws.numel(), stream),
                        "grf_gram_dense_split" if split else "grf_gram_dense_ws")
        except Exception:
            cache.pop(stream.value, None)
            raise
        return out[:, :n]

    @staticmethod
    def column_stats(phi: DeviceCSR, share: float = HUB_SHARE,
                     extend: Optional[float] = None) -> Tuple[int, bool]:
        """(hub_count, skewed) from one column count of Phi: skewed when the densest column holds at
        least SKEW_RATIO times the mean column's entries (the policy of ``row_cuts``).  extend: when at least
        one panel width of columns reaches ``share``, the hub count is taken at this (lower) share instead
        (``HUB_EXTEND_SHARE``, the split panel's).  One host read."""
        n = phi.n_cols
        if phi.nnz == 0 or n == 0:
            return 0, False
        c = torch.bincount(phi.idx[:phi.nnz].long(), minlength=n)
        low = share if extend is None else min(share, extend)
        hubs, wide, cmax = (int(x) for x in torch.stack([(c >= share * phi.n_rows).sum(),
                                                          (c >= low * phi.n_rows).sum(), c.max()]).tolist())
        hubs = hubs // 32 * 32
        if hubs and extend is not None:
            hubs = wide // 32 * 32
        return hubs, cmax >= SKEW_RATIO * phi.nnz / n

    def hub_extend_share(self) -> Optional[float]:
        """The panel's extension share for this engine's dense precision (None: the fp32 panel)."""
        return HUB_EXTEND_SHARE if self.dense_precision == "split" else None

    def hub_count(self, phi: DeviceCSR, share: float = HUB_SHARE) -> int:
        """Hub columns worth the dense MFMA panel of the hub-column split (the policy of ``gram_sparse_auto``
        and the bench's --hubs auto): the columns of Phi present in at least ``share`` of its rows, in
        multiples of 32 (the panel's width) -- with the split panel, once there are any, those down to
        ``HUB_EXTEND_SHARE``.  A column in c of the n rows saves ~c^2 / 2 gathered records and costs n^2 / 2
        MFMA multiply-adds, ~60x cheaper each on the fp32 panel, so it pays from c / n ~ 1 / sqrt(60) = 0.13
        (profiles/r02_hubs_sweep.txt); the split panel's 3/8 of that cost moved Enron's best count from 96 to
        192 columns (profiles/r05_hub_sweep_split.txt).  One host read."""
        return self.column_stats(phi, share, extend=self.hub_extend_share())[0]

    def gram_sparse_auto(self, phi: DeviceCSR, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Whole K on the sparse path exactly as the bench assembles it: the symmetric tiles + mirror,
        with the hub-column split when Phi has hub columns (``hub_count``)."""
        tr = self.transpose_banded(phi)
        hubs, skewed = self.column_stats(phi, extend=self.hub_extend_share())
        if hubs:
            return self.gram_sparse_sym_hubs(phi, tr, hubs, out=out, skewed=skewed)
        return self.gram_sparse_sym(phi, tr, out=out, skewed=skewed)

    def gram(self, phi: DeviceCSR, method: str = "auto") -> torch.Tensor:
        """K = Phi Phi^T (float32).  'dense' = MFMA on densified Phi, 'sparse' = LDS Gustavson (+ the
        hub-column split when Phi has hub columns); 'auto' picks by the measured crossover."""
        if method == "auto":
            method = "dense" if phi.n_rows <= DENSE_GRAM_MAX_N else "sparse"
        if method == "dense":
            return self.gram_dense(self.densify(phi), phi.n_cols)
        if method == "sparse":
            return self.gram_sparse_auto(phi)
        if method == "sparse-rows":
            return self.gram_sparse(phi, self.transpose_banded(phi, ROWS_BAND_WIDTH))
        raise ValueError(f"unknown gram method {method!r}")

    # ------------------------------------- K.v and CG (models/sparse_grf_model.py:21-45)
    def _row_map(self, rows) -> Optional[torch.Tensor]:
        if rows is None:
            return None
        return torch.as_tensor(rows, device=self.device).to(torch.int32).flatten().contiguous()

    def csr_transpose(self, phi: DeviceCSR, rows=None) -> DeviceCSR:
        """(Phi[rows])^T as CSR (n_cols x len(rows), float32); column lists in ascending row order."""
        rmap = self._row_map(rows)
        n_sel = phi.n_rows if rmap is None else rmap.numel()
        # the entries to transpose, or an upper bound of them (no host read; the C side ignores the tail)
        exact = True
        if rmap is None:
            nnz = phi.nnz_or_bound()
            exact = phi._nnz is not None
        elif phi.rows_entry_bound(n_sel) is not None:
            nnz, exact = phi.rows_entry_bound(n_sel), False
        else:
            rl = rmap.long()
            nnz = int((phi.ptr[rl + 1] - phi.ptr[rl]).sum().item()) if n_sel else 0
        t_ptr = self._empty(phi.n_cols + 1, torch.int64)
        t_idx = self._empty(nnz, torch.int32)
        t_val = self._empty(nnz, torch.float32)
        ws = self._ws(self.lib.grf_csr_transpose_workspace_bytes(n_sel, phi.n_cols, nnz))
        C.check(self.lib.grf_csr_transpose(n_sel, _p(phi.ptr), _p(phi.idx), _p(phi.val32), _p(rmap), phi.n_cols, nnz,
                                           _p(t_ptr), _p(t_idx), _p(t_val), _p(ws), ws.numel(), self.stream),
                "grf_csr_transpose")
        return DeviceCSR(phi.n_cols, n_sel, t_ptr, t_idx, None, t_val, nnz if exact else None, nnz_bound=nnz)

    def spmm(self, A: DeviceCSR, X: torch.Tensor, rows=None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Y = A[rows] X (X float32 or float64, n_cols x S with unit column stride; Y the same type)."""
        if X.dtype not in (torch.float32, torch.float64) or X.dim() != 2 or X.stride(1) != 1 \
                or X.shape[0] != A.n_cols:
            raise ValueError("spmm: X must be a float32/float64 (n_cols x S) row-major matrix")
        rmap = self._row_map(rows)
        n_out = A.n_rows if rmap is None else rmap.numel()
        S = X.shape[1]
        if out is None:
            out = torch.empty((n_out, S), dtype=X.dtype, device=self.device)
        fn = self.lib.grf_spmm_csr if X.dtype == torch.float32 else self.lib.grf_spmm_csr_f64
        C.check(fn(n_out, _p(A.ptr), _p(A.idx), _p(A.val32), _p(rmap), _p(X), X.stride(0), S, _p(out),
                   out.stride(0), self.stream), "grf_spmm_csr")
        return out

    def gram_matvec(self, phi: DeviceCSR, V: torch.Tensor, rows=None, cols=None, phi_t: Optional[DeviceCSR] = None,
                    noise: float = 0.0) -> torch.Tensor:
        """K[rows, cols] V = Phi[rows] (Phi[cols]^T V) (+ noise V when rows == cols), K never formed."""
        phi_t = self.csr_transpose(phi, cols) if phi_t is None else phi_t
        Y = self.spmm(phi, self.spmm(phi_t, V), rows)
        if noise:
            Y.add_(V, alpha=float(noise))
        return Y

    def cg_solve(self, phi: DeviceCSR, B: torch.Tensor, noise: float, rows=None, phi_t: Optional[DeviceCSR] = None,
                 tolerance: float = 1.0, max_iter: int = 1000, return_residuals: bool = False):
        """linear_cg on (Phi[rows] Phi[rows]^T + noise I) X = B for the columns of B (n x S, S <= 256).

        B float64 runs the recurrence in fp64, float32 in the reference's fp32.  Returns
        (X, iterations) [+ the final residual norms of the normalised columns].  tolerance / max_iter default to gpytorch's settings.cg_tolerance (1)
        and settings.max_cg_iterations (1000)."""
        rmap = self._row_map(rows)
        n_sys = phi.n_rows if rmap is None else rmap.numel()
        if B.dtype not in (torch.float32, torch.float64) or B.dim() != 2 or B.stride(1) != 1 \
                or B.shape[0] != n_sys:
            raise ValueError("cg_solve: B must be a float32/float64 (n_rows x S) row-major matrix")
        phi_t = self.csr_transpose(phi, rmap) if phi_t is None else phi_t
        S = B.shape[1]
        X = torch.empty((n_sys, S), dtype=B.dtype, device=self.device)
        ws = self._ws(self.lib.grf_cg_workspace_bytes(n_sys, phi.n_cols, S))
        iters = ctypes.c_int32(0)
        resid = np.zeros(S, np.float64)
        fn = self.lib.grf_cg_gram_solve if B.dtype == torch.float32 else self.lib.grf_cg_gram_solve_f64
        C.check(fn(n_sys, _p(phi.ptr), _p(phi.idx), _p(phi.val32), _p(rmap), phi.n_cols, _p(phi_t.ptr),
                   _p(phi_t.idx), _p(phi_t.val32), float(noise), _p(B), B.stride(0), S, float(tolerance),
                   int(max_iter), _p(X), X.stride(0), _p(ws), ws.numel(), ctypes.byref(iters),
                   resid.ctypes.data_as(ctypes.c_void_p), self.stream), "grf_cg_gram_solve")
        if return_residuals:
            return X, int(iters.value), resid
        return X, int(iters.value)

    def pathwise_predict(self, phi: DeviceCSR, train_idx, test_idx, y_train: torch.Tensor, noise: float,
                         eps1: torch.Tensor, eps2: torch.Tensor, tolerance: float = 1.0, max_iter: int = 1000,
                         dtype: torch.dtype = torch.float64):
        """SparseGraphGP.predict (models/sparse_grf_model.py:21-45) given its random draws.

        eps1: (S x n_nodes) prior weights, eps2: (S x n_train) noise draws (already scaled by
        the noise std).  dtype: float64 (default) or the reference's float32 for every dense
        block and the CG recurrence.  Returns (S x n_test) posterior samples (dtype) and the
        CG iteration count."""
        tr = self._row_map(train_idx)
        te = self._row_map(test_idx)
        E = eps1.to(self.device, dtype).t().contiguous()                      # n_nodes x S
        f_train = self.spmm(phi, E, tr)                                        # (eps1 @ phi_train.T)^T
        f_test = self.spmm(phi, E, te)
        y = y_train.to(self.device, dtype).flatten()
        B = y[:, None] - (f_train + eps2.to(self.device, dtype).t())          # b_batch^T
        phi_t = self.csr_transpose(phi, tr)
        V, iters = self.cg_solve(phi, B.contiguous(), noise, tr, phi_t, tolerance, max_iter)
        out = f_test + self.spmm(phi, self.spmm(phi_t, V), te)                # + K_test_train v
        return out.t(), iters

    # ------------------------------------------------------------- pipelines
    def kernel_matrix(self, A, modulator_vector: Sequence[float], walks_per_node: int, p_halt: float,
                      max_walk_length: int, *, rng: int = C.RNG_PHILOX, seed: int = 42, n_chunks: int = 1,
                      laplacian: bool = True, method: str = "auto", norm: int = C.NORM_MUL_RECIP) -> torch.Tensor:
        """Sparse-path K = Phi Phi^T (fast_grf_kernel_general.py:42-55), float32 on the device."""
        G = self.laplacian(A) if laplacian else self.to_device(A)
        slots = self.walk(G, walks_per_node, p_halt, max_walk_length, rng=rng, seed=seed, n_chunks=n_chunks)
        phi = self.compact(self.features(slots, modulator_vector, norm))
        return self.gram(phi, method)


_engines: dict = {}


def get_engine(device=None) -> GRFEngine:
    """Process-wide engine per device (GRF_AMD_DEVICE overrides the default)."""
    if device is None:
        device = os.environ.get("GRF_AMD_DEVICE")
    key = str(device)
    if key not in _engines:
        _engines[key] = GRFEngine(device)
    return _engines[key]
