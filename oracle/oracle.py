"""ctypes front-end of the CPU parity oracle (``oracle/grf_oracle.c``).

TEST INFRASTRUCTURE ONLY -- imported by ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg, and there only as the checker or the
timed CPU baseline.  The product package never imports this module.

Each helper restates one reference entry point (paths under /root/reference):

* :func:`sparse_random_walk` -- ``SparseRandomWalk.get_random_walk_matrices``
  (``efficient_graph_gp_sparse/random_walk_samplers_sparse/sparse_sampler.py:59-132``)
* :func:`dense_random_walk` -- ``RandomWalk.get_random_walk_matrices``
  (``efficient_graph_gp/random_walk_samplers/sampler.py:85-203``)
* :func:`laplacian_sparse` / :func:`laplacian_dense` -- the two
  ``get_normalized_laplacian`` variants
* :func:`phi_sparse` / :func:`gram_rows` -- ``Phi = sum f_l M_l`` and ``K = Phi Phi^T``
  (``efficient_graph_gp_sparse/graph_kernels_sparse/fast_grf_kernel_general.py:47-55``)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import scipy.sparse as sp

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libgrf_oracle.so")

LOAD_CUMULATIVE, LOAD_NONCUMULATIVE, LOAD_ABLATION = 0, 1, 2
RNG_PCG64, RNG_PHILOX = 0, 1
NORM_DIV, NORM_MUL_RECIP = 0, 1

_lib = None


def build() -> str:
    """Compile the oracle with gcc (idempotent)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
            os.path.join(_HERE, "grf_oracle.c")
        ):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.oracle_np_pairwise.restype = ctypes.c_double
        _lib.oracle_np_reduceat.restype = ctypes.c_double
        _lib.oracle_laplacian_sparse.restype = ctypes.c_int64
        _lib.oracle_walk_range.restype = ctypes.c_int
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


def _threads(n_threads):
    return int(n_threads if n_threads else (os.cpu_count() or 1))


# --------------------------------------------------------------------------- RNG
def seed_words(seed: int) -> np.ndarray:
    """numpy ``_int_to_uint32_array``: little-endian 32-bit words (0 -> [0])."""
    seed = int(seed)
    if seed < 0:
        raise ValueError("seed must be non-negative")
    w = []
    while seed:
        w.append(seed & 0xFFFFFFFF)
        seed >>= 32
    return np.array(w or [0], dtype=np.uint32)


def pcg64_init(seed: int) -> tuple[int, int]:
    w = seed_words(seed)
    out = np.zeros(4, np.uint64)
    lib().oracle_pcg64_init(_p(w), ctypes.c_int(len(w)), _p(out))
    return (int(out[0]) << 64) | int(out[1]), (int(out[2]) << 64) | int(out[3])


def pcg64_stream(seed: int, ops) -> np.ndarray:
    w = seed_words(seed)
    ops = np.ascontiguousarray(ops, dtype=np.uint32)
    out = np.zeros(len(ops), np.float64)
    lib().oracle_pcg64_stream(_p(w), ctypes.c_int(len(w)), _p(ops), ctypes.c_int64(len(ops)), _p(out))
    return out


def philox4x32_10(ctr, key) -> np.ndarray:
    c = np.ascontiguousarray(ctr, dtype=np.uint32)
    k = np.ascontiguousarray(key, dtype=np.uint32)
    out = np.zeros(4, np.uint32)
    lib().oracle_philox4x32_10(_p(c), _p(k), _p(out))
    return out


def np_pairwise(a) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().oracle_np_pairwise(_p(a), ctypes.c_int64(len(a)))


def np_reduceat(a) -> float:
    a = np.ascontiguousarray(a, dtype=np.float64)
    return lib().oracle_np_reduceat(_p(a), ctypes.c_int64(len(a)))


# ------------------------------------------------------------------ Laplacians
def _csr_arrays(A):
    A = sp.csr_matrix(A)
    return (
        np.ascontiguousarray(A.indptr, dtype=np.int64),
        np.ascontiguousarray(A.indices, dtype=np.int32),
        np.ascontiguousarray(A.data, dtype=np.float64),
    )


def laplacian_sparse(A) -> tuple[sp.csr_matrix, np.ndarray]:
    """scipy semantics (graph_utils.py:16-30); returns (L, degrees)."""
    A = sp.csr_matrix(A)
    n = A.shape[0]
    ip, ix, dx = _csr_arrays(A)
    nnz_cap = len(ix) + n
    op = np.zeros(n + 1, np.int64)
    ox = np.zeros(max(nnz_cap, 1), np.int32)
    odx = np.zeros(max(nnz_cap, 1), np.float64)
    deg = np.zeros(n, np.float64)
    nnz = lib().oracle_laplacian_sparse(ctypes.c_int64(n), _p(ip), _p(ix), _p(dx), _p(op), _p(ox), _p(odx), _p(deg))
    L = sp.csr_matrix((odx[:nnz].copy(), ox[:nnz].copy(), op.astype(np.int32)), shape=(n, n))
    return L, deg


def laplacian_dense(W, mode: int = 0) -> np.ndarray:
    """numpy semantics; mode 0 utils.py, 1 laplacian_np.py (safe), 2 combinatorial."""
    W = np.ascontiguousarray(W, dtype=np.float64)
    n = W.shape[0]
    out = np.zeros((n, n), np.float64)
    lib().oracle_laplacian_dense(ctypes.c_int64(n), _p(W), ctypes.c_int32(mode), _p(out))
    return out


def dense_to_walk_csr(Ld: np.ndarray):
    """Dense walk matrix -> CSR of its nonzeros in ascending column order
    (``np.flatnonzero(L[row])`` neighbour order, sampler.py:22-28)."""
    Ld = np.asarray(Ld, dtype=np.float64)
    mask = Ld != 0
    indptr = np.zeros(Ld.shape[0] + 1, np.int64)
    indptr[1:] = np.cumsum(mask.sum(axis=1))
    rows, cols = np.nonzero(mask)
    return indptr, cols.astype(np.int32), Ld[rows, cols].astype(np.float64)


# ----------------------------------------------------------------------- walks
def walk_slots(indptr, indices, data, m, p_halt, L, *, rng=RNG_PCG64, load_rule=LOAD_CUMULATIVE,
               n_chunks=1, seed=42, begin=None, end=None, n_threads=None):
    """Run walks; returns slot arrays node[n][L][m] (int32, -1 empty), load[n][L][m]."""
    n = len(indptr) - 1
    indptr = np.ascontiguousarray(indptr, np.int64)
    indices = np.ascontiguousarray(indices, np.int32)
    data = np.ascontiguousarray(data, np.float64)
    node = np.full((n, L, m), -1, np.int32)
    load = np.zeros((n, L, m), np.float64)
    if begin is None:
        begin, end = 0, (n_chunks if rng == RNG_PCG64 else n)
    rc = lib().oracle_walk_range(
        ctypes.c_int64(n), _p(indptr), _p(indices), _p(data), ctypes.c_int64(m), ctypes.c_double(p_halt),
        ctypes.c_int32(L), ctypes.c_int32(load_rule), ctypes.c_int32(rng), ctypes.c_int64(n_chunks),
        ctypes.c_uint64(seed), ctypes.c_int64(begin), ctypes.c_int64(end), _p(node), _p(load),
        ctypes.c_int(_threads(n_threads)))
    if rc != 0:
        raise ValueError("oracle_walk_range failed")
    return node, load


def reduce_steps(node, load, norm=NORM_MUL_RECIP, n_threads=None):
    """Slots -> list of L step CSR matrices (sorted columns, explicit zeros kept)."""
    n, L, m = node.shape
    node = np.ascontiguousarray(node, np.int32)
    load = np.ascontiguousarray(load, np.float64)
    cnt = np.zeros((n, L), np.int64)
    lib().oracle_reduce_count(ctypes.c_int64(n), ctypes.c_int64(m), ctypes.c_int32(L), _p(node), _p(load), _p(cnt),
                              ctypes.c_int(_threads(n_threads)))
    rowptr = np.zeros((L, n + 1), np.int64)
    rowptr[:, 1:] = np.cumsum(cnt.T, axis=1)
    l_off = np.zeros(L, np.int64)
    l_off[1:] = np.cumsum(rowptr[:, -1])[:-1]
    tot = int(rowptr[:, -1].sum())
    idx = np.zeros(max(tot, 1), np.int32)
    val = np.zeros(max(tot, 1), np.float64)
    lib().oracle_reduce_fill(ctypes.c_int64(n), ctypes.c_int64(m), ctypes.c_int32(L), ctypes.c_int32(norm), _p(node),
                             _p(load), _p(rowptr), _p(l_off), _p(idx), _p(val), ctypes.c_int(_threads(n_threads)))
    mats = []
    for l in range(L):
        a, b = int(l_off[l]), int(l_off[l] + rowptr[l, -1])
        mats.append(sp.csr_matrix((val[a:b].copy(), idx[a:b].copy(), rowptr[l].astype(np.int32)), shape=(n, n)))
    return mats


def phi_sparse(step_mats, f, n_threads=None) -> sp.csr_matrix:
    """scipy ``Phi += f_p * M_p`` semantics over ``min(len(f), len(steps))`` steps."""
    nsteps = min(len(f), len(step_mats))
    n = step_mats[0].shape[0]
    if nsteps == 0:
        return sp.csr_matrix((n, n))
    rowptr = np.stack([np.asarray(step_mats[l].indptr, np.int64) for l in range(nsteps)])
    l_off = np.zeros(nsteps, np.int64)
    l_off[1:] = np.cumsum([step_mats[l].nnz for l in range(nsteps)])[:-1]
    idx = np.ascontiguousarray(np.concatenate([step_mats[l].indices for l in range(nsteps)]), np.int32)
    val = np.ascontiguousarray(np.concatenate([step_mats[l].data for l in range(nsteps)]), np.float64)
    fa = np.ascontiguousarray(np.asarray(f, np.float64)[:nsteps])
    cnt = np.zeros(n, np.int64)
    t = ctypes.c_int(_threads(n_threads))
    args = (ctypes.c_int64(n), ctypes.c_int32(nsteps), _p(rowptr), _p(l_off), _p(idx), _p(val), _p(fa))
    lib().oracle_phi(*args, ctypes.c_void_p(0), _p(cnt), ctypes.c_void_p(0), ctypes.c_void_p(0), t)
    ptr = np.zeros(n + 1, np.int64)
    ptr[1:] = np.cumsum(cnt)
    pidx = np.zeros(max(int(ptr[-1]), 1), np.int32)
    pval = np.zeros(max(int(ptr[-1]), 1), np.float64)
    lib().oracle_phi(*args, _p(ptr), ctypes.c_void_p(0), _p(pidx), _p(pval), t)
    nnz = int(ptr[-1])
    return sp.csr_matrix((pval[:nnz], pidx[:nnz], ptr), shape=(n, n))


def gram_rows(phi: sp.csr_matrix, r0: int = 0, r1: int | None = None, n_threads=None) -> np.ndarray:
    """Dense rows [r0, r1) of Phi Phi^T with scipy csr_matmat summation order."""
    phi = sp.csr_matrix(phi)
    phi.sort_indices()
    n = phi.shape[0]
    r1 = n if r1 is None else r1
    pt = phi.T.tocsr()
    pt.sort_indices()
    ptr, idx, val = _csr_arrays(phi)
    tptr, tidx, tval = _csr_arrays(pt)
    K = np.zeros((r1 - r0, n), np.float64)
    lib().oracle_gram_rows(ctypes.c_int64(n), _p(ptr), _p(idx), _p(val), _p(tptr), _p(tidx), _p(tval),
                           ctypes.c_int64(r0), ctypes.c_int64(r1), _p(K), ctypes.c_int(_threads(n_threads)))
    return K


# --------------------------------------------------- reference-level restatements
def chunk_bounds(n: int, n_chunks: int) -> np.ndarray:
    """np.array_split(np.arange(n), n_chunks) boundaries."""
    base, extra = divmod(n, n_chunks)
    sizes = [base + (1 if i < extra else 0) for i in range(n_chunks)]
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)


def pstep_walk_matrix(W, p_max: int) -> np.ndarray:
    """Exact walk tensor ``T[:, :, l] = W^l`` for l < p_max: ``compute_pstep_walk_matrix``
    (``efficient_graph_gp/gpflow_kernels/general_kernel_pofm.py:7-42``; powers by repeated
    right-multiplication, slice 0 the identity).  The GRF estimator is unbiased for it:
    E[M_l] = W^l for the cumulative load rule."""
    W = np.asarray(W, np.float64)
    n = W.shape[0]
    T = np.zeros((n, n, p_max), np.float64)
    T[:, :, 0] = np.eye(n)
    cur = np.eye(n)
    for l in range(1, p_max):
        cur = cur @ W
        T[:, :, l] = cur
    return T


def clt_check(samples: np.ndarray, expected: np.ndarray, z: float = 6.0, rtol_exact: float = 1e-12,
              min_nonzero: float = 0.75):
    """Unbiasedness check of an estimator from independent replicas ``samples[r, ...]``.

    * entries whose replicas all agree must equal ``expected`` to ``rtol_exact`` (deterministic parts);
    * entries that are nonzero in at least ``min_nonzero`` of the replicas: the replica mean lies within
      ``z`` standard errors of ``expected`` (rarer entries are dominated by a few large walks, and their
      sample spread is no reliable standard error; the aggregate checks below cover them);
    * the sums over the last axis-but-one (row sums of every step) and the totals per step: within
      ``z`` standard errors as well -- these carry any systematic bias (a wrong halt probability
      scales a whole step by ((1-p')/(1-p))^l).
    Returns (ok, worst z-score, number of entries z-tested)."""
    R = samples.shape[0]

    def zs_of(S, E, mask=None):
        mean = S.mean(axis=0)
        se = S.std(axis=0, ddof=1) / np.sqrt(R)
        scale = np.maximum(np.abs(E), 1.0)
        spread = se > 1e-14 * scale
        exact = bool(np.all(np.abs(mean - E)[~spread] <= rtol_exact * scale[~spread]))
        sel = spread if mask is None else spread & mask
        return exact, np.abs(mean - E)[sel] / se[sel]

    nonzero = (samples != 0).mean(axis=0) >= min_nonzero
    ok1, z1 = zs_of(samples, expected, nonzero)
    ok2, z2 = zs_of(samples.sum(axis=-2), expected.sum(axis=-2))
    ok3, z3 = zs_of(samples.sum(axis=(-3, -2)), expected.sum(axis=(-3, -2)))
    allz = np.concatenate([z1, z2, z3])
    worst = float(allz.max()) if allz.size else 0.0
    return ok1 and ok2 and ok3 and worst <= z, worst, int(z1.size)


def sparse_random_walk(adj, num_walks, p_halt, max_walk_length, n_processes, seed=None, n_threads=None):
    """``SparseRandomWalk(adj, seed).get_random_walk_matrices(..., n_processes)``."""
    ip, ix, dx = _csr_arrays(adj)
    node, load = walk_slots(ip, ix, dx, num_walks, p_halt, max_walk_length, rng=RNG_PCG64,
                            load_rule=LOAD_CUMULATIVE, n_chunks=n_processes, seed=(seed or 42), n_threads=n_threads)
    return reduce_steps(node, load, NORM_MUL_RECIP, n_threads=n_threads)


def dense_random_walk(walk_matrix, num_walks, p_halt, max_walk_length, n_processes, seed=None, ablation=False,
                      n_threads=None):
    """``RandomWalk(Graph(W), seed).get_random_walk_matrices(..., n_processes, ablation)`` -> (N,N,L).

    Sequential path (sampler.py:115-116,148-186) when n_processes == 1 or N < 2*n_processes:
    one ``default_rng(seed)`` stream, non-cumulative (or ablation) load.  Otherwise the
    fork-pool path (sampler.py:119-146): chunks seeded (seed or 42)+i, cumulative load.
    """
    W = np.asarray(walk_matrix, dtype=np.float64)
    n = W.shape[0]
    ip, ix, dx = dense_to_walk_csr(W)
    if n_processes == 1 or n < 2 * n_processes:
        if seed is None:
            raise ValueError("sequential reference path with seed=None is not reproducible")
        rule = LOAD_ABLATION if ablation else LOAD_NONCUMULATIVE
        node, load = walk_slots(ip, ix, dx, num_walks, p_halt, max_walk_length, rng=RNG_PCG64, load_rule=rule,
                                n_chunks=1, seed=seed, n_threads=n_threads)
    else:
        node, load = walk_slots(ip, ix, dx, num_walks, p_halt, max_walk_length, rng=RNG_PCG64,
                                load_rule=LOAD_CUMULATIVE, n_chunks=n_processes, seed=(seed or 42),
                                n_threads=n_threads)
    mats = reduce_steps(node, load, NORM_DIV, n_threads=n_threads)
    F = np.zeros((n, n, max_walk_length), np.float64)
    for l, M in enumerate(mats):
        F[:, :, l] = M.toarray()
    return F


def step_functionals(node, load, src0: int = 0) -> np.ndarray:
    """Per-step functionals of one replica of walk slots (``node`` / ``load`` [n_src, L, m], node -1 =
    no visit; the reference's accumulator ``M_l[start, node] += load`` divided by m, sparse_sampler.py:40-54,
    130): for every step l the rows [visits V_l, sum |load| A_l, sum load T_l, sum of the loads that
    return to their source D_l, sum of the step's multipliers |load_l / load_(l-1)| G_l], each divided by
    m.  Array (L, 5).  Slot [s, l, w] is walk w's visit at step l.  G_l is bounded per walk
    ((deg + 1) max|w| / (1 - p)), so it pins the load rule of every single step without the heavy tail
    that the products A_l, T_l carry.  Equal in distribution for any two samplers of the same walk (the
    two-sample statistic below compares them)."""
    node = np.asarray(node)
    load = np.asarray(load, np.float64)
    m = node.shape[2]
    vis = node >= 0
    lv = np.where(vis, load, 0.0)
    src = (src0 + np.arange(node.shape[0]))[:, None, None]
    back = np.where(node == src, lv, 0.0)
    mult = np.zeros_like(lv)
    prev = lv[:, :-1, :]
    mult[:, 1:, :] = np.where(vis[:, 1:, :] & (prev != 0), np.abs(lv[:, 1:, :]) / np.where(prev != 0, np.abs(prev), 1.0),
                              0.0)
    return np.stack([vis.sum(axis=(0, 2)), np.abs(lv).sum(axis=(0, 2)), lv.sum(axis=(0, 2)),
                     back.sum(axis=(0, 2)), mult.sum(axis=(0, 2))], axis=1) / m


def mann_whitney_z(x: np.ndarray, y: np.ndarray) -> np.ndarray:
    """Two-sample Mann-Whitney U statistic as a z-score, per column of x (R_x, ...) and y (R_y, ...)
    (tie-corrected normal approximation).  Distribution-free under H0 (all replicas exchangeable), so
    the rare huge loads of the signed Laplacian's later steps (hub self-loops multiply a load by
    deg + 1) move one rank each instead of a mean: a statistic that tolerates those tails where a
    CLT bound on means does not."""
    from scipy.stats import rankdata
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    nx, ny = x.shape[0], y.shape[0]
    both = np.concatenate([x, y], axis=0)
    ranks = rankdata(both, axis=0)
    U = ranks[:nx].sum(axis=0) - nx * (nx + 1) / 2.0
    n = nx + ny
    # tie correction: sum over tie groups of (t^3 - t), per column
    flat = both.reshape(n, -1)
    tc = np.zeros(flat.shape[1])
    for c in range(flat.shape[1]):
        _, cnt = np.unique(flat[:, c], return_counts=True)
        tc[c] = ((cnt ** 3) - cnt).sum()
    var = nx * ny / 12.0 * ((n + 1) - tc.reshape(U.shape) / (n * (n - 1)))
    z = (U - nx * ny / 2.0) / np.sqrt(np.maximum(var, 1e-300))
    return np.where(var > 0, z, 0.0)
