"""Parity of the benchmarked path at the benchmarked sizes (BASELINE.json configs C4, C5, C3).

Each test runs ``grf_amd.pipeline`` -- the very functions ``bench.py`` times -- and checks it
against the oracle (``oracle/``, itself pinned to the reference's golden vectors):

* C4 (the headline, ``fast_grf_kernel_general.py:20-55`` at N = 100k, 1M edges, m = 128, L = 8):
  the whole fp32 Phi bit-exact against the oracle's fp64 Phi rounded once; K rows (first / last rows,
  both sides of every 4096-row band edge the Gram tiles and the mirror meet at, the highest-degree
  rows, random rows) within the K tolerance; exact symmetry of blocks across bands; diag K; and two
  size-independent checks over ALL 10^10 entries: K 1 and K v against Phi (Phi^T 1) and Phi (Phi^T v)
  in fp64, each within the summed elementwise bound.
* C5 (N = 1M power-law, m = 64, the column block K[:, 0:8192]): the whole Phi bit-exact; sampled
  rows of the block; column sums and a matrix-vector product over the whole block.
* C3 (Cora, the reference's dense path ``graph_kernels/fast_grf_kernel_general.py:11-39`` as
  ``bench.py --workload c3`` and the bench's MFMA leg run it): Phi bit-exact, K within tolerance.

K tolerance (fp32 K of fp32 Phi against the fp64 oracle), elementwise:
    |dK_ij| <= 3e-5 (|Phi| |Phi|^T)_ij + 1e-12 max(rowmax_i, rowmax_j) max|Phi|
and for a product K u with |u| <= 1 the same bound summed over j.
"""
import math
import time

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle as O

pytestmark = pytest.mark.gpu

N_THREADS = 16  # the GPU box's CPU share


def _diffusion(L):
    return np.array([(-1.0) ** l / (2.0 ** l * math.factorial(l)) for l in range(L)])


@pytest.fixture(scope="module")
def eng():
    from grf_amd.engine import GRFEngine
    return GRFEngine("cuda:0")


def _oracle_phi(A, m, p, L, f, seed=42):
    Ls, _ = O.laplacian_sparse(A)
    ip, ix, dx = O._csr_arrays(Ls)
    node, load = O.walk_slots(ip, ix, dx, m, p, L, rng=O.RNG_PHILOX, seed=seed, n_threads=N_THREADS)
    mats = O.reduce_steps(node, load, O.NORM_MUL_RECIP, n_threads=N_THREADS)
    del node, load
    return O.phi_sparse(mats, f, n_threads=N_THREADS)


def _assert_phi32_equal(phi_dev, ref64):
    """Device Phi (compact CSR, fp32 values) == the oracle's fp64 Phi rounded once to fp32."""
    ptr = phi_dev.ptr.cpu().numpy()
    nnz = int(ptr[-1])
    assert np.array_equal(ptr, np.asarray(ref64.indptr, np.int64))
    assert np.array_equal(phi_dev.idx[:nnz].cpu().numpy(), ref64.indices)
    got = phi_dev.val32[:nnz].cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref64.data.astype(np.float32).view(np.uint32))


def _bound_parts(ref64):
    absphi = abs(ref64).tocsr()
    rowmax = np.asarray(absphi.max(axis=1).todense()).ravel()
    return absphi, rowmax, float(absphi.max())


def _rows_close(K_rows, ref64, rows, cols=None, parts=None):
    """K_rows[r] vs (Phi[rows] Phi[cols]^T)[r] in fp64, elementwise bound."""
    absphi, rowmax, amax = parts or _bound_parts(ref64)
    B = ref64 if cols is None else ref64[cols]
    aB = absphi if cols is None else absphi[cols]
    cmax = rowmax if cols is None else rowmax[cols]
    Kref = (ref64[rows] @ B.T).toarray()
    bound = (absphi[rows] @ aB.T).toarray()
    fx = 1e-12 * np.maximum(rowmax[rows][:, None], cmax[None, :]) * amax
    err = np.abs(np.asarray(K_rows, np.float64) - Kref)
    bad = err > 3e-5 * bound + fx + 1e-30
    return not bad.any(), float(err.max()), int(bad.sum())


def _matvec_close(Ku, ref64, u, cols=None, parts=None):
    """Ku (K u summed on the GPU in fp64) vs Phi (Phi[cols]^T u) with the summed bound."""
    absphi, rowmax, amax = parts or _bound_parts(ref64)
    B = ref64 if cols is None else ref64[cols]
    aB = absphi if cols is None else absphi[cols]
    ref = ref64 @ (B.T @ u)
    bound = 3e-5 * (absphi @ (aB.T @ np.abs(u))) + 1e-12 * amax * np.abs(u).sum() * rowmax.max() \
        + 1e-7 * np.abs(ref)  # (+ the fp64 summation of fp32 entries on the GPU)
    err = np.abs(Ku - ref)
    return bool(np.all(err <= bound)), float((err / np.maximum(bound, 1e-300)).max())


def _k_matvec(K, u, chunk=4096):
    """K u in fp64 from the fp32 K on the device, chunked over rows (K is (rows x cols))."""
    import torch
    ut = torch.from_numpy(u).to(K.device)
    out = []
    for r0 in range(0, K.shape[0], chunk):
        out.append((K[r0:r0 + chunk].double() @ ut).cpu())
    return torch.cat(out).numpy()


def _kt_matvec(K, u, chunk=4096):
    """K^T u in fp64 (column sums for u = 1)."""
    import torch
    ut = torch.from_numpy(u).to(K.device)
    acc = torch.zeros(K.shape[1], dtype=torch.float64, device=K.device)
    for r0 in range(0, K.shape[0], chunk):
        acc += K[r0:r0 + chunk].double().t() @ ut[r0:r0 + chunk]
    return acc.cpu().numpy()


def test_c4_headline_path(eng):
    """C4 through pipeline.front + pipeline.k_assembly (symmetric tiles + the 1024-workgroup mirror of
    the pipelined bench), at the bench's exact size."""
    import torch
    from grf_amd import pipeline as P
    from grf_amd.engine import DeviceCSR
    from grf_amd.graphs import er_graph_exact_edges

    t0 = time.time()
    n, n_edges, m, L, p = 100_000, 1_000_000, 128, 8, 0.1
    A = er_graph_exact_edges(n, n_edges, seed=0)
    f = _diffusion(L)
    pl = P.plan_step(n, m, L, p, f)
    assert pl.mode == "sym" and pl.band_width == 4096
    K, fr = P.kernel_step(eng, DeviceCSR.from_scipy(A, eng.device), pl, mirror_workgroups=1024)
    torch.cuda.synchronize()
    Kv = P.k_view(K, pl)
    ref = _oracle_phi(A, m, p, L, f)
    print(f"[c4] gpu + oracle Phi {time.time() - t0:.1f} s, nnz {ref.nnz}", flush=True)
    _assert_phi32_equal(fr.phi, ref)
    parts = _bound_parts(ref)
    deg = np.diff(A.indptr)
    bw = pl.band_width
    edges = np.concatenate([[b - 1, b] for b in range(bw, n, bw)])
    rng = np.random.default_rng(5)
    rows = np.unique(np.concatenate([np.arange(64), np.arange(n - 64, n), edges,
                                     np.argsort(-deg, kind="stable")[:32], rng.integers(0, n, 256)]))
    for chunk in np.array_split(rows, max(1, len(rows) // 128)):
        ok, e, nbad = _rows_close(Kv[torch.from_numpy(chunk).to(K.device)].cpu().numpy(), ref, chunk, parts=parts)
        assert ok, (e, nbad, chunk[:4])
    print(f"[c4] {len(rows)} rows ok {time.time() - t0:.1f} s", flush=True)
    # exact symmetry: diagonal, band-straddling and far off-diagonal blocks
    for a, c in ((0, 0), (bw - 1024, bw - 1024), (bw - 512, 5 * bw + 100), (3, n - 2048), (40_000, 70_001)):
        B1 = Kv[a:a + 2048, c:c + 2048]
        B2 = Kv[c:c + 2048, a:a + 2048]
        assert torch.equal(B1, B2.t()), (a, c)
    diag = Kv.diagonal().cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(diag, np.asarray(ref.multiply(ref).sum(axis=1)).ravel(), rtol=3e-5)
    # all 10^10 entries: K 1 and K v
    for u in (np.ones(n), rng.choice([-1.0, 1.0], n)):
        ok, worst = _matvec_close(_k_matvec(Kv, u), ref, u, parts=parts)
        assert ok, worst
    print(f"[c4] symmetry, diag, K 1, K v ok {time.time() - t0:.1f} s", flush=True)
    del K, Kv


def test_c5_column_block_path(eng):
    """C5 (1M-node Chung-Lu power-law, m = 64) through the bench's column-block path: Phi of all 1M
    nodes and K[:, 0:8192] (= K rows 0..8191) from the transpose of those rows."""
    import torch
    from grf_amd import pipeline as P
    from grf_amd.engine import DeviceCSR
    from grf_amd.graphs import powerlaw_graph

    t0 = time.time()
    n, m, L, p, kr = 1_000_000, 64, 8, 0.1, 8192
    A = powerlaw_graph(n, 10.0, 2.5, seed=0)
    f = _diffusion(L)
    pl = P.plan_step(n, m, L, p, f, k_rows=kr)
    assert pl.mode == "cols" and pl.block_rows == kr
    K, fr = P.kernel_step(eng, DeviceCSR.from_scipy(A, eng.device), pl)
    torch.cuda.synchronize()
    Kv = P.k_view(K, pl)  # n x 8192
    ref = _oracle_phi(A, m, p, L, f)
    print(f"[c5] gpu + oracle Phi {time.time() - t0:.1f} s, nnz {ref.nnz}", flush=True)
    _assert_phi32_equal(fr.phi, ref)
    parts = _bound_parts(ref)
    cols = np.arange(kr)
    deg = np.diff(A.indptr)
    rng = np.random.default_rng(6)
    rows = np.unique(np.concatenate([np.arange(32), np.arange(kr - 32, kr + 32), np.arange(n - 32, n),
                                     np.argsort(-deg, kind="stable")[:32], rng.integers(0, n, 256)]))
    for chunk in np.array_split(rows, max(1, len(rows) // 128)):
        ok, e, nbad = _rows_close(Kv[torch.from_numpy(chunk).to(K.device)].cpu().numpy(), ref, chunk, cols,
                                  parts=parts)
        assert ok, (e, nbad, chunk[:4])
    # the whole block: K_blk 1 (row sums over the 8192 columns) and K_blk^T v (column sums weighted)
    u = rng.choice([-1.0, 1.0], kr)
    ok, worst = _matvec_close(_k_matvec(Kv, u), ref, u, cols=cols, parts=parts)
    assert ok, worst
    v = rng.choice([-1.0, 1.0], n)
    absphi, rowmax, amax = parts
    got = _kt_matvec(Kv, v)
    want = ref[cols] @ (ref.T @ v)
    bound = 3e-5 * (absphi[cols] @ (absphi.T @ np.abs(v))) + 1e-12 * amax * n * rowmax.max() + 1e-7 * np.abs(want)
    assert np.all(np.abs(got - want) <= bound), float((np.abs(got - want) / bound).max())
    print(f"[c5] rows, block matvecs ok {time.time() - t0:.1f} s", flush=True)
    del K, Kv


def test_c3_dense_leg_cora(eng):
    """C3: Cora through the dense path exactly as bench.py (--workload c3 / the MFMA leg) runs it:
    numpy-semantics dense Laplacian -> fused Philox walks -> Phi (dense sampler's divide-by-m rule)
    -> the padded rows straight to the dense Phi (grf_densify_padded, the bench's front) -> MFMA Gram; the
    dense Phi also equals compact + densify bit for bit.  Oracle: the dense Laplacian, the same walks,
    NORM_DIV steps, Phi, K."""
    import torch
    from grf_amd import _lib as C
    from bench import cora_adjacency

    W = cora_adjacency()
    n, m, L, p = W.shape[0], 128, 8, 0.1
    f = _diffusion(L)
    G = eng.walk_matrix_dense(torch.from_numpy(W).to(eng.device), C.LAP_NUMPY)
    rows = eng.walk_phi(G, m, p, L, f, seed=42, norm=C.NORM_DIV, want64=False)
    phi = eng.compact(rows, want64=False)
    dense = eng.densify_padded(rows)
    assert torch.equal(dense, eng.densify(phi))
    K = eng.gram_dense(dense, n).cpu().numpy()
    ip, ix, dx = O.dense_to_walk_csr(O.laplacian_dense(W, 0))
    node, load = O.walk_slots(ip, ix, dx, m, p, L, rng=O.RNG_PHILOX, seed=42, n_threads=N_THREADS)
    ref = O.phi_sparse(O.reduce_steps(node, load, O.NORM_DIV), f)
    _assert_phi32_equal(phi, ref)
    ok, e, nbad = _rows_close(K, ref, np.arange(n))
    assert ok, (e, nbad)
    assert np.array_equal(K, K.T)


def test_c3_dense_leg_cora_split_gram(eng):
    """C3's Gram on the bf16 three-plane split (grf_gram_dense_split, bench.py --gram-precision split):
    the same Cora operand as test_c3_dense_leg_cora, K against the oracle's Phi within the same bound
    as the fp32 path, its error against fp64 beside the fp32 path's, exactly symmetric."""
    import torch
    from grf_amd import _lib as C
    from bench import cora_adjacency

    W = cora_adjacency()
    n, m, L, p = W.shape[0], 128, 8, 0.1
    f = _diffusion(L)
    G = eng.walk_matrix_dense(torch.from_numpy(W).to(eng.device), C.LAP_NUMPY)
    dense = eng.densify_padded(eng.walk_phi(G, m, p, L, f, seed=42, norm=C.NORM_DIV, want64=False))
    Ks = eng.gram_dense(dense, n, precision="split")
    Kf = eng.gram_dense(dense, n, precision="fp32")
    P = dense[:, :n].double()
    ref = P @ P.t()
    bound = P.abs() @ P.abs().t() + 1e-30
    es = float(((Ks.double() - ref).abs() / bound).max())
    ef = float(((Kf.double() - ref).abs() / bound).max())
    print(f"[c3 split] max err / sum|ab|: split {es:.3e}, fp32 {ef:.3e}", flush=True)
    assert es <= 1e-5 and es <= 8.0 * ef + 1e-9, (es, ef)
    ip, ix, dx = O.dense_to_walk_csr(O.laplacian_dense(W, 0))
    node, load = O.walk_slots(ip, ix, dx, m, p, L, rng=O.RNG_PHILOX, seed=42, n_threads=N_THREADS)
    ref_phi = O.phi_sparse(O.reduce_steps(node, load, O.NORM_DIV), f)
    Kn = Ks.cpu().numpy()
    ok, e, nbad = _rows_close(Kn, ref_phi, np.arange(n))
    assert ok, (e, nbad)
    assert np.array_equal(Kn, Kn.T)


def test_dense_path_bench_pipelined_line():
    """bench.py's dense-path workload (C3) pipelined: the next step's front on a side stream beside this
    step's MFMA Gram.  The line keeps the contract fields, reports the pipelining, the serial latency
    beside it and the Gram's roofline from its time alone (the C3 parity of the same kernels:
    test_c3_dense_leg_cora)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {}
    for flag in ("", "--no-overlap"):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--workload", "c3", "--steps", "5",
                            "--warmup", "1", "--no-cpu-baseline"] + ([flag] if flag else []),
                           cwd=root, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out[flag] = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    pipe, ser = out[""], out["--no-overlap"]
    assert pipe["pipelined"] is True and ser["pipelined"] is False
    for d in (pipe, ser):
        assert d["unit"] == "K-matrices/s" and d["value"] > 0 and d["ms_per_step"] > 0 and d["serial_ms_per_step"] > 0
        rf = d["roofline"]
        assert rf["bound"] == "mfma" and 0 < rf["frac"] < 1 and rf["kernel_ms"] > 0 and rf["kernel_ms_pipelined"] > 0


