"""GPU parity: every HIP stage against the CPU oracle (and, through it, the reference).

Tolerances
  * Laplacian, walk slots, step rows, Phi (fp64): bit-exact.
  * K = Phi Phi^T in float32 against the fp64 oracle, elementwise
      |dK_ij| <= 3e-5 (|Phi| |Phi|^T)_ij + 1e-12 max_k|Phi_ik| max|Phi|
    (fp32 rounding of Phi's entries, fp32 output rounding, and the sparse kernel's
    int64 fixed-point resolution of 2^-50 per term), and relative Frobenius error <= 1e-6.  The sparse Gram kernel is
    much tighter than that (fp32 rounding of Phi's entries, then an exact
    fixed-point sum rounded once), the MFMA dense Gram is an fp32 FMA chain.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from golden_util import csr, same_csr
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    from grf_amd.engine import GRFEngine
    return GRFEngine("cuda:0")


def er_graph(n, avg_deg, seed, weighted=False):
    r = np.random.default_rng(seed)
    m = int(n * avg_deg / 2)
    u = r.integers(0, n, m)
    v = r.integers(0, n, m)
    keep = u != v
    u, v = u[keep], v[keep]
    w = r.uniform(0.2, 3.0, len(u)) if weighted else np.ones(len(u))
    A = sp.coo_matrix((w, (u, v)), shape=(n, n)).tocsr()
    A = (A + A.T).tocsr()
    if not weighted:
        A.data[:] = 1.0
    A.sum_duplicates()
    A.sort_indices()
    return A


def bit_equal(a, b):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def slots_equal(gpu, ora):
    gn, gl = gpu.node.cpu().numpy(), gpu.load.cpu().numpy()
    on, ol = ora
    if not np.array_equal(gn, on):
        return False
    mask = on >= 0
    return bit_equal(gl[mask], ol[mask])


def gram_close(K, phi64, rows=None):
    r0, r1 = rows or (0, phi64.shape[0])
    Kref = O.gram_rows(phi64, r0, r1)
    absphi = abs(phi64)
    bound = O.gram_rows(absphi, r0, r1)
    # fixed-point resolution of the sparse Gram kernel: 2^-50 max_k|Phi_ik| max|Phi| per term
    rowmax = np.asarray(absphi.max(axis=1).todense()).ravel()
    # (a mirrored entry K[j, i] of the symmetric mode carries row i's resolution)
    fx = 1e-12 * np.maximum(rowmax[r0:r1, None], rowmax[None, :]) * absphi.max()
    err = np.abs(np.asarray(K, np.float64) - Kref)
    ok_elem = bool(np.all(err <= 3e-5 * bound + fx + 1e-30))
    fro = np.linalg.norm(err) / max(np.linalg.norm(Kref), 1e-300)
    return ok_elem and fro <= 1e-6, fro


# ----------------------------------------------------------------- Laplacians
def test_laplacian_sparse_golden(eng, golden):
    d = golden("small_graphs")
    for name in d["names"]:
        A = d[f"{name}_A"]
        L = eng.laplacian(sp.csr_matrix(A)).to_scipy()
        assert same_csr(L, csr(d, f"{name}_Lsp", A.shape[0])), name


def test_laplacian_sparse_random(eng):
    for seed, weighted in [(0, False), (1, True), (2, True)]:
        A = er_graph(3000, 12, seed, weighted)
        A = A.tolil()
        A[5, :] = 0
        A[:, 5] = 0
        A = A.tocsr()
        A.eliminate_zeros()
        ref, _ = O.laplacian_sparse(A)
        got = eng.laplacian(A).to_scipy()
        assert same_csr(got, ref), seed


def _sparse_laplacian_cases():
    """CSR adjacencies (sorted columns, explicit entries kept as given) that reach every branch of the
    eight-rows-per-wave Laplacian kernels (grf_laplacian.hip): group rows of every length 0..63 and the
    leaf's tail sizes, whole-wave rows (>= 64 entries) and degree sums past one numpy leaf (> 129 entries),
    integral and non-integral weights, explicit / inserted / cancelling diagonals, zero and negative
    degrees, explicit zeros and -0.0 entries."""
    r = np.random.default_rng(17)
    lengths = [0, 1, 2, 5, 7, 8, 9, 15, 16, 17, 31, 62, 63, 64, 65, 127, 128, 129, 130, 131, 200, 300, 700]
    cases = {}
    for name, unit in (("mixed_weighted", False), ("mixed_unit", True)):
        n = 2300
        ptr, idx = [0], []
        for i in range(n):
            k = lengths[(i * 7) % len(lengths)]
            idx.extend(np.sort(r.choice(n, k, replace=False)).tolist())
            ptr.append(len(idx))
        val = np.ones(len(idx)) if unit else r.uniform(0.1, 2.0, len(idx))
        cases[name] = sp.csr_matrix((val, np.asarray(idx, np.int32), np.asarray(ptr, np.int64)), shape=(n, n))
    n = 600
    ptr, idx, val = [0], [], []
    for i in range(n):
        kind = i % 8
        cols = np.sort(r.choice(n, int(r.integers(1, 90)), replace=False))
        v = r.uniform(-1.0, 2.0, len(cols))
        if kind == 0:  # the diagonal alone: d - a_ii = 0 (dropped)
            cols, v = np.array([i]), np.array([2.5])
        elif kind == 1:  # +1 / -1: degree 0 (D^-1/2 = 0, nothing inserted)
            cols = np.array(sorted({(i + 1) % n, (i + 2) % n}))
            v = np.array([1.0, -1.0])
        elif kind == 2:  # explicit zeros and -0.0 among the entries
            v[::3] = 0.0
            v[1::5] = -0.0
        elif kind == 3:  # negative degree (D^-1/2 NaN)
            v = -np.abs(v) - 0.1
        elif kind == 4:  # an explicit diagonal inside the row
            cols = np.unique(np.append(cols, i))
            v = r.uniform(0.1, 2.0, len(cols))
        idx.extend(cols.tolist())
        val.extend(np.asarray(v, np.float64).tolist())
        ptr.append(len(idx))
    cases["signed_diag"] = sp.csr_matrix((np.asarray(val), np.asarray(idx, np.int32), np.asarray(ptr, np.int64)),
                                         shape=(n, n))
    return cases


@pytest.mark.parametrize("name", ["mixed_weighted", "mixed_unit", "signed_diag"])
def test_laplacian_sparse_group_branches(eng, name):
    """The sparse (scipy-semantics) Laplacian bit-exact against the oracle, row pointer included, on rows
    of every length class and the diagonal / zero / sign cases above."""
    A = _sparse_laplacian_cases()[name]
    ref, _ = O.laplacian_sparse(A)
    got = eng.laplacian(A).to_scipy()
    assert same_csr(got, ref), name


def test_laplacian_dense_modes(eng, golden):
    d = golden("small_graphs")
    for name in d["names"]:
        A = d[f"{name}_A"]
        for mode, key, ref_mode in ((1, "Ld", 0), (2, "Lnp", 1), (3, "Lcomb", 2)):
            G = eng.walk_matrix_dense(A, mode).to_scipy()
            ip, ix, dx = O.dense_to_walk_csr(d[f"{name}_{key}"])
            assert np.array_equal(G.indptr, ip) and np.array_equal(G.indices, ix), (name, key)
            assert bit_equal(G.data, dx), (name, key)
    r = np.random.default_rng(3)
    W = r.random((700, 700)) * (r.random((700, 700)) < 0.05)
    W = W + W.T
    for mode, ref_mode in ((1, 0), (2, 1), (3, 2)):
        G = eng.walk_matrix_dense(W, mode).to_scipy()
        ip, ix, dx = O.dense_to_walk_csr(O.laplacian_dense(W, ref_mode))
        assert np.array_equal(G.indices, ix) and bit_equal(G.data, dx), mode


def _dense_laplacian_cases():
    """Dense adjacencies that reach every branch of the stage / emit kernels (grf_laplacian.hip)."""
    r = np.random.default_rng(11)
    cases = {}
    # fully dense weighted rows: > 127 structural nonzeros (emit re-reads W), non-integral degrees
    # (numpy's plan), n odd (rows alternately start mid-16-B)
    W = r.random((301, 301))
    cases["dense_weighted_odd"] = W + W.T
    # sparse 0/1, odd n: the exact integer degree, staged rows, the diagonal inserted
    A = (r.random((1001, 1001)) < 0.004).astype(np.float64)
    A = np.maximum(A, A.T)
    np.fill_diagonal(A, 0.0)
    cases["unit_sparse_odd"] = A
    # asymmetric with zero rows, negative weights (degrees <= 0: D^-1/2 = 0 or the safe 1), explicit
    # diagonal entries and -0.0 entries
    B = (r.random((257, 257)) < 0.03) * r.uniform(-1.0, 2.0, (257, 257))
    B[5] = 0.0
    B[7] = -0.0
    B[9, 9] = 3.0
    B[10, :12] = -1.0
    cases["asym_signed"] = B
    # rows of mixed lengths around the stage's cap (127 staged + the diagonal)
    C = np.zeros((400, 400))
    for i in range(400):
        k = [0, 1, 126, 127, 128, 200][i % 6]
        C[i, r.choice(400, k, replace=False)] = 1.0
    cases["cap_edges"] = C
    # n > 8192 with weighted rows: the degree recursion beyond the host plan (wave_np_pairwise)
    D = np.zeros((8300, 8300))
    idx = r.integers(0, 8300, (8300, 12))
    D[np.arange(8300)[:, None], idx] = r.uniform(0.1, 2.0, (8300, 12))
    cases["large_weighted"] = D
    return cases


@pytest.mark.parametrize("name", ["dense_weighted_odd", "unit_sparse_odd", "asym_signed", "cap_edges", "large_weighted"])
def test_laplacian_dense_stage_emit_branches(eng, name):
    """The one-read dense Laplacian (stage + look-back emit) bit-exact against the oracle in every mode,
    row pointer included, on inputs that take each branch: exact-integer and recursion degrees, the
    host plan and wave_np_pairwise, staged rows and rows re-read from W, rows at the stage's cap,
    unaligned rows, zero / negative degrees, explicit and inserted diagonals."""
    W = _dense_laplacian_cases()[name]
    for mode, ref_mode in ((1, 0), (2, 1), (3, 2), (4, None)):
        G = eng.walk_matrix_dense(W, mode).to_scipy()
        ip, ix, dx = O.dense_to_walk_csr(W if ref_mode is None else O.laplacian_dense(W, ref_mode))
        assert np.array_equal(G.indptr, ip), (name, mode)
        assert np.array_equal(G.indices, ix) and bit_equal(G.data, dx), (name, mode)


# ---------------------------------------------------------------------- walks
@pytest.mark.parametrize("rule", [0, 1, 2])
def test_walk_philox_matches_oracle(eng, rule):
    A = er_graph(2000, 10, 4)
    Ls, _ = O.laplacian_sparse(A)
    G = eng.laplacian(A)
    ip, ix, dx = O._csr_arrays(Ls)
    for m, p, L, seed in [(16, 0.1, 8, 7), (33, 0.3, 5, 2**40 + 3), (1, 0.0, 3, 0)]:
        got = eng.walk(G, m, p, L, rng=1, seed=seed, load_rule=rule)
        ref = O.walk_slots(ip, ix, dx, m, p, L, rng=O.RNG_PHILOX, load_rule=rule, seed=seed)
        assert slots_equal(got, ref), (m, p, L, seed)


def test_walk_philox_shard_invariant(eng):
    A = er_graph(1500, 8, 5)
    G = eng.laplacian(A)
    full = eng.walk(G, 24, 0.15, 6, rng=1, seed=99)
    a = eng.walk(G, 24, 0.15, 6, rng=1, seed=99, src_begin=0, src_end=700)
    b = eng.walk(G, 24, 0.15, 6, rng=1, seed=99, src_begin=700, src_end=1500)
    import torch
    assert torch.equal(full.node, torch.cat([a.node, b.node]))
    mask = full.node >= 0
    assert torch.equal(full.load[mask], torch.cat([a.load, b.load])[mask])


@pytest.mark.parametrize("n_chunks", [1, 3, 8, 64])
def test_walk_pcg64_matches_oracle(eng, n_chunks):
    A = er_graph(800, 9, 6, weighted=True)
    Ls, _ = O.laplacian_sparse(A)
    G = eng.laplacian(A)
    ip, ix, dx = O._csr_arrays(Ls)
    got = eng.walk(G, 20, 0.2, 6, rng=0, seed=42, n_chunks=n_chunks)
    ref = O.walk_slots(ip, ix, dx, 20, 0.2, 6, rng=O.RNG_PCG64, n_chunks=n_chunks, seed=42)
    assert slots_equal(got, ref)


def test_pcg64_sampler_reproduces_reference_golden(eng, golden):
    """GPU reference-stream mode gives the reference's step matrices bit-for-bit."""
    d = golden("small_graphs")
    for name in d["names"]:
        n = d[f"{name}_A"].shape[0]
        Ls = csr(d, f"{name}_Lsp", n)
        p = 0.0 if name == "perm12" else 0.2
        G = eng.to_device(Ls)
        for nproc in (1, 3, 8):
            for seed in (None, 7):
                slots = eng.walk(G, 20, p, 4, rng=0, seed=(seed or 42), n_chunks=nproc)
                mats = eng.step_matrices(eng.steps(slots, norm=1))
                for l, M in enumerate(mats):
                    assert same_csr(M.to_scipy(), csr(d, f"{name}_sp_n{nproc}_s{seed}_l{l}", n)), (name, nproc, l)


def test_cora_m128_reference_digests(eng, golden):
    from golden_util import digest
    d = golden("cora")
    n = len(d["A_indptr"]) - 1
    G = eng.laplacian(csr(d, "A", n))
    assert digest(G.to_scipy()) == str(d["L_digest"][0])
    slots = eng.walk(G, 128, 0.1, 8, rng=0, seed=42, n_chunks=8)
    mats = eng.step_matrices(eng.steps(slots, norm=1))
    assert [digest(M.to_scipy()) for M in mats] == [str(x) for x in d["m128_digests"]]
    f = np.array([(-1.0) ** l / (2.0 ** l * float(np.prod(np.arange(1, l + 1)))) for l in range(8)])
    phi = eng.compact(eng.features(slots, f))
    assert digest(phi.to_scipy()) == str(d["m128_phi_digest"][0])
    K = eng.gram(phi, "sparse").cpu().numpy()
    np.testing.assert_allclose(K[:16], d["m128_K_rows0_16"], rtol=3e-5, atol=1e-6)
    np.testing.assert_allclose(np.diag(K), d["m128_K_diag"], rtol=3e-5)
    Kd = eng.gram(phi, "dense").cpu().numpy()
    np.testing.assert_allclose(Kd[:16], d["m128_K_rows0_16"], rtol=3e-5, atol=1e-6)


# -------------------------------------------------------------- steps / Phi
@pytest.mark.parametrize("m,L,p", [(16, 8, 0.1), (128, 8, 0.1), (50, 3, 0.1), (300, 4, 0.05), (7, 20, 0.02),
                                   (600, 8, 0.2)])  # (m L = 4800 > 4096: steps + phi, no fused kernel)
def test_steps_and_phi_bitexact(eng, m, L, p):
    A = er_graph(600, 7, m + L)
    Ls, _ = O.laplacian_sparse(A)
    G = eng.laplacian(A)
    slots = eng.walk(G, m, p, L, rng=1, seed=5)
    node, load = slots.node.cpu().numpy(), slots.load.cpu().numpy()
    load = np.where(node >= 0, load, 0.0)
    f = np.random.default_rng(m).standard_normal(L + 1)
    for norm in (0, 1):
        ref_steps = O.reduce_steps(node, load, norm)
        st = eng.steps(slots, norm)
        mats = eng.step_matrices(st)
        for l in range(L):
            assert same_csr(mats[l].to_scipy(), ref_steps[l]), (norm, l)
        ref_phi = O.phi_sparse(ref_steps, f[:L - 1])
        got = eng.compact(eng.phi(st, f[:L - 1])).to_scipy()
        assert same_csr(got, ref_phi), norm
        if m * L <= 4096:
            fused = eng.compact(eng.phi_fused(slots, f[:L - 1], norm)).to_scipy()
            assert same_csr(fused, ref_phi), norm


def test_steps_dense_tensor(eng):
    A = er_graph(200, 6, 11)
    G = eng.laplacian(A)
    slots = eng.walk(G, 12, 0.2, 4, rng=1, seed=1)
    st = eng.steps(slots, 0)
    F = eng.steps_dense(st).cpu().numpy()
    mats = [M.to_scipy().toarray() for M in eng.step_matrices(st)]
    for l in range(4):
        assert bit_equal(F[:, :, l], mats[l])


# ----------------------------------------------------------------------- Gram
@pytest.mark.parametrize("n,deg,m,L,bw", [(1000, 8, 32, 6, 64), (5000, 10, 64, 8, 256), (3000, 4, 16, 5, 8192), (777, 5, 8, 3, 128), (20000, 10, 32, 6, 4096), (4100, 6, 16, 4, 1024)])
def test_gram_sparse_vs_oracle(eng, n, deg, m, L, bw):
    A = er_graph(n, deg, n)
    G = eng.laplacian(A)
    slots = eng.walk(G, m, 0.1, L, rng=1, seed=3)
    f = [(-1.0) ** l / 2 ** l for l in range(L)]
    phi = eng.compact(eng.features(slots, f))
    tr = eng.transpose_banded(phi, bw)
    K = eng.gram_sparse(phi, tr).cpu().numpy()
    ok, fro = gram_close(K, phi.to_scipy())
    assert ok, fro
    # row block, and a rerun: bit-identical (fixed summation order)
    Kb = eng.gram_sparse(phi, tr, 17, 300).cpu().numpy()
    assert np.array_equal(Kb, K[17:300])
    assert np.array_equal(eng.gram_sparse(phi, eng.transpose_banded(phi, bw)).cpu().numpy(), K)
    # symmetric mode: the upper triangle is the same bits; the lower triangle is its mirror
    Ks = eng.gram_sparse_sym(phi, tr).cpu().numpy()
    assert np.array_equal(Ks, Ks.T)
    if bw % 64 == 0:  # the two halves of the symmetric mode, as the pipelined bench issues them
        import torch
        Ku = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
        eng.gram_sparse_upper(phi, tr, Ku, parts=(0, 7, 10))
        eng.gram_sparse_upper(phi, tr, Ku, parts=(7, 10, 10))
        assert np.array_equal(eng.gram_mirror(Ku, n, max_workgroups=37).cpu().numpy(), Ks)  # (grid-stride)
    upper = np.triu(np.ones((n, n), bool))
    assert np.array_equal(Ks[upper], K[upper])
    ok, fro = gram_close(Ks, phi.to_scipy())
    assert ok, fro


def test_gram_sparse_band_invariance(eng):
    """The int64 fixed-point K is independent of the band width (many small tiles vs few wide
    ones, 313 bands at W = 64) -- bit for bit."""
    n = 20000
    A = er_graph(n, 6, 99)
    G = eng.laplacian(A)
    slots = eng.walk(G, 4, 0.3, 3, rng=1, seed=5)
    phi = eng.compact(eng.features(slots, [1.0, -0.5, 0.25]))
    K_wide = eng.gram_sparse(phi, eng.transpose_banded(phi, 4096)).cpu().numpy()
    K_narrow = eng.gram_sparse(phi, eng.transpose_banded(phi, 64)).cpu().numpy()
    assert np.array_equal(K_wide, K_narrow)
    # 8192-wide bands run 8-wave tiles (76 KiB of LDS): the same bits
    K_8k = eng.gram_sparse(phi, eng.transpose_banded(phi, 8192)).cpu().numpy()
    assert np.array_equal(K_wide, K_8k)
    ok, fro = gram_close(K_wide[:16], phi.to_scipy(), (0, 16))
    assert ok, fro


@pytest.mark.parametrize("unit", [128, 12])
@pytest.mark.parametrize("n,deg,m,L,bw", [(20000, 10, 32, 6, 4096), (5000, 10, 64, 8, 64), (3000, 20, 128, 8, 4096),
                                          (4100, 6, 16, 4, 1024)])
def test_transpose_staged_fill_matches_atomic_fill(eng, n, deg, m, L, bw, unit):
    """The binned two-pass fill (LDS region images; the dense 3000-node case overflows the LDS
    cap and takes the global-cursor fallback) gives the same descriptors, the same multiset of
    records per bucket, the same row shifts -- hence bit-identical K -- in both record layouts
    (buckets on 128-byte lines and packed 12-byte pairs), and the two layouts give the same K."""
    A = er_graph(n, deg, n + 7)
    G = eng.laplacian(A)
    phi = eng.compact(eng.walk_phi(G, m, 0.15, L, [1.0, -0.5, 0.25, -0.125, 0.1, -0.05, 0.02, -0.01][:L], seed=4))
    ta = eng.transpose_banded(phi, bw, staged=False, rec_unit=unit)
    ts = eng.transpose_banded(phi, bw, staged=True, rec_unit=unit, self_count=False)
    tself = eng.transpose_banded(phi, bw, rec_unit=unit, self_count=True) if bw % 64 == 0 else ts
    assert ta.rec_unit == ts.rec_unit == tself.rec_unit == unit
    assert np.array_equal(ta.t_desc.cpu().numpy(), ts.t_desc.cpu().numpy())
    for t in (ts, tself):
        assert np.array_equal(ta.t_rowshift.cpu().numpy(), t.t_rowshift.cpu().numpy())
        assert ta.t_maxabs.item() == t.t_maxabs.item()
    desc = ta.t_desc.cpu().numpy().view(np.uint32).reshape(-1, 2)
    dself = tself.t_desc.cpu().numpy().view(np.uint32).reshape(-1, 2)
    nb = -(-n // bw)
    assert np.array_equal(desc[:nb * n, 1], dself[:nb * n, 1])  # same pairs per bucket
    # the slabs keep (band, column) order: first units never decrease within a band
    assert all(np.all(np.diff(dself[J * n:(J + 1) * n, 0].astype(np.int64)) >= 0) for J in range(nb))
    ra, rs, rself = ta.t_rec.cpu().numpy(), ts.t_rec.cpu().numpy(), tself.t_rec.cpu().numpy()
    rng = np.random.default_rng(0)
    for b in rng.choice(nb * n, size=min(nb * n, 3000), replace=False):
        pairs = int(desc[b, 1])
        if pairs == 0:
            continue

        def recs(buf, line):
            seg = buf[line * unit: line * unit + 12 * pairs].reshape(pairs, 12)
            cols = seg[:, :4].copy().view(np.uint16).reshape(pairs, 2)
            vals = seg[:, 4:].copy().view(np.float32).reshape(pairs, 2)
            return sorted(zip(cols.ravel().tolist(), vals.ravel().tolist()))
        assert recs(ra, int(desc[b, 0])) == recs(rs, int(desc[b, 0])) == recs(rself, int(dself[b, 0])), b
    Ka = eng.gram_sparse(phi, ta, 0, 300).cpu().numpy()
    Ks = eng.gram_sparse(phi, ts, 0, 300).cpu().numpy()
    assert np.array_equal(Ka, Ks)
    assert np.array_equal(eng.gram_sparse(phi, tself, 0, 300).cpu().numpy(), Ka)
    other = eng.transpose_banded(phi, bw, rec_unit=140 - unit)  # the other layout
    assert np.array_equal(eng.gram_sparse(phi, other, 0, 300).cpu().numpy(), Ka)
    if bw % 64 == 0:
        assert np.array_equal(eng.gram_sparse_sym(phi, other).cpu().numpy(), eng.gram_sparse_sym(phi, ts).cpu().numpy())


@pytest.mark.parametrize("n,bw,unit", [(20000, 4096, 128), (20000, 8192, 128), (5000, 64, 128), (9000, 1024, 12),
                                        (3000, 4096, 128)])
def test_transpose_sub_band_split(eng, n, bw, unit):
    """The self-count transpose's sub-band split: every bucket lists its entries by sub-band (the 8
    row ranges of bw / 8 rows, in order) and t_split holds the entry offsets of the sub-bands; the
    symmetric Gram's diagonal tiles start their buckets at their row's sub-band (no pairs of the
    earlier sub-bands fetched) -- K is bit-identical to the unsplit transpose's in every symmetric
    entry point (whole K, the upper tiles in parts + mirror, the column block's square, the row
    block's interior, the hub-column split), because the skipped products only reach entries below
    the diagonal, which the mirror overwrites."""
    import torch
    A = er_graph(n, 8, n + 3)
    G = eng.laplacian(A)
    phi = eng.compact(eng.walk_phi(G, 32, 0.15, 5, [1.0, -0.5, 0.25, -0.125, 0.1], seed=9))
    ts = eng.transpose_banded(phi, bw, rec_unit=unit, split=True)
    tn = eng.transpose_banded(phi, bw, rec_unit=unit)
    assert ts.t_split is not None and tn.t_split is None
    nb = -(-n // bw)
    desc = ts.t_desc.cpu().numpy().view(np.uint32).reshape(-1, 2)
    split = ts.t_split.cpu().numpy().view(np.uint16).reshape(-1, 8).astype(np.int64)
    rec = ts.t_rec.cpu().numpy()
    P = phi.to_scipy().tocsc()
    rng = np.random.default_rng(1)
    for b in rng.choice(nb * n, size=min(nb * n, 2000), replace=False):
        J, k = divmod(int(b), n)
        lo, hi = J * bw, min(n, (J + 1) * bw)
        rows = P.indices[P.indptr[k]:P.indptr[k + 1]]
        rows = rows[(rows >= lo) & (rows < hi)] - lo
        c = len(rows)
        assert int(desc[b, 1]) == (c + 1) // 2
        if c == 0:
            continue
        seg = rec[int(desc[b, 0]) * unit: int(desc[b, 0]) * unit + 12 * ((c + 1) // 2)].reshape(-1, 12)
        got = seg[:, :4].copy().view(np.uint16).reshape(-1)[:c].astype(np.int64) // 8  # rows in the band
        sub = got * 8 // bw
        assert np.all(np.diff(sub) >= 0), b  # sub-band order
        exp = np.searchsorted(sub, np.arange(8), side="left")
        if split[b].any():  # (0 everywhere: a region over the LDS image cap, order unspecified)
            assert np.array_equal(split[b], exp), b
        assert sorted(got.tolist()) == sorted(rows.tolist())
    Ks = eng.gram_sparse_sym(phi, ts)
    assert torch.equal(Ks, eng.gram_sparse_sym(phi, tn))
    Ku = torch.full((n, eng.leading_dim(n)), float("nan"), dtype=torch.float32, device=eng.device)
    eng.gram_sparse_upper(phi, ts, Ku, parts=(0, 3, 7))
    eng.gram_sparse_upper(phi, ts, Ku, parts=(3, 7, 7))
    assert torch.equal(eng.gram_mirror(Ku, n), Ks)
    # column block with its symmetric square (rows [b, e) transposed with their own bands)
    b, e = n // 4, n // 4 + min(n // 2, 3 * bw // 2)
    loc = eng.compact(eng.walk_phi(G, 32, 0.15, 5, [1.0, -0.5, 0.25, -0.125, 0.1], seed=9, src_begin=b, src_end=e))
    sh = eng.phi_row_shifts(phi)
    Kc = eng.gram_sparse_cols(phi, sh, eng.transpose_banded(loc, bw, rec_unit=unit, split=True), sym_row0=b)
    Kn = eng.gram_sparse_cols(phi, sh, eng.transpose_banded(loc, bw, rec_unit=unit), sym_row0=b)
    assert torch.equal(Kc, Kn)
    # the hub-column split adds to the dense panel's K with the same skip
    if unit == 128 and bw >= 1024:
        Kh = eng.gram_sparse_sym_hubs(phi, eng.transpose_banded(phi, bw, split=True), 32)
        Khn = eng.gram_sparse_sym_hubs(phi, eng.transpose_banded(phi, bw), 32)
        assert torch.equal(Kh, Khn)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_gram_kslice_partials_sum_to_K(eng, world):
    """The all-reduce option: partial Grams over disjoint inner-dimension slices
    are each exact against the oracle's column-restricted Gram and sum to K (fp32 sum of fp32
    partials: within the fp32 tolerance of gram_close)."""
    from grf_amd.dist import shard_range
    n = 3000
    A = er_graph(n, 8, 11)
    G = eng.laplacian(A)
    phi = eng.compact(eng.features(eng.walk(G, 16, 0.2, 4, rng=1, seed=9), [1.0, -0.5, 0.25, -0.125]))
    tr = eng.transpose_banded(phi, 1024)
    phi64 = phi.to_scipy()
    Ksum = np.zeros((n, n), np.float64)
    for r in range(world):
        kb, ke = shard_range(n, r, world)
        Kr = eng.gram_sparse_kslice(phi, tr, kb, ke).cpu().numpy()
        mask = np.zeros(n)
        mask[kb:ke] = 1.0
        sub = (phi64 @ sp.diags(mask)).tocsr()
        ok, fro = gram_close(Kr, sub)
        assert ok, (r, fro)
        Ksum += Kr
    ok, fro = gram_close(Ksum, phi64)
    assert ok, fro
    if world == 1:
        assert np.array_equal(Ksum.astype(np.float32), eng.gram_sparse(phi, tr).cpu().numpy())
    # a row block of a slice is the same bits as those rows of the whole slice
    kb, ke = shard_range(n, 0, world)
    assert np.array_equal(eng.gram_sparse_kslice(phi, tr, kb, ke, 100, 400).cpu().numpy(),
                          eng.gram_sparse_kslice(phi, tr, kb, ke).cpu().numpy()[100:400])


@pytest.mark.parametrize("n", [1, 31, 64, 65, 128, 1000, 2708, 4500])
def test_gram_dense_mfma_vs_oracle(eng, n):
    A = er_graph(max(n, 2), 6, n + 1)[:n, :n]
    G = eng.laplacian(A)
    slots = eng.walk(G, 24, 0.15, 5, rng=1, seed=2)
    phi = eng.compact(eng.features(slots, [1.0, -0.5, 0.25, -0.125, 0.0625]))
    K = eng.gram(phi, "dense").cpu().numpy()
    ok, fro = gram_close(K, phi.to_scipy())
    assert ok, fro
    assert np.array_equal(K, K.T)  # (upper tiles + mirror: exactly symmetric)


def test_gram_dense_asymmetric_layout(eng):
    """A = I-style check with an asymmetric operand: catches row/col swaps in the MFMA C map."""
    import torch
    n = 160
    Ad = np.zeros((n, 176), np.float32)
    r = np.random.default_rng(0)
    Ad[:, :150] = r.standard_normal((n, 150)).astype(np.float32)
    At = torch.from_numpy(Ad).cuda()
    K = eng.gram_dense(At, 150).cpu().numpy()
    ref = Ad.astype(np.float64) @ Ad.astype(np.float64).T
    np.testing.assert_allclose(K, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("n,k", [(300, 900), (2708, 2708), (1500, 4000), (4200, 1000), (4200, 20), (5000, 4999)])
def test_gram_dense_split_k(eng, n, k):
    """Split-K dense Gram against fp64 and against the unsplit kernel (no workspace); exactly symmetric,
    run-to-run identical.  Small n: every tile cut into k-slices summed in order by the last piece; from
    256 tiles on (n >= 4200 here) the stream-K slots, whose pieces span slot boundaries -- k = 20 gives
    tiles of 2 k-tiles over slots of 3, so most tiles are cut."""
    import torch
    from grf_amd import _lib as C
    lda = -(-k // 64) * 64
    Ad = np.zeros((n, lda), np.float32)
    r = np.random.default_rng(n)
    Ad[:, :k] = (r.standard_normal((n, k)) * (r.random((n, k)) < 0.1)).astype(np.float32)
    At = torch.from_numpy(Ad).to(eng.device)
    assert eng.lib.grf_gram_dense_workspace_bytes(n, k) > 16  # (the split path is taken)
    Ks = eng.gram_dense(At, k)
    K1 = torch.empty((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
    C.check(eng.lib.grf_gram_dense(n, k, At.data_ptr(), lda, K1.data_ptr(), K1.stride(0), eng.stream),
            "grf_gram_dense")
    ref = Ad.astype(np.float64) @ Ad.astype(np.float64).T
    bound = np.abs(Ad).astype(np.float64) @ np.abs(Ad).astype(np.float64).T
    for K in (Ks.cpu().numpy(), K1[:, :n].cpu().numpy()):
        assert np.all(np.abs(K - ref) <= 1e-5 * bound + 1e-30)
    Ksn = Ks.cpu().numpy()
    assert np.array_equal(Ksn, Ksn.T)
    assert np.array_equal(eng.gram_dense(At, k).cpu().numpy(), Ksn)


@pytest.mark.parametrize("n,k", [(160, 150), (300, 900), (2708, 2708), (4200, 1000), (4200, 20), (5000, 4999)])
def test_gram_dense_split_vs_fp64_and_fp32(eng, n, k):
    """The bf16 three-plane split Gram (grf_gram_dense_split) against fp64: within the fp32 path's test bound
    (1e-5 of sum |a b|), its typical error within a small factor of the fp32 MFMA path's (fp32-class, not a
    reduced precision), exactly symmetric, run-to-run identical; every decomposition (whole tiles, per-tile
    split-K below 256 tiles, stream-K from 256 on, k of one stage)."""
    import torch
    lda = -(-k // 64) * 64
    Ad = np.zeros((n, lda), np.float32)
    r = np.random.default_rng(n + k)
    # Phi-like: nonnegative entries spread over four decades, and signed ones in every other row
    v = (r.random((n, k)) * 10.0 ** r.uniform(-3, 1, (n, k))) * (r.random((n, k)) < 0.2)
    v[::2] *= np.sign(r.standard_normal((n // 2 + n % 2, k)))
    Ad[:, :k] = v.astype(np.float32)
    At = torch.from_numpy(Ad).to(eng.device)
    Ks = eng.gram_dense(At, k, precision="split")
    Kf = eng.gram_dense(At, k, precision="fp32")
    ref = Ad.astype(np.float64) @ Ad.astype(np.float64).T
    bound = np.abs(Ad).astype(np.float64) @ np.abs(Ad).astype(np.float64).T + 1e-30
    es = np.abs(Ks.cpu().numpy() - ref) / bound
    ef = np.abs(Kf.cpu().numpy() - ref) / bound
    assert es.max() <= 1e-5, es.max()
    assert np.sqrt((es ** 2).mean()) <= 4.0 * np.sqrt((ef ** 2).mean()) + 1e-9, (es.max(), ef.max())
    Ksn = Ks.cpu().numpy()
    assert np.array_equal(Ksn, Ksn.T) and np.isfinite(Ksn).all()
    assert np.array_equal(eng.gram_dense(At, k, precision="split").cpu().numpy(), Ksn)


@pytest.mark.parametrize("n,k", [(100, 37), (300, 900), (1153, 1153), (2708, 2708), (4200, 20), (4200, 1000),
                                 (4500, 16), (8200, 300)])
def test_gram_dense_split_wide(eng, monkeypatch, n, k):
    """The split Gram's wide workgroups (256 x 128 items, stream-K; the default from 64 tile rows on, forced
    here with GRF_DENSE_WIDE=1 at small n): odd tile-row counts (the item's second row block past n), k of
    one or two k-tiles (items cut at many slot boundaries), against fp64 within the fp32 path's bound, against
    the 128-tile split kernel (GRF_DENSE_WIDE=0) within twice that bound, exactly symmetric, run-to-run
    identical, tickets back at zero; at n = 8200 (65 tile rows) the default takes the wide path (same bits as
    forced)."""
    import torch
    lda = -(-k // 64) * 64
    Ad = np.zeros((n, lda), np.float32)
    r = np.random.default_rng(n * 7 + k)
    v = (r.random((n, k)) * 10.0 ** r.uniform(-3, 1, (n, k))) * (r.random((n, k)) < 0.2)
    v[1::2] *= np.sign(r.standard_normal((n // 2, k)))
    Ad[:, :k] = v.astype(np.float32)
    At = torch.from_numpy(Ad).to(eng.device)
    monkeypatch.setenv("GRF_DENSE_WIDE", "1")
    Kw = eng.gram_dense(At, k, precision="split").cpu().numpy()
    Kw2 = eng.gram_dense(At, k, precision="split").cpu().numpy()
    ws = eng._dense_ws[eng.stream.value]
    assert int(ws[:4096].view(torch.int32).abs().sum()) == 0
    monkeypatch.setenv("GRF_DENSE_WIDE", "0")
    Kn = eng.gram_dense(At, k, precision="split").cpu().numpy()
    ref = Ad.astype(np.float64) @ Ad.astype(np.float64).T
    bound = np.abs(Ad).astype(np.float64) @ np.abs(Ad).astype(np.float64).T + 1e-30
    assert (np.abs(Kw - ref) / bound).max() <= 1e-5
    assert (np.abs(Kw.astype(np.float64) - Kn) / bound).max() <= 2e-5
    assert np.isfinite(Kw).all() and np.array_equal(Kw, Kw.T) and np.array_equal(Kw, Kw2)
    monkeypatch.delenv("GRF_DENSE_WIDE")
    Kd = eng.gram_dense(At, k, precision="split").cpu().numpy()
    assert np.array_equal(Kd, Kw if -(-n // 128) >= 64 else Kn)


@pytest.mark.parametrize("planes", ["1", "0"])
@pytest.mark.parametrize("n,k", [(8192, 300), (10000, 160), (11520, 64)])
def test_gram_dense_wide_xcd_rounds(eng, monkeypatch, n, k, planes):
    """The wide kernels' whole-item rounds in XCD-contiguous slot order, then stream-K over the rest
    (sk_plan_wide): 1056 items (a rest of 32 < 64 joins a round: 3 rounds + 288 items cut), 1600 (C2's count:
    6 rounds + 64 items cut in four) and 2070 (7 rounds + 278); the planes kernel (the default here) and the
    in-register split (GRF_DENSE_PLANES=0); against fp64 within the fp32 path's bound, against round 5's
    stream-K-only schedule (GRF_DENSE_XCD=0) within twice that bound, exactly symmetric, run-to-run identical,
    tickets back at zero."""
    import torch
    monkeypatch.setenv("GRF_DENSE_PLANES", planes)
    lda = -(-k // 64) * 64
    g = torch.Generator(device=eng.device).manual_seed(n + k)
    A = torch.zeros((n, lda), dtype=torch.float32, device=eng.device)
    A[:, :k] = torch.rand((n, k), device=eng.device, generator=g) * (
        torch.rand((n, k), device=eng.device, generator=g) < 0.3)
    K1 = eng.gram_dense(A, k, precision="split")
    K2 = eng.gram_dense(A, k, precision="split")
    ws = eng._dense_ws[eng.stream.value]
    assert int(ws[:4096].view(torch.int32).abs().sum()) == 0
    assert torch.equal(K1, K2) and torch.equal(K1, K1.t()) and bool(torch.isfinite(K1).all())
    monkeypatch.setenv("GRF_DENSE_XCD", "0")
    K0 = eng.gram_dense(A, k, precision="split")
    monkeypatch.delenv("GRF_DENSE_XCD")
    rows = torch.arange(0, n, 61, device=eng.device)
    Ad = A[:, :k].double()
    ref = Ad[rows] @ Ad.t()
    bound = 1e-5 * (Ad[rows].abs() @ Ad.abs().t()) + 1e-30
    assert float(((K1[rows].double() - ref).abs() / bound).max()) <= 1.0
    assert float(((K1[rows].double() - K0[rows].double()).abs() / bound).max()) <= 2.0


@pytest.mark.parametrize("n,k", [(2708, 2708), (1000, 1000), (300, 17), (4000, 500)])
def test_gram_dense_planes_tile_kernel(eng, monkeypatch, n, k):
    """The 128-tile kernel on the planes (gram_planes_tile_kernel, below 64 tile rows): below 256 tiles the
    in-register split runs the same work items (gram_split_mfma_kernel), so the bits are identical (C3's size
    among them); from 256 tiles on the in-register path is stream-K (other k pieces): within twice the fp32
    path's bound of it.  Both within the bound of fp64, exactly symmetric, run-to-run identical, tickets zero."""
    import torch
    lda = -(-k // 64) * 64
    g = torch.Generator(device=eng.device).manual_seed(n * 3 + k)
    A = torch.zeros((n, lda), dtype=torch.float32, device=eng.device)
    A[:, :k] = torch.randn((n, k), device=eng.device, generator=g) * (
        torch.rand((n, k), device=eng.device, generator=g) < 0.3)
    monkeypatch.setenv("GRF_DENSE_PLANES", "0")
    K0 = eng.gram_dense(A, k, precision="split").clone()
    monkeypatch.setenv("GRF_DENSE_PLANES", "1")
    K1 = eng.gram_dense(A, k, precision="split").clone()
    K2 = eng.gram_dense(A, k, precision="split")
    ws = eng._dense_ws[eng.stream.value]
    assert int(ws[:4096].view(torch.int32).abs().sum()) == 0
    assert torch.equal(K1, K2) and torch.equal(K1, K1.t()) and bool(torch.isfinite(K1).all())
    tiles = (-(-n // 128)) * (-(-n // 128) + 1) // 2
    Ad = A[:, :k].double()
    rows = torch.arange(0, n, 7, device=eng.device)
    bound = 1e-5 * (Ad[rows].abs() @ Ad.abs().t()) + 1e-30
    assert float(((K1[rows].double() - Ad[rows] @ Ad.t()).abs() / bound).max()) <= 1.0
    if tiles < 256:
        assert torch.equal(K0, K1), float((K0 - K1).abs().max())
    else:
        assert float(((K1[rows].double() - K0[rows].double()).abs() / bound).max()) <= 2.0


def test_gram_dense_c2_size_stream_k(eng):
    """the stream-K path at the bench's C2 size (n = k = 10 000; the split Gram's wide
    workgroups: 1600 items of 256 x 128 over 256 slots, items cut at slot boundaries and summed through
    slabs) against fp64 on sampled rows, exactly symmetric, run-to-run identical bits."""
    import torch
    n = k = 10000
    lda = -(-k // 64) * 64
    g = torch.Generator(device=eng.device).manual_seed(10)
    A = torch.zeros((n, lda), dtype=torch.float32, device=eng.device)
    A[:, :k] = torch.rand((n, k), device=eng.device, generator=g) * (
        torch.rand((n, k), device=eng.device, generator=g) < 0.05)
    K1 = eng.gram_dense(A, k)
    K2 = eng.gram_dense(A, k)
    assert torch.equal(K1, K2) and torch.equal(K1, K1.t())
    rows = torch.arange(0, n, 97, device=eng.device)
    Ad = A[:, :k].double()
    ref = Ad[rows] @ Ad.t()
    bound = 1e-5 * (Ad[rows].abs() @ Ad.abs().t()) + 1e-30
    assert float(((K1[rows].double() - ref).abs() / bound).max()) <= 1.0


def test_gram_dense_workspace_reused_across_sizes(eng):
    """One engine workspace serves split-K calls of different sizes in any order (the ticket block
    sits at a fixed place ahead of the slabs): small -> large -> small gives each size's bits of a
    fresh engine's call."""
    import torch
    from grf_amd.engine import GRFEngine
    r = np.random.default_rng(7)
    ops = []
    for n in (1000, 2708, 300, 4500, 1000):
        k = n + 17
        lda = -(-k // 64) * 64
        Ad = np.zeros((n, lda), np.float32)
        Ad[:, :k] = (r.standard_normal((n, k)) * (r.random((n, k)) < 0.05)).astype(np.float32)
        ops.append((torch.from_numpy(Ad).to(eng.device), k))
    got = [eng.gram_dense(A, k).cpu().numpy() for A, k in ops]
    for (A, k), K in zip(ops, got):
        fresh = GRFEngine(eng.device).gram_dense(A, k).cpu().numpy()
        assert np.array_equal(K, fresh) and np.isfinite(K).all()


@pytest.mark.parametrize("n", [2708, 4500])
def test_gram_dense_first_call_on_dirty_allocator_block(eng, n):
    """Round 4's NaN (profiles/AB_LOG.md, "dense-Gram NaN"): the split-K tickets live in the caller's
    workspace and must be zero on first use; the engine once took it uninitialised from the caching
    allocator, whose block had held other data.  Here the allocator's free block is filled with 0xFF
    (every ticket -1) before a FRESH engine's first call at n = 2708 (the per-tile split: 253 tiles x
    2 pieces) and n = 4500 (stream-K): K must be finite, exactly symmetric and within the fp64 bound,
    the tickets must come back zero, and a second call must repeat the bits."""
    import torch
    from grf_amd import _lib as C
    from grf_amd.engine import GRFEngine
    k = n
    lda = -(-k // 64) * 64
    r = np.random.default_rng(n + 3)
    Ad = np.zeros((n, lda), np.float32)
    Ad[:, :k] = (r.standard_normal((n, k)) * (r.random((n, k)) < 0.05)).astype(np.float32)
    At = torch.from_numpy(Ad).to(eng.device)
    need = int(eng.lib.grf_gram_dense_workspace_bytes(n, k))
    assert need > 4096  # (tickets + slabs: the split path runs)
    torch.cuda.synchronize()
    dirty = torch.full((need + (1 << 20),), 0xFF, dtype=torch.uint8, device=eng.device)
    torch.cuda.synchronize()
    del dirty  # (the block stays in the caching allocator, 0xFF-filled, for the next allocation)
    fresh = GRFEngine(eng.device)
    K = fresh.gram_dense(At, k).cpu().numpy()
    assert np.isfinite(K).all() and np.array_equal(K, K.T)
    ref = Ad.astype(np.float64) @ Ad.astype(np.float64).T
    bound = np.abs(Ad).astype(np.float64) @ np.abs(Ad).astype(np.float64).T
    assert np.all(np.abs(K - ref) <= 1e-5 * bound + 1e-30)
    # the cached workspace came back with every ticket zero: a second call gives the same bits
    ws = next(iter(fresh._dense_ws.values()))
    assert int(ws[:4096].view(torch.int32).abs().sum()) == 0
    assert np.array_equal(fresh.gram_dense(At, k).cpu().numpy(), K)
    # the hub panel's upper-only launch takes no workspace (whole tiles only): same upper triangle
    Ku = torch.zeros((n, eng.leading_dim(n)), dtype=torch.float32, device=eng.device)
    C.check(eng.lib.grf_gram_dense_upper(n, k, At.data_ptr(), lda, Ku.data_ptr(), Ku.stride(0), eng.stream),
            "grf_gram_dense_upper")
    Ku = np.triu(Ku[:, :n].cpu().numpy())
    assert np.all(np.abs(Ku - np.triu(ref)) <= 1e-5 * np.triu(bound) + 1e-30)


def test_full_pipeline_c2_scale(eng):
    """ER N=10k (C2-like) -- Philox walks vs oracle on a source sample, K rows vs oracle, symmetry."""
    n = 10000
    A = er_graph(n, 10, 2024)
    G = eng.laplacian(A)
    slots = eng.walk(G, 128, 0.1, 8, rng=1, seed=42)
    Ls, _ = O.laplacian_sparse(A)
    ip, ix, dx = O._csr_arrays(Ls)
    ref = O.walk_slots(ip, ix, dx, 128, 0.1, 8, rng=O.RNG_PHILOX, seed=42, begin=0, end=n)
    assert slots_equal(slots, ref)
    f = [(-1.0) ** l / (2.0 ** l * float(np.prod(np.arange(1, l + 1)))) for l in range(8)]
    phi = eng.compact(eng.features(slots, f))
    node, load = ref
    ref_phi = O.phi_sparse(O.reduce_steps(node, np.where(node >= 0, load, 0.0), 1), f)
    assert same_csr(phi.to_scipy(), ref_phi)
    K = eng.gram(phi, "sparse")
    rows = np.r_[0:64, 5000:5064, n - 64:n]
    ok, fro = gram_close(K[rows[:64]].cpu().numpy(), ref_phi, (0, 64))
    assert ok, fro
    Kc = K.cpu().numpy()
    sub = Kc[:2000, :2000]
    assert np.max(np.abs(sub - sub.T)) <= 1e-5 * np.max(np.abs(sub))


@pytest.mark.parametrize("n,deg,m,L,p,rule", [(3000, 8, 128, 8, 0.1, 0), (500, 3, 16, 5, 0.3, 1), (800, 12, 64, 3, 0.0, 2),
                                             (300, 4, 7, 6, 0.2, 0), (2000, 10, 256, 16, 0.05, 0)])
def test_walk_phi_fused_bitexact(eng, n, deg, m, L, p, rule):
    """grf_walk_phi == grf_walk (Philox) + grf_phi_fused, bit for bit, on a graph with isolated nodes."""
    A = er_graph(n, deg, n + m)
    A = A.tolil()
    A[5, :] = 0
    A[:, 5] = 0
    A = A.tocsr()
    A.eliminate_zeros()
    G = eng.laplacian(A)
    f = [(-0.7) ** l for l in range(L - 1)]  # shorter than L: truncated like the sparse reference
    for src in [(0, n), (17, 211)]:
        slots = eng.walk(G, m, p, L, rng=1, seed=9, load_rule=rule, src_begin=src[0], src_end=src[1])
        ref = eng.compact(eng.phi_fused(slots, f)).to_scipy()
        got = eng.compact(eng.walk_phi(G, m, p, L, f, seed=9, load_rule=rule, src_begin=src[0], src_end=src[1]))
        assert same_csr(got.to_scipy(), ref), src
        # float32-only output (the bench path): the same columns and float32 values
        g32 = eng.compact(eng.walk_phi(G, m, p, L, f, seed=9, load_rule=rule, src_begin=src[0], src_end=src[1],
                                       want64=False), want64=False)
        import torch
        assert torch.equal(g32.ptr, got.ptr) and torch.equal(g32.idx[:got.nnz], got.idx[:got.nnz])
        assert torch.equal(g32.val32[:got.nnz], got.val32[:got.nnz])
    # bucket counts from the walk kernel == the transpose's own counting (same K, bit for bit)
    bw = 256
    ws = eng.transpose_workspace(n, n, bw)
    phi = eng.compact(eng.walk_phi(G, m, p, L, f, seed=9, load_rule=rule, count_ws=ws, band_width=bw))
    K1 = eng.gram_sparse(phi, eng.transpose_banded(phi, bw, counted_ws=ws)).cpu().numpy()
    K2 = eng.gram_sparse(phi, eng.transpose_banded(phi, bw)).cpu().numpy()
    assert np.array_equal(K1, K2)


# ------------------------------------------------- real graphs
def _diffusion(L):
    return np.array([(-1.0) ** l / (2.0 ** l * float(np.prod(np.arange(1, l + 1)))) for l in range(L)])


def _k_bound_close(Krows, phi64, rows, Kref):
    """|dK| <= 3e-5 (|Phi||Phi|^T) + the fixed-point resolution, on selected rows."""
    absphi = abs(phi64)
    bound = (absphi[rows] @ absphi.T).toarray()
    rowmax = np.asarray(absphi.max(axis=1).todense()).ravel()
    fx = 1e-12 * np.maximum(rowmax[rows][:, None], rowmax[None, :]) * absphi.max()
    err = np.abs(np.asarray(Krows, np.float64) - Kref)
    return bool(np.all(err <= 3e-5 * bound + fx + 1e-30)), float(err.max())


@pytest.mark.parametrize("name", ["facebook", "enron"])
def test_snap_graph_reference_stream(eng, golden, name):
    """Facebook / Enron (self-loops, heavy-tailed degrees): Laplacian, the 8 step matrices and Phi
    bit-identical to the reference's own sparse path; K rows (hubs included) within tolerance."""
    from golden_util import digest, snap_adjacency, snap_k_rows
    d = golden("snap")
    A = snap_adjacency(d, name)
    n = A.shape[0]
    m, p, L = (int(d[f"{name}_walk"][0]), float(d[f"{name}_walk"][1]), int(d[f"{name}_walk"][2]))
    G = eng.laplacian(A)
    assert digest(G.to_scipy()) == str(d[f"{name}_L_digest"][0])
    slots = eng.walk(G, m, p, L, rng=0, seed=42, n_chunks=8)
    mats = eng.step_matrices(eng.steps(slots, norm=1))
    assert [digest(M.to_scipy()) for M in mats] == [str(x) for x in d[f"{name}_step_digests"]]
    phi = eng.compact(eng.features(slots, _diffusion(L)))
    phi64 = phi.to_scipy()
    assert digest(phi64) == str(d[f"{name}_phi_digest"][0])
    rows = d[f"{name}_K_rows"].astype(np.int64)
    K = eng.gram(phi, "sparse")
    import torch
    Kr = K[torch.from_numpy(rows).to(K.device)].cpu().numpy()
    ok, e = _k_bound_close(Kr, phi64, rows, snap_k_rows(d, name, n))
    assert ok, e
    diag = K.diagonal().cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(diag, d[f"{name}_K_diag"], rtol=3e-5)
    del K


@pytest.mark.parametrize("name", ["enron", "powerlaw"])
def test_bench_path_heavy_tailed_graphs(eng, golden, name):
    """The bench's path (fused Philox walk -> Phi with bucket counting, sync-free compaction, staged
    transpose, symmetric Gram + mirror) on heavy-tailed graphs -- the real Enron graph and a C5-style
    Chung-Lu power-law graph: Phi bit-exact against the oracle, K exactly symmetric, the symmetric
    and row modes bit-identical, rows (hubs included) within tolerance."""
    import torch
    from golden_util import snap_adjacency
    from grf_amd.engine import DEFAULT_BAND_WIDTH
    from grf_amd.graphs import powerlaw_graph
    A = snap_adjacency(golden("snap"), name) if name != "powerlaw" else powerlaw_graph(50_000, 10.0, 2.5, seed=3)
    n = A.shape[0]
    m, p, L = 64, 0.1, 8
    f = _diffusion(L)
    G = eng.laplacian(A)
    tws = eng.transpose_workspace(n, n)
    rows_p = eng.walk_phi(G, m, p, L, f, seed=42, count_ws=tws, band_width=DEFAULT_BAND_WIDTH)
    phi = eng.compact(rows_p, want64=True, want32=True, sync_free=True)
    Ls, _ = O.laplacian_sparse(A)
    ip, ix, dx = O._csr_arrays(Ls)
    node, load = O.walk_slots(ip, ix, dx, m, p, L, rng=O.RNG_PHILOX, seed=42)
    ref_phi = O.phi_sparse(O.reduce_steps(node, load, O.NORM_MUL_RECIP), f)
    phi64 = phi.to_scipy()
    assert same_csr(phi64, ref_phi)
    tr = eng.transpose_banded(phi, counted_ws=tws, nnz_bound=phi.nnz_bound)
    K = eng.gram_sparse_sym(phi, tr)
    sample = np.r_[0, 1, np.argsort(-np.diff(A.indptr), kind="stable")[:4], n - 1].astype(np.int64)
    si = torch.from_numpy(sample).to(K.device)
    Ks = K[si].cpu().numpy()
    ok, e = _k_bound_close(Ks, ref_phi, sample, (ref_phi[sample] @ ref_phi.T).toarray())
    assert ok, e
    assert torch.equal(K[:, :2048][:2048], K[:2048, :2048].t())  # exact symmetry (a diagonal block)
    assert torch.equal(K[si, :].t().contiguous(), K[:, si].contiguous())
    # row mode = symmetric mode on and above the diagonal (the mirror carries the upper triangle)
    for r0, r1 in ((0, 4096), (n - 5000, n)):
        Kr = eng.gram_sparse(phi, tr, r0, r1)
        up = torch.triu(torch.ones(r1 - r0, n, dtype=torch.bool, device=K.device), diagonal=r0)
        assert torch.equal(Kr[up], K[r0:r1][up])
    del K, Kr


@pytest.mark.parametrize("name,hubs", [("enron", 64), ("enron", 256), ("powerlaw", 100), ("er", 32)])
def test_hub_column_split(eng, golden, name, hubs):
    """Hub-column split (grf_hub_panel + grf_transpose_drop_columns + grf_gram_dense_upper +
    grf_gram_sparse_upper_add + mirror): the panel holds exactly Phi's chosen columns, their buckets
    are emptied, K is exactly symmetric and within the K tolerance of the fp64 oracle product (and of
    the all-sparse K) on sampled rows, hubs included; hubs = 0 is the all-sparse K bit for bit."""
    import torch
    from golden_util import snap_adjacency
    from grf_amd import pipeline as P
    from grf_amd.graphs import powerlaw_graph
    if name == "enron":
        A = snap_adjacency(golden("snap"), name)
    elif name == "powerlaw":
        A = powerlaw_graph(20_000, 10.0, 2.5, seed=5)
    else:
        A = er_graph(9000, 6, 13)
    n = A.shape[0]
    m, p, L = 32, 0.1, 8
    f = _diffusion(L)
    G = eng.laplacian(A)
    phi = eng.compact(eng.walk_phi(G, m, p, L, f, seed=42), want64=True, want32=True)
    phi64 = phi.to_scipy()
    K0 = eng.gram_sparse_sym(phi, eng.transpose_banded(phi))
    tr = eng.transpose_banded(phi)
    Pn, cols = eng.hub_split(phi, tr, hubs)
    c = cols.cpu().numpy().astype(np.int64)
    assert c.size == hubs and np.all(np.diff(c) > 0)
    cnt = np.bincount(phi64.indices, minlength=n)
    # the chosen columns are the densest by record pairs: no unchosen column has more entries than
    # twice the sparsest chosen one plus a band's rounding (pairs ~ entries / 2 per band)
    nb = -(-n // tr.band_width)
    assert cnt[np.setdiff1d(np.arange(n), c)].max(initial=0) <= 2 * cnt[c].min() + 2 * nb
    panel = Pn[:, :hubs].cpu().numpy()
    want = phi64.astype(np.float32)[:, c].toarray()
    assert np.array_equal(panel, want) and not Pn[:, hubs:].any()
    d = tr.t_desc[:2 * nb * n].view(nb, n, 2)[:, :, 1]
    assert int(d[:, cols.long()].abs().sum()) == 0
    tr = eng.transpose_banded(phi)
    Kh = eng.gram_sparse_sym_hubs(phi, tr, hubs)
    assert torch.equal(Kh, Kh.t())
    sample = np.r_[0, 1, np.argsort(-np.diff(A.indptr), kind="stable")[:4], c[:2], n - 1].astype(np.int64)
    si = torch.from_numpy(sample).to(Kh.device)
    ref = (phi64[sample] @ phi64.T).toarray()
    ok, e = _k_bound_close(Kh[si].cpu().numpy(), phi64, sample, ref)
    assert ok, e
    ok, e = _k_bound_close(Kh[si].cpu().numpy(), phi64, sample, K0[si].cpu().numpy().astype(np.float64))
    assert ok, e
    # the bench's pipeline with the split (pl.hubs): the same K
    pl = P.plan_step(n, m, L, p, f, seed=42)
    pl.hubs = hubs
    Kb = P.k_view(P.k_assembly(eng, P.Front(phi, eng.transpose_banded(phi), phi), pl, P.alloc_k(eng, pl)), pl)
    assert torch.equal(Kb, Kh)
    assert torch.equal(eng.gram_sparse_sym_hubs(phi, eng.transpose_banded(phi), 0), K0)
    del K0, Kh, Kb


def test_sharded_counts_and_phi_equal_single_gpu(eng):
    """The multi-GPU assembly, emulated in one process: per-shard fused walk -> Phi with bucket
    counting, counts summed (the all-reduce of dist.gather_phi) and rows concatenated (the
    all-gather) give the single-GPU transpose bit for bit, and the row-block Grams match K."""
    import torch
    from grf_amd.dist import shard_range
    from grf_amd.engine import DEFAULT_BAND_WIDTH, DeviceCSR
    n = 20000
    A = er_graph(n, 10, 11)
    G = eng.laplacian(A)
    m, L = 32, 6
    f = [1.0, -0.5, 0.125, -0.02, 0.003, -0.0004]
    nbk = -(-n // DEFAULT_BAND_WIDTH) * n
    ws1 = eng.transpose_workspace(n, n)
    one = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=5, count_ws=ws1, band_width=DEFAULT_BAND_WIDTH),
                      want64=False)
    cnt1 = ws1[:4 * nbk].clone()  # (the transpose reuses its workspace)
    tr1 = eng.transpose_banded(one, counted_ws=ws1, nnz_bound=n * m * L)
    K1 = eng.gram_sparse(one, tr1)
    world = 3
    wsum = eng.transpose_workspace(n, n)
    parts = []
    for r in range(world):
        b, e = shard_range(n, r, world)
        ws = eng.transpose_workspace(n, n)
        loc = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=5, src_begin=b, src_end=e, count_ws=ws,
                                       band_width=DEFAULT_BAND_WIDTH), want64=False)
        wsum[:4 * nbk].view(torch.int32).add_(ws[:4 * nbk].view(torch.int32))
        parts.append(loc)
    cnt = torch.cat([p.ptr[1:] - p.ptr[:-1] for p in parts])
    ptr = torch.zeros(n + 1, dtype=torch.int64, device=cnt.device)
    ptr[1:] = torch.cumsum(cnt, 0)
    phi = DeviceCSR(n, n, ptr, torch.cat([p.idx[:p.nnz] for p in parts]), None,
                    torch.cat([p.val32[:p.nnz] for p in parts]), int(ptr[-1].item()))
    assert torch.equal(wsum[:4 * nbk], cnt1)
    assert torch.equal(phi.ptr, one.ptr) and torch.equal(phi.idx, one.idx[:one.nnz])
    tr = eng.transpose_banded(phi, counted_ws=wsum, nnz_bound=n * m * L)
    assert torch.equal(tr.t_desc, tr1.t_desc) and torch.equal(tr.t_rowshift, tr1.t_rowshift)
    for r in range(world):
        b, e = shard_range(n, r, world)
        assert torch.equal(eng.gram_sparse(phi, tr, b, e), K1[b:e])


def _sym_square(Kc, b, e):
    """Kc = K[:, b:e] with its square K[b:e, b:e] made symmetric from its upper triangle."""
    import torch
    out = Kc.clone()
    sq = Kc[b:e]
    out[b:e] = torch.triu(sq) + torch.triu(sq, 1).T
    return out


@pytest.mark.parametrize("world", [2, 3, 8])
def test_column_block_gram_from_local_transpose(eng, world):
    """The column-block multi-GPU Gram: each rank transposes only its own Phi rows and computes
    K[:, b:e] against all (gathered) rows with the row shifts of the whole Phi -- bit-identical to
    the single-GPU row mode's columns, for any band width of the local transpose and row subset."""
    import torch
    from grf_amd.dist import shard_range
    n = 20000
    A = er_graph(n, 10, 12)
    G = eng.laplacian(A)
    m, L = 32, 6
    f = [1.0, -0.5, 0.125, -0.02, 0.003, -0.0004]
    phi = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=8), want64=False)
    tr = eng.transpose_banded(phi, 8192)
    K = eng.gram_sparse(phi, tr)
    shift = eng.phi_row_shifts(phi)
    assert torch.equal(shift[:n], tr.t_rowshift[:n])
    for r in range(world):
        b, e = shard_range(n, r, world)
        loc = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=8, src_begin=b, src_end=e), want64=False)
        assert loc.n_rows == e - b and loc.n_cols == n
        want_sym = _sym_square(K[:, b:e], b, e)
        for bw in (64, 4096, 8192):
            tb = eng.transpose_banded(loc, bw)
            Kc = eng.gram_sparse_cols(phi, shift, tb)
            assert torch.equal(Kc, K[:, b:e]), (r, bw)
            # the symmetric square K[b:e, b:e]: upper tiles + mirror
            assert torch.equal(eng.gram_sparse_cols(phi, shift, tb, sym_row0=b), want_sym), (r, bw)
        Kp = eng.gram_sparse_cols(phi, shift, eng.transpose_banded(loc, 4096), 123, 4567)
        assert torch.equal(Kp, K[123:4567, b:e])
        # a K-row block narrower than the rank's rows (bench --k-rows): the first k of its rows
        from grf_amd.engine import DeviceCSR
        k = min(1000, e - b)
        sub = DeviceCSR(k, n, loc.ptr[:k + 1], loc.idx, None, loc.val32)
        assert torch.equal(eng.gram_sparse_cols(phi, shift, eng.transpose_banded(sub, 1024, nnz_bound=k * 32 * 6)),
                           K[:, b:b + k])


@pytest.mark.parametrize("graph", ["powerlaw", "er"])
def test_slot_transpose_gram_bit_identical(eng, graph):
    """The GRF_REC_SLOT transpose (each bucket's header and first two pairs in a 32-byte slot, the rest
    in the overflow area) gives the Gram the same bits as the packed pairs it replaces: column blocks
    with and without the symmetric square, a row sub-block, the whole symmetric K and the row mode, on
    a hub-heavy power-law graph (buckets of hundreds of entries overflow, oversized regions place
    through global memory) and an Erdos-Renyi one; ragged block sizes."""
    import torch
    from grf_amd import _lib as C
    from grf_amd.graphs import powerlaw_graph
    n = 30000
    A = powerlaw_graph(n, 8.0, 2.2, seed=4) if graph == "powerlaw" else er_graph(n, 6, 21)
    G = eng.laplacian(A)
    m, L = 24, 6
    f = [1.0, -0.5, 0.125, -0.02, 0.003, -0.0004]
    phi = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=5), want64=False)
    shift = eng.phi_row_shifts(phi)
    for b, e in ((0, 8192), (1000, 6077), (n - 5003, n)):
        loc = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=5, src_begin=b, src_end=e), want64=False)
        bw = 8192 if e - b > 4096 else 4160
        tp = eng.transpose_banded(loc, bw, rec_unit=C.REC_PACKED)
        ts = eng.transpose_banded(loc, bw, rec_unit=C.REC_SLOT)  # (any bucket size: most overflow here)
        assert torch.equal(ts.t_rowshift[:e - b], tp.t_rowshift[:e - b])
        assert torch.equal(eng.gram_sparse_cols(phi, shift, ts), eng.gram_sparse_cols(phi, shift, tp)), (b, e)
        assert torch.equal(eng.gram_sparse_cols(phi, shift, ts, sym_row0=b),
                           eng.gram_sparse_cols(phi, shift, tp, sym_row0=b)), (b, e)
        assert torch.equal(eng.gram_sparse_cols(phi, shift, ts, 77, 2345),
                           eng.gram_sparse_cols(phi, shift, tp, 77, 2345)), (b, e)
    # the whole K: slot transposes of all rows through the symmetric and the row-mode Gram
    tp = eng.transpose_banded(phi, 8192, rec_unit=C.REC_PACKED)
    ts = eng.transpose_banded(phi, 8192, rec_unit=C.REC_SLOT)
    assert torch.equal(eng.gram_sparse_sym(phi, ts), eng.gram_sparse_sym(phi, tp))
    assert torch.equal(eng.gram_sparse(phi, ts, 0, 3000), eng.gram_sparse(phi, tp, 0, 3000))
    # (the packed path's K is pinned to the oracle by test_gram_sparse_vs_oracle / the C5 headline test)
    # slots=True takes the slot layout where packed pairs would be chosen (sparse buckets, bands > 4096)
    phs = eng.compact(eng.walk_phi(G, 4, 0.3, 3, f[:3], seed=5), want64=False)
    t_auto = eng.transpose_banded(phs, 8192, slots=True)
    assert t_auto.rec_unit == C.REC_SLOT
    assert torch.equal(eng.gram_sparse(phs, t_auto, 0, 2000),
                       eng.gram_sparse(phs, eng.transpose_banded(phs, 8192, rec_unit=C.REC_PACKED), 0, 2000))


@pytest.mark.parametrize("pipe", ["1"])
def test_gram_cols_pipelined_bit_identical(eng, pipe):
    """The persistent, software-pipelined column-block Gram kernel for slot buckets (gram_slot_pipe_kernel, the
    default) gives the tile-per-workgroup kernel's bits (GRF_GRAM_PIPE=0): m = 256 walks of up to 6 visits on a
    degree-40 graph (rows of over 768 nonzeros, past 64 per gather wave: the batch-by-batch tail of a share),
    one band (8192 columns), three bands with a ragged last one, a band width that is not a power of two, a
    row range, and t_rows not a multiple of 4."""
    import os

    import torch
    from grf_amd import _lib as C
    n = 30001
    A = er_graph(n, 40, 7)
    G = eng.laplacian(A)
    m, L = 256, 6
    f = [1.0, -0.5, 0.125, -0.02, 0.003, -0.0004]
    phi = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=3, want64=False), want64=False)
    shift = eng.phi_row_shifts(phi)
    assert int((phi.ptr[1:] - phi.ptr[:-1]).max()) > 64 * 12  # (shares past one batch of 64 per wave)
    old = os.environ.get("GRF_GRAM_PIPE")
    try:
        for b, e, bw, rows in ((0, 8192, 8192, None), (5000, 25000, 8192, None), (101, 6101, 6016, None),
                               (2000, 10190, 8192, (333, 29001)), (7, 8194, 8192, None)):
            loc = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=3, src_begin=b, src_end=e, want64=False), want64=False)
            ts = eng.transpose_banded(loc, bw, rec_unit=C.REC_SLOT)
            r0, r1 = rows or (0, n)
            os.environ["GRF_GRAM_PIPE"] = "0"
            K0 = eng.gram_sparse_cols(phi, shift, ts, r0, r1).clone()
            os.environ["GRF_GRAM_PIPE"] = pipe
            K1 = eng.gram_sparse_cols(phi, shift, ts, r0, r1)
            assert torch.equal(K0, K1), (pipe, b, e, bw, rows)
    finally:
        if old is None:
            os.environ.pop("GRF_GRAM_PIPE", None)
        else:
            os.environ["GRF_GRAM_PIPE"] = old


def test_gram_cols_padded_rows_bit_identical(eng):
    """Phi as the walk's padded rows (grf_phi_row_shifts_padded + grf_gram_sparse_cols_padded: one GPU's C5
    block with no compaction of Phi) gives the compacted path's bits: the row shifts,
    and K[r0:r1, B] for the same blocks as test_gram_cols_pipelined_bit_identical (rows past 64 per gather wave, a
    ragged last band, a band width that is not a power of two, a row range); the padded rows themselves, compacted,
    are the plain walk's Phi.  Then the pipeline's one-GPU column-block step both ways (GRF_PADDED_PHI)."""
    import torch
    from grf_amd import _lib as C
    from grf_amd import pipeline as P
    from grf_amd.engine import DeviceCSR
    n = 30001
    A = er_graph(n, 40, 7)
    G = eng.laplacian(A)
    m, L = 256, 6
    f = [1.0, -0.5, 0.125, -0.02, 0.003, -0.0004]
    rows = eng.walk_phi(G, m, 0.1, L, f, seed=3, want64=False)
    phi = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=3, want64=False), want64=False)
    shift = eng.phi_row_shifts(phi)
    shift_p = eng.phi_row_shifts(rows)
    assert torch.equal(shift, shift_p)
    cp = eng.compact(rows, want64=False)
    assert torch.equal(cp.ptr, phi.ptr) and torch.equal(cp.idx[:phi.nnz], phi.idx[:phi.nnz])
    assert torch.equal(cp.val32[:phi.nnz], phi.val32[:phi.nnz])
    for b, e, bw, rr in ((0, 8192, 8192, None), (5000, 25000, 8192, None), (101, 6101, 6016, None),
                         (2000, 10190, 8192, (333, 29001)), (7, 8194, 8192, None)):
        loc = eng.compact(eng.walk_phi(G, m, 0.1, L, f, seed=3, src_begin=b, src_end=e, want64=False), want64=False)
        ts = eng.transpose_banded(loc, bw, rec_unit=C.REC_SLOT)
        r0, r1 = rr or (0, n)
        K0 = eng.gram_sparse_cols(phi, shift, ts, r0, r1).clone()
        K1 = eng.gram_sparse_cols(rows, shift_p, ts, r0, r1)
        assert torch.equal(K0, K1), (b, e, bw, rr)
    # the pipeline's step (plan_step cols mode, one GPU: C5's shape at 600k nodes, slot buckets) with and
    # without the padded front
    from grf_amd.graphs import powerlaw_graph
    A2 = powerlaw_graph(600_000, 10.0, 2.5, seed=1)
    pl = P.plan_step(600_000, 64, 8, 0.1, np.array([1.0, -0.5, 0.125, -0.02, 0.003, -0.0004, 1e-5, -1e-6]),
                     k_rows=8192)
    assert pl.mode == "cols"
    Ad = DeviceCSR.from_scipy(A2, eng.device)
    old = P.PADDED_PHI
    try:
        P.PADDED_PHI = False
        Ka, fra = P.kernel_step(eng, Ad, pl)
        Ka = Ka.clone()
        P.PADDED_PHI = True
        Kb, frb = P.kernel_step(eng, Ad, pl)
        assert isinstance(frb.phi, P.PaddedPhi) and not isinstance(fra.phi, P.PaddedPhi)
        assert torch.equal(P.k_view(Ka, pl), P.k_view(Kb, pl))
        assert torch.equal(fra.row_shift, frb.row_shift)
        assert torch.equal(fra.phi.ptr, frb.phi.ptr)
        assert P.k_block_check(eng, frb, pl, Kb)["max_ratio"] <= 1.0
    finally:
        P.PADDED_PHI = old


@pytest.mark.parametrize("unit", [128, 12])
def test_transpose_wide_regions(eng, unit):
    """A graph large enough that the staged fill widens its column regions (n_rows * n_cols / (16 cr)
    above 32 M: cr = 256 at 300k nodes) gives the atomic fill's descriptors and the same K rows."""
    n = 300_000
    A = er_graph(n, 4, 21)
    G = eng.laplacian(A)
    phi = eng.compact(eng.walk_phi(G, 4, 0.2, 3, [1.0, -0.5, 0.25], seed=8))
    ta = eng.transpose_banded(phi, 8192, staged=False, rec_unit=unit)
    ts = eng.transpose_banded(phi, 8192, staged=True, rec_unit=unit, self_count=False)
    tself = eng.transpose_banded(phi, 8192, rec_unit=unit, self_count=True)
    assert np.array_equal(ta.t_desc.cpu().numpy(), ts.t_desc.cpu().numpy())
    assert np.array_equal(ta.t_rowshift.cpu().numpy(), ts.t_rowshift.cpu().numpy())
    assert np.array_equal(ta.t_rowshift.cpu().numpy(), tself.t_rowshift.cpu().numpy())
    for r0 in (0, n - 200):
        Ka = eng.gram_sparse(phi, ta, r0, r0 + 200).cpu().numpy()
        assert np.array_equal(Ka, eng.gram_sparse(phi, ts, r0, r0 + 200).cpu().numpy())
        assert np.array_equal(Ka, eng.gram_sparse(phi, tself, r0, r0 + 200).cpu().numpy())
    ok, fro = gram_close(eng.gram_sparse(phi, ts, 0, 50).cpu().numpy(), phi.to_scipy(), (0, 50))
    assert ok, fro


@pytest.mark.parametrize("rule", [0, 1, 2])
def test_walk_phi_augmented_matrix_bitexact(eng, rule):
    """One-round-trip walks over the augmented walk matrix (grf_walk_aug) take the same draws and
    give the same Phi bits as the two-round-trip walks, on a weighted heavy-tailed graph with
    isolated nodes; and both match the oracle."""
    import torch
    from grf_amd.graphs import powerlaw_graph
    A = powerlaw_graph(6000, 6.0, 2.2, seed=5)
    A.data = np.random.default_rng(1).uniform(0.2, 3.0, A.nnz)
    A = ((A + A.T) * 0.5).tocsr()
    A.sort_indices()
    G = eng.laplacian(A)
    f = [1.0, -0.5, 0.125, -0.02, 0.003]
    a = eng.walk_phi(G, 40, 0.15, 5, f, seed=11, load_rule=rule, use_aug=True)
    b = eng.walk_phi(G, 40, 0.15, 5, f, seed=11, load_rule=rule, use_aug=False)
    assert torch.equal(a.cnt, b.cnt)
    mask = torch.arange(a.cap, device=a.cnt.device)[None, :] < a.cnt[:, None]
    assert torch.equal(a.idx.view(-1, a.cap)[mask], b.idx.view(-1, b.cap)[mask])
    assert torch.equal(a.val.view(-1, a.cap)[mask], b.val.view(-1, b.cap)[mask])
    # the 16-byte records (the default here: the ids, starts and lengths fit 64 bits) and the 32-byte
    # ones (GRF_WALK_AUG16=0) take the same walks
    hdr = eng.walk_aug(G)[:16].view(torch.int32).cpu().numpy()
    assert hdr[0] == 1, hdr
    import os
    os.environ["GRF_WALK_AUG16"] = "0"
    try:
        G32 = eng.laplacian(A)
        assert eng.walk_aug(G32)[:16].view(torch.int32).cpu().numpy()[0] == 0
        c = eng.walk_phi(G32, 40, 0.15, 5, f, seed=11, load_rule=rule, use_aug=True)
    finally:
        del os.environ["GRF_WALK_AUG16"]
    assert torch.equal(c.cnt, a.cnt)
    assert torch.equal(c.idx.view(-1, c.cap)[mask], a.idx.view(-1, a.cap)[mask])
    assert torch.equal(c.val.view(-1, c.cap)[mask], a.val.view(-1, a.cap)[mask])
    Ls, _ = O.laplacian_sparse(A)
    ip, ix, dx = O._csr_arrays(Ls)
    node, load = O.walk_slots(ip, ix, dx, 40, 0.15, 5, rng=O.RNG_PHILOX, load_rule=rule, seed=11)
    ref = O.phi_sparse(O.reduce_steps(node, load, O.NORM_MUL_RECIP), f)
    assert same_csr(eng.compact(a).to_scipy(), ref)


@pytest.mark.parametrize("rule", [0, 1, 2])
def test_walk_slots_augmented_matrix_bitexact(eng, rule):
    """The slot walks (grf_walk_ex: the PCG64 reference-stream replay and Philox) over the augmented
    walk matrix take the same draws and give the same visit slots as grf_walk's two round trips per
    step, in both record formats, on a weighted heavy-tailed graph with isolated nodes; and the PCG64
    replay still matches the oracle's reference stream."""
    import os
    import torch
    from grf_amd.graphs import powerlaw_graph
    A = powerlaw_graph(3000, 5.0, 2.2, seed=7)
    A.data = np.random.default_rng(3).uniform(0.2, 3.0, A.nnz)
    A = ((A + A.T) * 0.5).tocsr()
    A.sort_indices()
    G = eng.laplacian(A)
    os.environ["GRF_WALK_AUG16"] = "0"
    try:
        G32 = eng.laplacian(A)
        assert eng.walk_aug(G32)[:16].view(torch.int32).cpu().numpy()[0] == 0  # (32-byte records)
    finally:
        del os.environ["GRF_WALK_AUG16"]
    assert eng.walk_aug(G)[:16].view(torch.int32).cpu().numpy()[0] == 1      # (16-byte records)
    for rng, chunks in ((0, 1), (0, 5), (0, 64), (1, 1)):
        kw = dict(rng=rng, seed=13, n_chunks=chunks, load_rule=rule)
        a = eng.walk(G, 12, 0.2, 6, use_aug=False, **kw)
        for g in (G, G32):
            b = eng.walk(g, 12, 0.2, 6, use_aug=True, **kw)
            assert torch.equal(a.node, b.node), (rng, chunks)
            mask = a.node >= 0
            assert torch.equal(a.load[mask], b.load[mask]), (rng, chunks)
    Ls, _ = O.laplacian_sparse(A)
    ip, ix, dx = O._csr_arrays(Ls)
    got = eng.walk(G, 12, 0.2, 6, rng=0, seed=13, n_chunks=5, load_rule=rule)
    ref = O.walk_slots(ip, ix, dx, 12, 0.2, 6, rng=O.RNG_PCG64, n_chunks=5, seed=13, load_rule=rule)
    assert slots_equal(got, ref)


def _sharded_worker(rank, world, port, mode, q, graph="er", policy="nodes"):
    """One rank of a gloo group on cuda:0 (device tensors staged through host memory)."""
    import os

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from grf_amd.dist import balanced_shards, sharded_kernel_matrix
        from grf_amd.engine import GRFEngine
        from grf_amd.graphs import powerlaw_graph
        eng = GRFEngine("cuda:0")
        if graph == "er":
            n = 6000
            A = er_graph(n, 8, 21)
        else:
            n = 20000
            A = powerlaw_graph(n, 10.0, 2.5, seed=4)
        f = [1.0, -0.5, 0.125, -0.02, 0.003]
        m, p, L = 24, 0.15, 5
        shards = balanced_shards(eng, A, m, p, L, f, world, seed=3, policy=policy)
        Kb, (b, e) = sharded_kernel_matrix(eng, A, f, m, p, L, seed=3, mode=mode, shards=shards)
        phi = eng.compact(eng.walk_phi(eng.laplacian(A), m, p, L, f, seed=3), want64=False)
        K = eng.gram_sparse(phi, eng.transpose_banded(phi, 8192))
        if mode == "allreduce":
            # partial fp32 K's summed by the collective: within the K tolerance of the exact sums
            phi64 = phi.to_scipy()
            rows = torch.tensor([0, 1, n // 2, n - 1], device=K.device)
            ok, _ = _k_bound_close(Kb[rows].cpu().numpy(), phi64, rows.cpu().numpy(),
                                   (phi64[rows.cpu().numpy()] @ phi64.T).toarray())
            q.put((rank, bool(ok and torch.allclose(Kb[:, :n], K, rtol=1e-5, atol=1e-6 * float(K.abs().max())))))
            return
        if mode == "cols":
            sq = 4 * (e - b) >= n  # the square K[b:e, b:e] is mirrored when the block is a large share
            want = _sym_square(K[:, b:e], b, e) if sq else K[:, b:e]
        else:
            want = K[b:e]
        q.put((rank, bool(torch.equal(Kb, want)) and (b, e) == tuple(shards[rank])))
    except Exception as exc:  # (reported through the queue: a hung peer would hide it)
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


def _run_sharded(world, mode, graph="er", policy="nodes"):
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, mode, q, graph, policy)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    return res


@pytest.mark.parametrize("mode", ["cols", "rows"])
def test_sharded_kernel_matrix_two_ranks_gloo(mode):
    """The multi-GPU assembly end to end with two ranks on one GPU: each rank's block (row block,
    or the column block from its own-rows transpose) equals the single-GPU K's, bit for bit."""
    assert _run_sharded(2, mode) == [(0, True), (1, True)]


@pytest.mark.parametrize("world,mode,policy", [(2, "cols", "phi"), (3, "cols", "phi"), (3, "rows", "phi"),
                                               (2, "rows", "nodes"), (5, "cols", "nodes"), (8, "cols", "nodes"),
                                               (8, "cols", "phi")])
def test_sharded_powerlaw_balanced_gloo(world, mode, policy):
    """A 20k-node Chung-Lu power-law graph (hubs) on 2 / 3 gloo ranks with cost-balanced shards
    (dist.balanced_shards: the per-row estimate from one setup walk) and with equal node counts:
    every rank's block is bit-identical to the single-GPU K's (the fixed-point Gram does not depend
    on the split), through the sync-free bounded Phi all-gather."""
    assert _run_sharded(world, mode, "powerlaw", policy) == [(r, True) for r in range(world)]


def test_sharded_allreduce_mode_within_tolerance_gloo():
    """The north star's literal option: per-rank partial K over inner slices, summed by the
    all-reduce -- within the K tolerance of the single-GPU K (not bit-identical: fp32 partials are
    added in the collective's order; dist.py)."""
    assert _run_sharded(2, "allreduce") == [(0, True), (1, True)]


def _bench_front_worker(rank, world, port, mode, q):
    """One gloo rank of the bench's own N > 1 step (grf_amd.pipeline, cuda:0): the setup walk's exact
    per-rank entries bound the sync-free Phi all-gather (bench.py --gather-bound exact)."""
    import os

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        from grf_amd import pipeline as P
        from grf_amd.dist import check_gather_overflow, setup_phi, shard_entries
        from grf_amd.engine import DeviceCSR, GRFEngine
        from grf_amd.graphs import powerlaw_graph
        eng = GRFEngine("cuda:0")
        n = 12000
        A = DeviceCSR.from_scipy(powerlaw_graph(n, 10.0, 2.5, seed=6), eng.device)
        f = [1.0, -0.5, 0.125, -0.02, 0.003]
        m, p, L = 32, 0.15, 5
        phi0 = setup_phi(eng, A, m, p, L, f, seed=42)
        pl = P.plan_step(n, m, L, p, f, seed=42, world=world, rank=rank, mode=mode)
        pl.gather_bound = max(shard_entries(phi0, pl.shards))
        Kb, fr = P.kernel_step(eng, A, pl)
        Kb = P.k_view(Kb, pl)
        check_gather_overflow(eng.device)
        K = eng.gram_sparse(phi0, eng.transpose_banded(phi0, 8192))
        b, e = pl.src
        if mode == "cols":
            want = _sym_square(K[:, b:e], b, e) if pl.cols_sym else K[:, b:e]
        else:
            want = K[b:e]
        ok = bool(torch.equal(Kb, want)) and fr.phi.ptr.numel() == n + 1 and \
            int(fr.phi.ptr[-1]) == int(phi0.ptr[-1]) and fr.phi.idx.numel() == world * pl.gather_bound
        q.put((rank, ok))
    except Exception as exc:
        q.put((rank, repr(exc)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "cols"), (3, "cols"), (2, "rows"), (5, "cols"), (8, "cols")])
def test_bench_step_exact_gather_bound_gloo(world, mode):
    """The bench's N > 1 step with the Phi all-gather sized by the setup walk's exact per-rank entries
    (not rows x the padded row capacity): every rank's K block bit-identical to the single-GPU K's.
    World 5 and 8 (the driver's N = 8 node run): column blocks without the mirrored own square
    (4 |R_r| < n), several local bands per rank, the bounded gather over 8 ranks."""
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_front_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
    assert res == [(r, True) for r in range(world)]


@pytest.mark.parametrize("name", ["single", "empty", "star", "components", "path", "pair", "er_sparse"])
def test_bench_path_on_degenerate_graphs(eng, name):
    """The bench's device path (fused Philox walks -> Phi -> banded transpose -> symmetric Gram +
    mirror, row mode, and the column blocks with their symmetric square) on degenerate graphs:
    Phi bit-exact against walk + features, every K mode against the fp64 oracle Gram."""
    import torch
    from test_gpu_api import _degenerate_graphs
    A = sp.csr_matrix(_degenerate_graphs()[name])
    n = A.shape[0]
    G = eng.laplacian(A)
    f = [1.0, -0.5, 0.25, -0.125]
    phi = eng.compact(eng.walk_phi(G, 16, 0.2, 4, f, seed=4), want64=False)
    ref = eng.compact(eng.features(eng.walk(G, 16, 0.2, 4, rng=1, seed=4), f))
    assert same_csr(eng.compact(eng.walk_phi(G, 16, 0.2, 4, f, seed=4)).to_scipy(), ref.to_scipy())
    tr = eng.transpose_banded(phi, 4096)
    K = eng.gram_sparse(phi, tr)
    ok, fro = gram_close(K.cpu().numpy(), ref.to_scipy())
    assert ok, fro
    Ks = eng.gram_sparse_sym(phi, tr)
    assert torch.equal(Ks, Ks.T) and torch.equal(torch.triu(Ks), torch.triu(K))
    b, e = n // 3, n - n // 4
    if e > b:
        loc = eng.compact(eng.walk_phi(G, 16, 0.2, 4, f, seed=4, src_begin=b, src_end=e), want64=False)
        Kc = eng.gram_sparse_cols(phi, eng.phi_row_shifts(phi), eng.transpose_banded(loc, 64), sym_row0=b)
        assert torch.equal(Kc, _sym_square(K[:, b:e], b, e))


@pytest.mark.parametrize("mode,world", [("cols", 2), ("allreduce", 2), ("cols", 5), ("cols", 8)])
def test_bench_line_n2_reports_parity_and_collectives_gloo(mode, world):
    """bench.py's N > 1 line is self-validating and collective-evident (what the driver's 8-GPU run
    will print): two gloo ranks on one GPU (GRF_DIST_BACKEND=gloo, the host-staged rehearsal of the
    RCCL path) run the bench's own step; the line carries the communicator's backend and world size,
    every rank's Gram ms, all-gather ms and bytes, and the in-run K block check
    (pipeline.k_block_check: K_blk u and K_blk^T v against the gathered Phi) passing on every rank."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GRF_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--n-nodes", "20000",
           "--edges", "200000", "--mode", mode]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == world
    d = line["distributed"]
    assert d["backend"] == "gloo" and d["world_size"] == world
    assert len(d["gram_ms_per_rank"]) == world and all(x > 0 for x in d["gram_ms_per_rank"])
    assert all(x > 0 for x in d["gather_bytes_sent_per_rank"]) and all(x > 0 for x in d["gather_ms_per_rank"])
    assert sum(d["rank_rows"]) == 20000
    assert line["parity"]["ok"] and line["parity"]["max_ratio"] <= 1.0 and len(line["parity"]["per_rank"]) == world


_C4_REF_PRINTS = {}  # (b, e, cols_sym) -> fingerprint of the one-GPU K's columns [b, e)


def _c4_reference_prints(eng, worlds=(2, 4, 8)):
    """Fingerprints (tools/gram_hash.py) of the one-GPU K's column blocks K[:, R_r] for every rank of the
    given world sizes at the headline size (C4: ER N = 100k, 1M edges, m = 128, L = 8, p = 0.1, Philox
    seed 42).  The one-GPU K is the row-mode Gram of the setup walk's Phi (every entry from its own row,
    as a rank's column block computes it; the block's own square symmetrised from its upper triangle
    when the bench does, 4 |R_r| >= n).  Computed once per session (40 GB of K), then freed."""
    import torch
    from grf_amd.dist import setup_phi, shard_range
    from grf_amd.engine import DeviceCSR
    from grf_amd.graphs import er_graph_exact_edges
    from tools.gram_hash import fingerprint
    import bench
    if _C4_REF_PRINTS:
        return _C4_REF_PRINTS
    n, m, L, p = 100_000, 128, 8, 0.1
    A = DeviceCSR.from_scipy(er_graph_exact_edges(n, 1_000_000, seed=0), eng.device)
    phi = setup_phi(eng, A, m, p, L, bench.diffusion_modulator(L, 1.0), seed=42)
    K = eng.gram_sparse(phi, eng.transpose_banded(phi, 8192))
    del phi, A
    for w in worlds:
        for r in range(w):
            b, e = shard_range(n, r, w)
            sym = 4 * (e - b) >= n
            if (b, e, sym) in _C4_REF_PRINTS:
                continue
            blk = K[:, b:e].clone()
            if sym:
                sq = blk[b:e].clone()
                blk[b:e] = torch.triu(sq) + torch.triu(sq, 1).T
                del sq
            _C4_REF_PRINTS[(b, e, sym)] = fingerprint(blk)
            del blk
    del K
    torch.cuda.empty_cache()
    return _C4_REF_PRINTS


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_cols_at_headline_size_gloo(eng, world):
    """the N > 1 column-block step at the HEADLINE size (C4: N = 100k, 1M edges,
    m = 128), `world` gloo ranks sharing the one GPU: bench.py --gpus W under torch.distributed.run
    (the real 43.5 M-entry Phi all-gather with its exact bound, 100k / W-column blocks and their band
    widths; world 8 without the mirrored own square).  Every rank's K[:, R_r] must be bit-identical to
    the same columns of the one-GPU K (fingerprints, tools/gram_hash.py), the in-run K check passes,
    and the line reports every rank's Gram time re-run alone (--rank-turns).  GRF_TEST_OUT=<dir> keeps
    the line (profiles/r05_bench_gloo_n<W>.json)."""
    import json
    import os
    import shutil
    import socket
    import subprocess
    import sys
    import tempfile
    from grf_amd.dist import shard_range
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    fp_dir = tempfile.mkdtemp(prefix="grf_fp_")
    try:
        env = dict(os.environ, GRF_DIST_BACKEND="gloo")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
               "--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--rank-turns",
               "--fingerprint-dir", fp_dir]
        r = _run_beating(cmd, root, env, 800, f"c4_gloo_n{world}")
        assert r.returncode == 0, r.stderr[-3000:]
        line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        out_dir = os.environ.get("GRF_TEST_OUT")
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            with open(os.path.join(out_dir, f"r06_bench_gloo_n{world}.json"), "w") as fh:
                fh.write(json.dumps(line) + "\n")
        d = line["distributed"]
        assert line["n_gpus"] == world and d["backend"] == "gloo" and d["world_size"] == world
        assert line["config"]["n_nodes"] == 100_000 and line["config"]["walks_per_node"] == 128
        assert line["parity"]["ok"] and len(line["parity"]["per_rank"]) == world
        assert all(x > 0 for x in d["gram_ms_alone_per_rank"]) and all(x > 0 for x in d["gather_bytes_sent_per_rank"])
        prints = [json.load(open(os.path.join(fp_dir, f"rank{q}.json"))) for q in range(world)]
    finally:
        shutil.rmtree(fp_dir, ignore_errors=True)
    ref = _c4_reference_prints(eng)
    for q, fp in enumerate(prints):
        b, e = shard_range(100_000, q, world)
        assert fp["mode"] == "cols" and fp["shard"] == [b, e] and fp["cols_sym"] == (4 * (e - b) >= 100_000)
        h, sm = ref[(b, e, fp["cols_sym"])]
        assert fp["hash"] == h, f"rank {q} of {world}: K block bits differ from the one-GPU K"
        assert abs(fp["sum"] - sm) <= 1e-12 * abs(sm), (q, fp["sum"], sm)


def _run_beating(cmd, cwd, env, timeout, tag):
    """subprocess.run(capture_output=True, text=True) that appends a line to $GRF_TEST_OUT/<tag>.beat every
    30 s while the child runs (a long silent multi-rank run stays visibly alive to a hang watchdog)."""
    import os
    import subprocess
    import tempfile
    import time
    out_dir = os.environ.get("GRF_TEST_OUT")
    with tempfile.TemporaryFile("w+") as fo, tempfile.TemporaryFile("w+") as fe:
        p = subprocess.Popen(cmd, cwd=cwd, env=env, stdout=fo, stderr=fe, text=True)
        t0 = time.time()
        while True:
            try:
                p.wait(timeout=30)
                break
            except subprocess.TimeoutExpired:
                if time.time() - t0 > timeout:
                    p.kill()
                    p.wait()
                    raise
                if out_dir:
                    os.makedirs(out_dir, exist_ok=True)
                    with open(os.path.join(out_dir, f"{tag}.beat"), "a") as fh:
                        fh.write(f"{time.time() - t0:.0f} s\n")
        fo.seek(0)
        fe.seek(0)
        return subprocess.CompletedProcess(cmd, p.returncode, fo.read(), fe.read())


_C5_REF_PRINTS = {}  # (b, kr_end) -> fingerprint of the one-GPU K's columns [b, kr_end) at C5


def _c5_reference_prints(eng, blocks):
    """Fingerprints of the one-GPU C5 column blocks K[:, b:kr_end] (N = 1M Chung-Lu power-law, seed 0,
    m = 64, L = 8, p = 0.1, Philox seed 42).  Phi of all 1M nodes from ONE un-sharded walk (setup_phi, no
    collective); each block from the transpose of its rows walked on their own (walk_phi src_begin /
    src_end) in a different layout from the bench's -- 4096-row bands of packed pairs, not one
    8192-row band of 32-B slots -- so only the exact fixed-point sums are shared (the Gram's bits do not
    depend on the band width or the record layout).  Every row's shift from a pass over Phi's values."""
    import torch
    from grf_amd.dist import setup_phi
    from grf_amd.engine import DeviceCSR
    from grf_amd.graphs import powerlaw_graph
    from tools.gram_hash import fingerprint
    import bench
    todo = [blk for blk in blocks if blk not in _C5_REF_PRINTS]
    if not todo:
        return _C5_REF_PRINTS
    n, m, L, p = 1_000_000, 64, 8, 0.1
    f = bench.diffusion_modulator(L, 1.0)
    A = DeviceCSR.from_scipy(powerlaw_graph(n, 10.0, 2.5, seed=0), eng.device)
    G = eng.laplacian(A)
    phi = setup_phi(eng, A, m, p, L, f, seed=42)
    shifts = eng.phi_row_shifts(phi)
    for b, ke in todo:
        loc = eng.compact(eng.walk_phi(G, m, p, L, f, seed=42, src_begin=b, src_end=ke, want64=False),
                          want64=False)
        tr = eng.transpose_banded(loc, 4096)
        Kb = eng.gram_sparse_cols(phi, shifts, tr)
        _C5_REF_PRINTS[(b, ke)] = fingerprint(Kb)
        del Kb, tr, loc
        torch.cuda.empty_cache()
    del phi, shifts, G, A
    torch.cuda.empty_cache()
    return _C5_REF_PRINTS


@pytest.mark.timeout(1100)
@pytest.mark.parametrize("world,k_rows", [(2, 8192), (4, 8192), (8, 4096)])
def test_bench_c5_cols_at_size_gloo(eng, world, k_rows):
    """BASELINE config 5's multi-rank step at its full size -- bench.py --workload c5
    --gpus W under torch.distributed.run (gloo, W ranks sharing the one GPU): N = 1M power-law, m = 64,
    every rank walks 1M / W sources, the 176 M-entry Phi all-gather with its exact bound, the per-rank
    slot transpose of rows [b, b + k_rows) and the column block K[:, b:b + k_rows] over all 1M rows.
    World 8 takes 4096-column blocks: 8 x 32.8 GB of 8192-column blocks would not fit in the one GPU's
    288 GB beside eight ranks' Phi (8 x 16.4 GB does).  Every rank's block must be bit-identical to the
    same columns computed by one GPU from an un-sharded walk (_c5_reference_prints), its in-run K
    check passes, and the line reports every rank's Gram time re-run alone (--rank-turns) and its
    all-gather bytes.  GRF_TEST_OUT=<dir> keeps the line (profiles/r06_bench_c5_gloo_n<W>.json)."""
    import json
    import os
    import shutil
    import socket
    import subprocess
    import sys
    import tempfile
    from grf_amd.dist import shard_range
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = 1_000_000
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    fp_dir = tempfile.mkdtemp(prefix="grf_fp5_")
    try:
        env = dict(os.environ, GRF_DIST_BACKEND="gloo")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
               "--workload", "c5", "--k-rows", str(k_rows), "--gpus", str(world), "--steps", "2", "--warmup", "1",
               "--no-cpu-baseline", "--rank-turns", "--fingerprint-dir", fp_dir]
        r = _run_beating(cmd, root, env, 1000, f"c5_gloo_n{world}")
        if r.returncode != 0 and os.environ.get("GRF_TEST_OUT"):
            with open(os.path.join(os.environ["GRF_TEST_OUT"], f"c5_gloo_n{world}.failed.log"), "w") as fh:
                fh.write(r.stdout + "\n----- stderr -----\n" + r.stderr)
        assert r.returncode == 0, r.stderr[-3000:]
        line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        out_dir = os.environ.get("GRF_TEST_OUT")
        if out_dir:
            os.makedirs(out_dir, exist_ok=True)
            with open(os.path.join(out_dir, f"r06_bench_c5_gloo_n{world}.json"), "w") as fh:
                fh.write(json.dumps(line) + "\n")
        d = line["distributed"]
        assert line["n_gpus"] == world and d["backend"] == "gloo" and d["world_size"] == world
        assert line["config"]["n_nodes"] == n and line["config"]["walks_per_node"] == 64
        assert line["unit"] == "K-rows/s" and line["config"]["k_rows_per_gpu"] == k_rows
        assert line["parity"]["ok"] and len(line["parity"]["per_rank"]) == world
        assert all(x > 0 for x in d["gram_ms_alone_per_rank"]) and all(x > 0 for x in d["gather_bytes_sent_per_rank"])
        prints = [json.load(open(os.path.join(fp_dir, f"rank{q}.json"))) for q in range(world)]
    finally:
        shutil.rmtree(fp_dir, ignore_errors=True)
    blocks = [(shard_range(n, q, world)[0], shard_range(n, q, world)[0] + k_rows) for q in range(world)]
    ref = _c5_reference_prints(eng, blocks)
    for q, fp in enumerate(prints):
        b, e = shard_range(n, q, world)
        assert fp["mode"] == "cols" and fp["shard"] == [b, e] and not fp["cols_sym"] and fp["k_rows"] == k_rows
        h, sm = ref[blocks[q]]
        assert fp["hash"] == h, f"rank {q} of {world}: C5 K block bits differ from the one-GPU block"
        assert abs(fp["sum"] - sm) <= 1e-12 * abs(sm), (q, fp["sum"], sm)


@pytest.mark.timeout(1500)
def test_bench_allreduce_at_headline_size_gloo():
    """the north star's literal multi-GPU option -- per-rank partial K over an inner slice
    of Phi's columns, summed by a bucketed all-reduce on the final kernel matrix -- once at the headline size
    (C4: N = 100k, 1M edges, m = 128): two gloo ranks on the one GPU, each holding the whole 40 GB K, one timed
    step, no serial steps (host-staged all-reduces of 40 GB take minutes).  The in-run check holds every
    rank's K to the K tolerance of Phi Phi^T (K 1 and K v over all 10^10 entries against the gathered Phi) --
    not bit-identity: fp32 partials are added in the collective's order.  The line reports every rank's
    all-reduce time and bytes.  GRF_TEST_OUT=<dir> keeps it (profiles/r06_bench_allreduce_gloo_n2.json)."""
    import json
    import os
    import socket
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GRF_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "2", "--mode", "allreduce", "--steps", "1", "--warmup", "1", "--serial-steps", "0",
           "--no-cpu-baseline"]
    r = _run_beating(cmd, root, env, 1400, "allreduce_gloo_n2")
    out_dir = os.environ.get("GRF_TEST_OUT")
    if r.returncode != 0 and out_dir:
        with open(os.path.join(out_dir, "allreduce_gloo_n2.failed.log"), "w") as fh:
            fh.write(r.stdout + "\n----- stderr -----\n" + r.stderr)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "r06_bench_allreduce_gloo_n2.json"), "w") as fh:
            fh.write(json.dumps(line) + "\n")
    d = line["distributed"]
    assert line["n_gpus"] == 2 and d["backend"] == "gloo" and d["world_size"] == 2
    assert line["config"]["n_nodes"] == 100_000 and line["config"]["walks_per_node"] == 128
    assert line["parity"]["ok"] and len(line["parity"]["per_rank"]) == 2, line["parity"]
    assert all(x > 0 for x in d["allreduce_ms_per_rank"])
    assert all(x >= 100_000 * 100_000 * 4 for x in d["allreduce_bytes_per_rank"])


@pytest.mark.parametrize("mode", ["cols", "rows", "allreduce"])
def test_bench_multi_gpu_path_on_rccl_one_rank(mode):
    """The N > 1 bench step on RCCL itself (backend "nccl"), one rank on the one-GPU box
    (GRF_DIST_FORCE=1): the Phi all-gather, the timing / parity all-reduces and the all-reduce mode's
    bucketed K sums run through RCCL with exactly the code the driver's 8-GPU run takes; the in-run
    K block check passes.  (Several ranks on one GPU need gloo: the test above.)"""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GRF_DIST_FORCE="1")
    env.pop("GRF_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
           "--gpus", "1", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--n-nodes", "20000",
           "--edges", "200000", "--mode", mode]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    d = line["distributed"]
    assert d["backend"] == "nccl" and d["world_size"] == 1
    assert d["rank_rows"] == [20000] and d["gram_ms_per_rank"][0] > 0
    if mode != "allreduce":
        assert d["gather_bytes_sent_per_rank"][0] > 0 and d["gather_ms_per_rank"][0] > 0
    assert line["parity"]["ok"] and line["parity"]["max_ratio"] <= 1.0


@pytest.mark.parametrize("hubs", [0, 64])
def test_gram_row_cuts_bit_identical(eng, hubs):
    """Pair-balanced wave shares (grf_gram_row_cuts + grf_gram_sparse_upper_ex) give the same K bits as
    the plain whole-K Gram on a hub-heavy power-law graph, with and without the hub-column split; and
    the cuts are monotone, start at 0 and end within each row."""
    import torch

    import grf_amd.engine as E
    from grf_amd.graphs import powerlaw_graph
    A = powerlaw_graph(20000, 10.0, 2.5, seed=11)
    G = eng.laplacian(A)
    phi = eng.compact(eng.walk_phi(G, 32, 0.1, 6, [1.0, -0.5, 0.125, -0.02, 0.003, -0.0005], seed=5, want64=False),
                      want64=False)
    old = E.ROW_CUTS
    try:
        E.ROW_CUTS = "0"
        K0 = eng.gram_sparse_sym_hubs(phi, eng.transpose_banded(phi, 4096), hubs).clone()
        E.ROW_CUTS = "1"
        tr = eng.transpose_banded(phi, 4096)
        cuts = eng.row_cuts(phi, tr).view(-1, 8).cpu().numpy()
        K1 = eng.gram_sparse_sym_hubs(phi, tr, hubs)
    finally:
        E.ROW_CUTS = old
    nnz = np.diff(phi.ptr.cpu().numpy())
    assert (cuts[:, 0] == 0).all() and (np.diff(cuts, axis=1) >= 0).all() and (cuts[:, 7] <= nnz).all()
    assert torch.equal(K0, K1)


def test_compaction_row_stats_give_same_shifts(eng):
    """compact(..., stats=True) leaves the rows' Gram shift statistics; phi_row_shifts from them equals
    the separate pass over the values bit for bit (power-law graph, rows of very different norms; a row
    count that leaves the last wave's group of four rows partial)."""
    import torch

    from grf_amd.graphs import powerlaw_graph
    A = powerlaw_graph(30003, 10.0, 2.5, seed=4)
    G = eng.laplacian(A)
    rows = eng.walk_phi(G, 64, 0.1, 8, [1.0, 0.5, 0.25, 0.125, 0.06, 0.03, 0.015, 0.008], seed=9, want64=False)
    a = eng.compact(rows, want64=False, want32=True, sync_free=True, stats=True)
    b = eng.compact(rows, want64=False, want32=True, sync_free=True)
    assert a.row_stats is not None and b.row_stats is None
    nnz = int(a.ptr[-1])
    assert torch.equal(a.ptr, b.ptr) and torch.equal(a.idx[:nnz], b.idx[:nnz])
    assert torch.equal(a.val32[:nnz], b.val32[:nnz])
    assert torch.equal(eng.phi_row_shifts(a), eng.phi_row_shifts(b))


@pytest.mark.parametrize("n,k", [(1000, 1000), (3001, 2708), (8193, 777), (300, 17)])
def test_gram_dense_planes_bit_identical(eng, n, k):
    """The split Gram on planes written once (grf_split_planes / grf_densify_padded_planes +
    grf_gram_dense_planes) gives the in-register split's wide path (GRF_DENSE_WIDE=1) the same K bits: the same
    planes, the same six products per block in the same order; odd n, k not a multiple of 16, a single tile
    row.  The fused producer's planes equal the separate split's, byte for byte."""
    import os

    import torch
    g = torch.Generator(device="cpu").manual_seed(n + k)
    A = torch.zeros((n, max(64, -(-k // 64) * 64)), dtype=torch.float32)
    vals = torch.randn((n, k), generator=g) * torch.rand((n, k), generator=g).pow(3)
    A[:, :k] = torch.where(torch.rand((n, k), generator=g) < 0.3, vals, torch.zeros_like(vals))
    A = A.to(eng.device)
    old = {v: os.environ.get(v) for v in ("GRF_DENSE_WIDE", "GRF_DENSE_PLANES")}
    try:
        os.environ["GRF_DENSE_WIDE"] = "1"
        os.environ["GRF_DENSE_PLANES"] = "0"
        Kw = eng.gram_dense(A, k, precision="split").clone()
        P = eng.split_planes(A, k)
        Kp = eng.gram_dense(P, k, precision="split")
        assert torch.equal(Kw, Kp), float((Kw - Kp).abs().max())
        os.environ["GRF_DENSE_PLANES"] = "1"
        assert torch.equal(eng.gram_dense(A, k, precision="split"), Kw)  # (split inside gram_dense)
    finally:
        for v, x in old.items():
            if x is None:
                os.environ.pop(v, None)
            else:
                os.environ[v] = x
    # the fused producer: padded walk rows straight to the planes
    Ad = er_graph(n, 6, 5)
    G = eng.laplacian(Ad)
    rows = eng.walk_phi(G, 16, 0.2, 4, [1.0, -0.5, 0.25, -0.125], seed=3, want64=False)
    Pf = eng.densify_padded(rows, planes=True)
    Ps = eng.split_planes(eng.densify_padded(rows), n)
    assert torch.equal(Pf.P, Ps.P)
