"""Pin the CPU oracle against golden vectors produced by the reference itself.

These run on CPU only.  If the oracle disagrees with a golden vector the
oracle is wrong; every GPU parity test downstream trusts it.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from golden_util import csr, digest, same_csr, snap_adjacency, snap_k_rows
from oracle import oracle as O


# ----------------------------------------------------------------------------- RNG
def test_pcg64_streams_match_numpy(golden):
    d = golden("rng")
    for si in range(6):
        seed = int(str(d[f"seed{si}"][0]))
        st, inc = O.pcg64_init(seed)
        assert str(st) == str(d[f"state{si}"][0]) and str(inc) == str(d[f"state{si}"][1])
        out = O.pcg64_stream(seed, d[f"ops{si}"])
        assert np.array_equal(out.view(np.uint64), d[f"out{si}"].view(np.uint64))


def test_philox_known_answers():
    # Random123 kat_vectors for philox4x32_10
    assert list(O.philox4x32_10([0, 0, 0, 0], [0, 0])) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    ff = 0xFFFFFFFF
    assert list(O.philox4x32_10([ff] * 4, [ff, ff])) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert list(O.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_numpy_summation_orders():
    r = np.random.default_rng(11)
    for _ in range(300):
        n = int(r.integers(1, 700))
        a = r.standard_normal(n) * 10.0 ** r.integers(-6, 15, size=n)
        assert O.np_pairwise(a) == np.sum(a)
        assert O.np_reduceat(a) == np.add.reduceat(a, [0])[0]


# ------------------------------------------------------------------------ Laplacians
def test_laplacians(golden):
    d = golden("small_graphs")
    for name in d["names"]:
        A = d[f"{name}_A"]
        n = A.shape[0]
        L, _ = O.laplacian_sparse(sp.csr_matrix(A))
        assert same_csr(L, csr(d, f"{name}_Lsp", n)), name
        for mode, key in ((0, "Ld"), (1, "Lnp"), (2, "Lcomb")):
            got = O.laplacian_dense(A, mode)
            assert np.array_equal(got.view(np.uint64), d[f"{name}_{key}"].view(np.uint64)), (name, key)


# --------------------------------------------------------------------------- samplers
def test_sparse_sampler_bitwise(golden):
    d = golden("small_graphs")
    for name in d["names"]:
        n = d[f"{name}_A"].shape[0]
        Ls = csr(d, f"{name}_Lsp", n)
        p = 0.0 if name == "perm12" else 0.2
        for nproc in (1, 3, 8):
            for seed in (None, 7):
                mats = O.sparse_random_walk(Ls, 20, p, 4, n_processes=nproc, seed=seed)
                for l, M in enumerate(mats):
                    assert same_csr(M, csr(d, f"{name}_sp_n{nproc}_s{seed}_l{l}", n)), (name, nproc, seed, l)
        mats = O.sparse_random_walk(sp.csr_matrix(d[f"{name}_A"]), 15, 0.3, 3, n_processes=2, seed=0)
        for l, M in enumerate(mats):
            assert same_csr(M, csr(d, f"{name}_spA_l{l}", n)), (name, "rawA", l)


def test_dense_sampler_bitwise(golden):
    d = golden("small_graphs")
    for name in d["names"]:
        A = d[f"{name}_A"]
        n = A.shape[0]
        Ld = d[f"{name}_Ld"]
        p = 0.0 if name == "perm12" else 0.2
        for seed in (0, 5):
            F = O.dense_random_walk(Ld, 12, p, 4, n_processes=1, seed=seed)
            assert np.array_equal(F.view(np.uint64), d[f"{name}_dseq_s{seed}"].view(np.uint64)), (name, seed)
        F = O.dense_random_walk(Ld, 12, p, 4, n_processes=1, seed=0, ablation=True)
        assert np.array_equal(F.view(np.uint64), d[f"{name}_dabl_s0"].view(np.uint64)), name
        for nproc in (2, 3):
            key = f"{name}_dpar_n{nproc}"
            if key in d:
                F = O.dense_random_walk(Ld, 12, p, 4, n_processes=nproc, seed=None)
                assert np.array_equal(F.view(np.uint64), d[key].view(np.uint64)), (name, nproc)


# ----------------------------------------------------------------------- entry points
def _sparse_entry(A, f, m, p, L, nproc):
    Ls, _ = O.laplacian_sparse(sp.csr_matrix(A))
    mats = O.sparse_random_walk(Ls, m, p, L, n_processes=nproc, seed=None)
    phi = O.phi_sparse(mats, f)
    return O.gram_rows(phi)


def test_entry_points(golden):
    d = golden("entry_points")
    g = golden("small_graphs")
    nproc = int(d["cpu_count"][0])
    f = np.array([1.0, 0.5, 0.25])
    # sparse entry point: scipy SpGEMM order restated exactly -> bitwise
    K = _sparse_entry(g["readme_A"], f, 50, 0.1, 3, nproc)
    assert np.array_equal(K, d["readme_sparse_K"])
    K = _sparse_entry(g["cycle4_A"], f, 10, 0.2, 3, nproc)
    assert np.array_equal(K, d["cycle4_sparse_K"])
    K = _sparse_entry(g["er40_A"], [1.0, -0.4, 0.3, 0.1, -0.05], 32, 0.15, 5, nproc)
    assert np.array_equal(K, d["er40_sparse_K"])
    # dense entry point (README quickstart, K[0,:] quoted in SURVEY.md): BLAS order -> 1e-12
    A = g["readme_A"]
    F = O.dense_random_walk(O.laplacian_dense(A, 0), 50, 0.1, 3, n_processes=nproc, seed=42)
    Phi = np.einsum("ijl,l->ij", F, f)
    K = Phi @ Phi.T
    np.testing.assert_allclose(K, d["readme_dense_K"], rtol=1e-12, atol=1e-14)
    assert abs(d["readme_dense_K"][0, 0] - 2.1806250000000005) < 1e-12
    fm = d["diff_mod_b1"][:3]
    Phi = np.einsum("ijl,l->ij", F, fm)
    np.testing.assert_allclose(Phi @ Phi.T, d["readme_dense_diff_K"], rtol=1e-12, atol=1e-14)


def test_cora(golden):
    d = golden("cora")
    n = len(d["A_indptr"]) - 1
    A = csr(d, "A", n)
    Lc, _ = O.laplacian_sparse(A)
    assert digest(Lc) == str(d["L_digest"][0])
    mats = O.sparse_random_walk(Lc, 16, 0.1, 4, n_processes=8)
    for l, M in enumerate(mats):
        assert same_csr(M, csr(d, f"m16_l{l}", n)), l
    mats = O.sparse_random_walk(Lc, 128, 0.1, 8, n_processes=8)
    assert [digest(M) for M in mats] == [str(x) for x in d["m128_digests"]]
    f = np.array([(-1.0) ** l / (2.0 ** l * float(np.prod(np.arange(1, l + 1)))) for l in range(8)])
    phi = O.phi_sparse(mats, f)
    assert digest(phi) == str(d["m128_phi_digest"][0])
    K = O.gram_rows(phi, 0, 16)
    assert np.array_equal(K, d["m128_K_rows0_16"])


def test_reference_smoke_properties(toy_cycle_adj, toy_cycle_csr):
    """The reference's own 4 tests (tests/test_grf_dense.py, tests/test_grf_sparse.py) on the oracle."""
    F = O.dense_random_walk(toy_cycle_adj, 5, 0.2, 3, n_processes=1, seed=0)
    assert F.shape == (4, 4, 3) and np.allclose(np.diag(F[:, :, 0]), 1.0)
    mats = O.sparse_random_walk(toy_cycle_csr, 5, 0.2, 3, n_processes=1, seed=0)
    assert len(mats) == 3 and all(M.shape == (4, 4) for M in mats)
    assert np.allclose(mats[0].diagonal(), 1.0)
    K = _sparse_entry(toy_cycle_csr, [1.0, 0.5, 0.25], 10, 0.2, 3, 1)
    assert np.allclose(K, K.T, atol=1e-8) and np.linalg.eigvalsh(K).min() >= -1e-8


@pytest.mark.parametrize("rule", [O.LOAD_CUMULATIVE, O.LOAD_NONCUMULATIVE, O.LOAD_ABLATION])
def test_philox_walk_is_deterministic_and_chunk_free(rule):
    r = np.random.default_rng(0)
    U = np.triu((r.random((50, 50)) < 0.1).astype(float), 1)
    L, _ = O.laplacian_sparse(sp.csr_matrix(U + U.T))
    ip, ix, dx = O._csr_arrays(L)
    a = O.walk_slots(ip, ix, dx, 16, 0.2, 5, rng=O.RNG_PHILOX, load_rule=rule, seed=9, n_threads=1)
    b = O.walk_slots(ip, ix, dx, 16, 0.2, 5, rng=O.RNG_PHILOX, load_rule=rule, seed=9, n_threads=8)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert (a[0][:, 0, :] == np.arange(50)[:, None]).all()


@pytest.mark.parametrize("name", ["facebook", "enron"])
def test_snap_graphs(golden, name):
    """Real social graphs the reference ships: the oracle reproduces the reference's
    Laplacian, step matrices and Phi bit-exactly (8 chunks), and its K rows (tests/golden/make_snap.py)."""
    d = golden("snap")
    A = snap_adjacency(d, name)
    m, p, L = d[f"{name}_walk"]
    Lc, _ = O.laplacian_sparse(A)
    assert digest(Lc) == str(d[f"{name}_L_digest"][0])
    mats = O.sparse_random_walk(Lc, int(m), float(p), int(L), n_processes=8)
    assert [digest(M) for M in mats] == [str(x) for x in d[f"{name}_step_digests"]]
    f = np.array([(-1.0) ** l / (2.0 ** l * float(np.prod(np.arange(1, l + 1)))) for l in range(int(L))])
    phi = O.phi_sparse(mats, f)
    assert digest(phi) == str(d[f"{name}_phi_digest"][0])
    rows = d[f"{name}_K_rows"]
    Kref = snap_k_rows(d, name, A.shape[0])
    for i, r in enumerate(rows):
        np.testing.assert_allclose(O.gram_rows(phi, int(r), int(r) + 1)[0], Kref[i], rtol=1e-12, atol=1e-15)
    np.testing.assert_allclose(np.asarray(phi.multiply(phi).sum(axis=1)).ravel(), d[f"{name}_K_diag"], rtol=1e-12)


def test_pstep_restatement_matches_reference(golden):
    """oracle.pstep_walk_matrix restates compute_pstep_walk_matrix (general_kernel_pofm.py:7-42);
    the fixture is the reference function's own output (tests/golden/make_golden.py pstep)."""
    d = golden("pstep")
    sg = golden("small_graphs")
    p_max = int(d["p_max"][0])
    for name in d["names"]:
        A = sg[f"{name}_A"]
        L = csr(sg, f"{name}_Lsp", A.shape[0]).toarray()
        np.testing.assert_allclose(O.pstep_walk_matrix(L, p_max), d[f"{name}_pstep"], rtol=1e-13, atol=1e-15)
    np.testing.assert_array_equal(O.pstep_walk_matrix(sg["perm12_A"], p_max), d["perm12_raw_pstep"])


def _estimator_replicas(W, m, p, p_max, seeds, rng=O.RNG_PHILOX):
    ip, ix, dx = O._csr_arrays(sp.csr_matrix(W))
    reps = []
    for seed in seeds:
        node, load = O.walk_slots(ip, ix, dx, m, p, p_max, rng=rng, seed=seed, n_chunks=1)
        reps.append(np.stack([M.toarray() for M in O.reduce_steps(node, load, O.NORM_MUL_RECIP)], axis=-1))
    return np.stack(reps)


@pytest.mark.parametrize("name,p", [("er40", 0.1), ("wer30", 0.3), ("iso25", 0.2), ("star10", 0.5)])
@pytest.mark.parametrize("rng", [O.RNG_PHILOX, O.RNG_PCG64])
def test_oracle_estimator_is_unbiased(golden, name, p, rng):
    """SURVEY.md §7 gate (iii) on the oracle's walks (both RNG streams): E[M_l] = W^l, the reference's
    exact walk tensor (compute_pstep_walk_matrix), within CLT bounds over independent seeds.  W is the
    row-stochastic D^-1 A (weighted, isolated rows, a star), where every load is (1-p)^-l and the
    replica means are near-Gaussian; this pins the estimator itself (halt threshold, Lemire draw,
    cumulative load deg*w/(1-p)), not one implementation against another."""
    d = golden("pstep")
    reps = _estimator_replicas(d[f"{name}_P"], 256, p, int(d["p_max"][0]), range(100, 228), rng)
    ok, worst, k = O.clt_check(reps, d[f"{name}_rw_pstep"])
    assert ok and k > 0, (worst, k)


@pytest.mark.parametrize("name", ["er40", "wer30"])
def test_oracle_estimator_on_laplacian_short_walks(golden, name):
    """The same on the normalised Laplacian itself (signed weights, diagonal entries walked) for the
    first three steps; later steps' loads grow like (deg/(1-p))^l and are too heavy-tailed for a
    CLT bound at test sizes (the reference's PCG64 stream shows the same spread)."""
    d = golden("pstep")
    sg = golden("small_graphs")
    A = sg[f"{name}_A"]
    Ls = csr(sg, f"{name}_Lsp", A.shape[0])
    reps = _estimator_replicas(Ls, 1024, 0.1, 3, range(200, 248))
    ok, worst, k = O.clt_check(reps, d[f"{name}_pstep"][:, :, :3])
    assert ok and k > 0, (worst, k)


def test_oracle_degree_one_walks_are_exact(golden):
    """Degree-1 walks with p_halt = 0 draw nothing and never halt: M_l = P^l exactly (the raw
    permutation matrix walked as given)."""
    d = golden("pstep")
    P = golden("small_graphs")["perm12_A"]
    ip, ix, dx = O._csr_arrays(sp.csr_matrix(P))
    node, load = O.walk_slots(ip, ix, dx, 64, 0.0, 5, rng=O.RNG_PHILOX, seed=3)
    mats = O.reduce_steps(node, load, O.NORM_MUL_RECIP)
    np.testing.assert_array_equal(np.stack([M.toarray() for M in mats], axis=-1), d["perm12_raw_pstep"])
