"""Statistical pin of the GPU's Philox estimator (SURVEY.md §7 gate iii).

Every other GPU test compares the HIP walks with the oracle's C restatement of the same walk, so a
slip shared by both (halt threshold ceil(p 2^32), the Lemire neighbour draw, the load rule, the
skipped last move) would pass them all.  Here the GPU's walks are checked against the *exact*
walk tensor the reference itself computes, ``compute_pstep_walk_matrix``
(``efficient_graph_gp/gpflow_kernels/general_kernel_pofm.py:7-42``; fixture
``tests/golden/pstep.npz`` made by ``make_golden.py pstep`` from the reference function):
E[M_l] = W^l, and for the bench's fused walk -> Phi kernel E[Phi] = sum_l f_l W^l, within CLT bounds
over independent seeds (``oracle.clt_check``: z <= 6 per entry that is nonzero in >= 75 % of the
replicas, per row sum and per step total).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from golden_util import csr
from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEEDS = range(100, 228)


@pytest.fixture(scope="module")
def eng():
    from grf_amd.engine import GRFEngine
    return GRFEngine("cuda:0")


def _gpu_step_replicas(eng, W, m, p, L, seeds):
    G = eng.to_device(sp.csr_matrix(W))
    reps = []
    for s in seeds:
        st = eng.steps(eng.walk(G, m, p, L, seed=s))
        reps.append(eng.steps_dense(st).cpu().numpy())
    return np.stack(reps)


@pytest.mark.parametrize("name,p", [("er40", 0.1), ("wer30", 0.3), ("iso25", 0.2), ("star10", 0.5)])
def test_philox_walk_steps_unbiased(eng, golden, name, p):
    d = golden("pstep")
    reps = _gpu_step_replicas(eng, d[f"{name}_P"], 256, p, int(d["p_max"][0]), SEEDS)
    ok, worst, k = O.clt_check(reps, d[f"{name}_rw_pstep"])
    assert ok and k > 0, (worst, k)


@pytest.mark.parametrize("name", ["er40", "wer30"])
def test_philox_walk_steps_unbiased_on_laplacian(eng, golden, name):
    """Signed weights, diagonal entries walked: the first three steps (see the oracle test)."""
    d = golden("pstep")
    sg = golden("small_graphs")
    A = sg[f"{name}_A"]
    reps = _gpu_step_replicas(eng, csr(sg, f"{name}_Lsp", A.shape[0]), 1024, 0.1, 3, range(200, 248))
    ok, worst, k = O.clt_check(reps, d[f"{name}_pstep"][:, :, :3])
    assert ok and k > 0, (worst, k)


@pytest.mark.parametrize("name,p", [("er40", 0.1), ("wer30", 0.3), ("star10", 0.5)])
def test_fused_walk_phi_unbiased(eng, golden, name, p):
    """The bench's kernel (grf_walk_phi over the augmented walk matrix, fp32 Phi): E[Phi] = sum f_l W^l."""
    d = golden("pstep")
    W = d[f"{name}_P"]
    T = d[f"{name}_rw_pstep"]
    L = T.shape[2]
    f = np.array([1.0, -0.6, 0.3, -0.15, 0.05])[:L]
    G = eng.to_device(sp.csr_matrix(W))
    reps = []
    for s in SEEDS:
        phi = eng.compact(eng.walk_phi(G, 256, p, L, f, seed=s, want64=False), want64=False)
        reps.append(phi.to_scipy().toarray())
    ok, worst, k = O.clt_check(np.stack(reps)[..., None], (T @ f)[..., None])
    assert ok and k > 0, (worst, k)


def test_degree_one_walks_exact(eng, golden):
    """Degree-1 walks with p_halt = 0 draw nothing and never halt: M_l = P^l exactly, in both the
    slot walker and the fused walk -> Phi kernel."""
    d = golden("pstep")
    P = golden("small_graphs")["perm12_A"]
    T = d["perm12_raw_pstep"]
    got = _gpu_step_replicas(eng, P, 64, 0.0, T.shape[2], [3])[0]
    np.testing.assert_array_equal(got, T)
    f = np.array([1.0, 0.5, 0.25, 0.125, 0.0625])
    G = eng.to_device(sp.csr_matrix(P))
    phi = eng.compact(eng.walk_phi(G, 64, 0.0, T.shape[2], f, seed=3)).to_scipy().toarray()
    np.testing.assert_array_equal(phi, T @ f)


def _gpu_functionals(eng, G, m, p, L, rng, seed, n_chunks=1):
    """oracle.step_functionals of one GPU replica, computed on the device from the walk slots."""
    import torch
    sl = eng.walk(G, m, p, L, rng=rng, seed=seed, n_chunks=n_chunks)
    node, load = sl.node, sl.load
    vis = node >= 0
    lv = torch.where(vis, load, torch.zeros((), dtype=load.dtype, device=load.device))
    src = torch.arange(node.shape[0], device=node.device)[:, None, None]
    back = torch.where(node == src, lv, torch.zeros((), dtype=lv.dtype, device=lv.device))
    prev = lv[:, :-1, :]
    mult = torch.zeros_like(lv)
    mult[:, 1:, :] = torch.where(vis[:, 1:, :] & (prev != 0), lv[:, 1:, :].abs() / torch.where(prev != 0, prev.abs(),
                                                                                               torch.ones_like(prev)),
                                 torch.zeros((), dtype=lv.dtype, device=lv.device))
    f = torch.stack([vis.sum(dim=(0, 2)).to(torch.float64), lv.abs().sum(dim=(0, 2)), lv.sum(dim=(0, 2)),
                     back.sum(dim=(0, 2)), mult.sum(dim=(0, 2))], dim=1) / m
    return f.cpu().numpy()


@pytest.mark.parametrize("name", ["cora", "wer30"])
def test_philox_vs_reference_stream_all_steps(eng, golden, name):
    """Every step the bench walks (L = 8) on the signed normalised Laplacian: the GPU's Philox walker
    against the GPU's replay of the reference's own PCG64 stream (bit-exact to the reference's golden
    step matrices elsewhere in this suite), by the two-sample rank statistic of
    tests/test_estimator_twosample.py (per-step visits, sum |load|, sum load, loads back at the source,
    summed step multipliers; Mann-Whitney |z| <= 5 for each of the 35 (step, functional) pairs; a planted
    1 % bias at step 5 reaches |z| = 6.8 on the oracle).  Cora: the golden adjacency, m = 1024;
    wer30: the weighted 30-node golden graph, m = 65536."""
    from grf_amd import _lib as C
    if name == "cora":
        d = golden("cora")
        n = len(d["A_indptr"]) - 1
        A = sp.csr_matrix((d["A_data"], d["A_indices"], d["A_indptr"]), shape=(n, n))
        G = eng.laplacian(A)
        m = 1024
    else:
        sg = golden("small_graphs")
        n = sg["wer30_A"].shape[0]
        G = eng.to_device(csr(sg, "wer30_Lsp", n))
        m = 65536
    R, L, p = 32, 8, 0.1
    x = np.stack([_gpu_functionals(eng, G, m, p, L, C.RNG_PHILOX, 3000 + r) for r in range(R)])
    y = np.stack([_gpu_functionals(eng, G, m, p, L, C.RNG_PCG64, 200000 + 10000 * r, n_chunks=n) for r in range(R)])
    z = O.mann_whitney_z(x, y)
    assert np.abs(z).max() <= 5.0, np.round(z, 2)
