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
