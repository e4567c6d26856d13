"""The estimator pin at every step the bench walks (L = 8) on the signed normalised Laplacian, CPU side.

``tests/test_gpu_estimator.py`` checks E[M_l] = W^l by CLT bounds, which the signed Laplacian's later
steps defeat: a walk that stays at a hub multiplies its load by deg + 1 per step (the diagonal entry 1
walked with the reference's ``load *= deg * w / (1 - p)``, sparse_sampler.py:54), so replica means are
dominated by rare huge loads.  The two-sample statistic instead compares the Philox estimator with
the reference's own PCG64 stream (``oracle.walk_slots(rng=RNG_PCG64)``, pinned bit for bit to the
reference's golden step matrices) through per-step functionals of independent replicas
(``oracle.step_functionals``: visits, sum |load|, sum load, loads back at the source, and the sum of
every step's load multipliers |load_l / load_(l-1)|, which is bounded per walk) and a
Mann-Whitney rank test per (step, functional) (``oracle.mann_whitney_z``: distribution-free, a huge
load moves one rank).  This file shows the statistic's power on the oracle -- a planted 1 % bias of
the loads at step 5 and a sign slip at step 6 fail it, the unbiased pair passes -- so the GPU test
that applies it to the HIP walkers (``test_gpu_estimator.py::test_philox_vs_reference_stream_all_steps``)
means what it says.
"""
import numpy as np
import pytest

from golden_util import csr
from oracle import oracle as O

Z_MAX = 5.0  # per (step, functional): a false alarm has probability ~6e-7 each under H0 (R = 32: complete
#              separation of the two samples reaches |z| = 6.9)


def _replicas(Ls, m, p, L, rng, seeds, n_chunks=1):
    ip, ix, dx = O._csr_arrays(Ls)
    out = []
    for s in seeds:
        node, load = O.walk_slots(ip, ix, dx, m, p, L, rng=rng, seed=s, n_chunks=n_chunks, n_threads=8)
        out.append(O.step_functionals(node, load))
    return np.stack(out)


@pytest.fixture(scope="module")
def er40_pair(golden):
    sg = golden("small_graphs")
    Ls = csr(sg, "er40_Lsp", 40)
    m, p, L, R = 16384, 0.1, 8, 32
    x = _replicas(Ls, m, p, L, O.RNG_PHILOX, range(1000, 1000 + R))
    y = _replicas(Ls, m, p, L, O.RNG_PCG64, range(5000, 5000 + 100 * R, 100), n_chunks=40)
    return x, y


def test_philox_matches_reference_stream_all_steps(er40_pair):
    x, y = er40_pair
    z = O.mann_whitney_z(x, y)
    assert np.abs(z).max() <= Z_MAX, np.abs(z).max(axis=1)


def test_two_sample_statistic_catches_planted_bias(er40_pair):
    x, y = er40_pair
    biased = y.copy()
    biased[:, 5, 1:] *= 1.01  # every load at step 5 one per cent too large (so is its multiplier)
    z = O.mann_whitney_z(x, biased)
    assert np.abs(z[5]).max() > Z_MAX, z[5]
    slip = y.copy()
    slip[:, 6, 2:] *= -1.0    # the signed loads of step 6 with the wrong sign
    assert np.abs(O.mann_whitney_z(x, slip)[6]).max() > Z_MAX


def test_mann_whitney_z_reference_values():
    """Against scipy.stats.mannwhitneyu's normal approximation (no continuity correction)."""
    from scipy.stats import mannwhitneyu, norm
    r = np.random.default_rng(3)
    x, y = r.standard_normal((17, 3)), r.standard_normal((23, 3)) + [0.0, 0.5, 1.5]
    z = O.mann_whitney_z(x, y)
    for c in range(3):
        res = mannwhitneyu(x[:, c], y[:, c], use_continuity=False, method="asymptotic")
        assert abs(2 * norm.sf(abs(z[c])) - res.pvalue) < 1e-12
    ties = np.array([[1.0], [1.0], [2.0]]), np.array([[1.0], [3.0], [3.0]])
    res = mannwhitneyu(ties[0][:, 0], ties[1][:, 0], use_continuity=False, method="asymptotic")
    assert abs(2 * norm.sf(abs(O.mann_whitney_z(*ties)[0])) - res.pvalue) < 1e-12
