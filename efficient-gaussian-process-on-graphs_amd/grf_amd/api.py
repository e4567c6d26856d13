"""Host-side implementation of the reference's GRF entry points on the MI355X engine.

The mirror packages ``efficient_graph_gp`` / ``efficient_graph_gp_sparse`` keep the
reference's module paths and signatures and call into this module; this module
only marshals arrays to the device and calls :class:`grf_amd.engine.GRFEngine`
(every arithmetic step runs in ``libgrf_amd.so``).

RNG modes (keyword ``rng`` on every entry point, default from ``GRF_AMD_RNG``,
else ``"reference"``):

``"reference"``
    numpy PCG64 replay with the reference's own chunking and seeds -- the step
    matrices are bit-identical to the reference's on the same ``n_processes``
    (which the reference takes from ``os.cpu_count()`` when None).
``"philox"``
    counter-based Philox4x32-10 keyed by (seed, source, walk): same estimator,
    independent of the process / GPU count, and fully parallel on the GPU.
"""
from __future__ import annotations

import os
import secrets
from typing import Optional, Sequence

import numpy as np
import scipy.sparse as sp
import torch

from . import _lib as C
from .engine import DeviceCSR, GRFEngine, get_engine

RNG_MODES = ("reference", "philox")


def resolve_rng(rng: Optional[str]) -> str:
    rng = (rng or os.environ.get("GRF_AMD_RNG") or "reference").lower()
    if rng not in RNG_MODES:
        raise ValueError(f"rng must be one of {RNG_MODES}, got {rng!r}")
    return rng


def resolve_processes(n_processes: Optional[int]) -> int:
    """The reference's default: os.cpu_count() (sampler.py:111-112, sparse_sampler.py:351-352)."""
    n = os.cpu_count() if n_processes is None else int(n_processes)
    if n < 1:
        raise ValueError("n_processes must be >= 1")
    return n


def _check_len(modulator_vector, max_walk_length):
    f = np.asarray(modulator_vector, dtype=np.float64).reshape(-1)
    if f.shape[0] != max_walk_length:
        # numpy's matmul error in the reference (fast_grf_kernel_general.py:38)
        raise ValueError(f"matmul: Input operand 1 has a mismatch in its core dimension 0 "
                         f"(size {f.shape[0]} is different from {max_walk_length})")
    return f


# --------------------------------------------------------------------- sparse path
def sparse_laplacian(adj, device=None) -> sp.csr_matrix:
    """utils_sparse/graph_utils.py:5-30 on the device."""
    eng = get_engine(device)
    return eng.laplacian(_canonical_csr(adj)).to_scipy()


def _canonical_csr(adj) -> sp.csr_matrix:
    A = sp.csr_matrix(adj, dtype=np.float64)
    if A.shape[0] != A.shape[1]:
        raise ValueError("Adjacency matrix must be square.")
    if not A.has_canonical_format:
        A = A.copy()
        A.sum_duplicates()  # scipy would take its non-canonical binop path; we canonicalise
    return A


def _sparse_walk(eng: GRFEngine, G: DeviceCSR, num_walks, p_halt, max_walk_length, seed, n_processes, rng):
    rng = resolve_rng(rng)
    base = int(seed or 42)
    if rng == "reference":
        return eng.walk(G, num_walks, p_halt, max_walk_length, rng=C.RNG_PCG64, seed=base,
                        n_chunks=resolve_processes(n_processes))
    return eng.walk(G, num_walks, p_halt, max_walk_length, rng=C.RNG_PHILOX, seed=base)


def sparse_step_matrices(walk_matrix, num_walks, p_halt, max_walk_length, seed=None, n_processes=None, rng=None,
                         device=None) -> list:
    """SparseRandomWalk(walk_matrix, seed).get_random_walk_matrices(...) (sparse_sampler.py:72-132)."""
    return [M.to_scipy() for M in sparse_step_matrices_device(walk_matrix, num_walks, p_halt, max_walk_length, seed,
                                                              n_processes, rng, device)]


def sparse_step_matrices_device(walk_matrix, num_walks, p_halt, max_walk_length, seed=None, n_processes=None,
                                rng=None, device=None, laplacian: bool = False) -> list:
    """The step matrices as device CSR (fp64 values), never leaving the GPU.  laplacian=True walks
    the normalised Laplacian of ``walk_matrix`` (GraphPreprocessor.preprocess_graph, :101-108)."""
    eng = get_engine(device)
    A = _canonical_csr(walk_matrix)
    G = eng.laplacian(A) if laplacian else eng.to_device(A)
    slots = _sparse_walk(eng, G, num_walks, p_halt, max_walk_length, seed, n_processes, rng)
    return eng.step_matrices(eng.steps(slots, C.NORM_MUL_RECIP))


def sparse_features(adj, modulator_vector, walks_per_node, p_halt, max_walk_length, *, n_processes=None, rng=None,
                    device=None, seed=None) -> DeviceCSR:
    """Phi = sum_l f_l M_l on the normalised Laplacian (graph_kernels_sparse/fast_grf_kernel_general.py:42-52)."""
    eng = get_engine(device)
    G = eng.laplacian(_canonical_csr(adj))
    f = np.asarray(modulator_vector, dtype=np.float64).reshape(-1)
    if resolve_rng(rng) == "philox" and walks_per_node * max_walk_length <= 4096:
        # the benchmarked kernel: fused Philox walks straight to Phi rows (no visit slots; the same
        # numbers as walk + features)
        return eng.compact(eng.walk_phi(G, walks_per_node, p_halt, max_walk_length, f, seed=int(seed or 42),
                                        norm=C.NORM_MUL_RECIP))
    slots = _sparse_walk(eng, G, walks_per_node, p_halt, max_walk_length, seed, n_processes, rng)
    return eng.compact(eng.features(slots, f, C.NORM_MUL_RECIP))


def sparse_kernel(adj, modulator_vector, walks_per_node=50, p_halt=0.1, max_walk_length=10, *, n_processes=None,
                  rng=None, return_format="scipy", device=None, method="auto"):
    """fast_general_grf_kernel (sparse): K = Phi Phi^T, float32 on the device."""
    eng = get_engine(device)
    phi = sparse_features(adj, modulator_vector, walks_per_node, p_halt, max_walk_length, n_processes=n_processes,
                          rng=rng, device=device)
    K = eng.gram(phi, method)
    if return_format == "torch":
        return K
    if return_format == "numpy":
        return K.cpu().numpy().astype(np.float64)
    if return_format == "scipy":
        n = K.shape[0]
        if n * n > 4_000_000_000:
            raise MemoryError(f"K has {n}x{n} entries; request return_format='torch' to keep it on the GPU")
        # built on the device, one host copy of (indptr, indices, data); drops exact zeros, like scipy's SpGEMM
        return eng.dense_to_scipy_csr(K)
    raise ValueError(f"unknown return_format {return_format!r}")


# ---------------------------------------------------------------------- dense path
def dense_walk_matrix(W, mode, device=None) -> DeviceCSR:
    eng = get_engine(device)
    W = np.asarray(W, dtype=np.float64)
    if W.ndim != 2 or W.shape[0] != W.shape[1]:
        raise ValueError("Adjacency matrix must be square.")
    return eng.walk_matrix_dense(W, mode)


def dense_laplacian(W, mode=C.LAP_NUMPY, device=None) -> np.ndarray:
    """graph_kernels/utils.py:21-26 (mode LAP_NUMPY) / preprocessing/laplacian_np.py (SAFE, COMBINATORIAL)."""
    W = np.asarray(W, dtype=np.float64)
    G = dense_walk_matrix(W, mode, device)
    Lc = G.to_scipy()
    out = np.zeros(W.shape, np.float64)
    r = np.repeat(np.arange(W.shape[0]), np.diff(Lc.indptr))
    out[r, Lc.indices] = Lc.data
    return out


def _dense_slots(eng, G, num_walks, p_halt, max_walk_length, seed, n_processes, ablation, rng):
    """Path selection of RandomWalk.get_random_walk_matrices (sampler.py:109-146)."""
    rng = resolve_rng(rng)
    n = G.n_rows
    nproc = resolve_processes(n_processes)
    sequential = nproc == 1 or n < 2 * nproc
    if sequential:
        rule = C.LOAD_ABLATION if ablation else C.LOAD_NONCUMULATIVE
        s = seed if seed is not None else secrets.randbits(63)  # default_rng(None): fresh entropy
        if rng == "reference":
            return eng.walk(G, num_walks, p_halt, max_walk_length, rng=C.RNG_PCG64, seed=int(s), n_chunks=1,
                            load_rule=rule)
        return eng.walk(G, num_walks, p_halt, max_walk_length, rng=C.RNG_PHILOX, seed=int(s), load_rule=rule)
    base = int(seed or 42)
    if rng == "reference":
        return eng.walk(G, num_walks, p_halt, max_walk_length, rng=C.RNG_PCG64, seed=base, n_chunks=nproc)
    return eng.walk(G, num_walks, p_halt, max_walk_length, rng=C.RNG_PHILOX, seed=base)


def dense_step_tensor_device(walk_matrix, num_walks, p_halt, max_walk_length, seed=None, n_processes=None,
                             ablation=False, rng=None, device=None, laplacian_mode=C.LAP_NONE) -> torch.Tensor:
    """RandomWalk(Graph(W), seed).get_random_walk_matrices(...) as an (N, N, L) float64 tensor that
    stays on the device (the GPflow wrappers keep it there: no host round trip).  W is
    ``walk_matrix`` itself (LAP_NONE) or its Laplacian of the given mode, built on the device
    (``Graph(get_normalized_laplacian(adj))``, gpflow_kernels/general_kernel_fast_grf.py:53-55)."""
    eng = get_engine(device)
    G = dense_walk_matrix(walk_matrix, laplacian_mode, device)
    slots = _dense_slots(eng, G, num_walks, p_halt, max_walk_length, seed, n_processes, ablation, rng)
    st = eng.steps(slots, C.NORM_DIV)
    return eng.steps_dense(st)


def dense_step_tensor(walk_matrix, num_walks, p_halt, max_walk_length, seed=None, n_processes=None, ablation=False,
                      rng=None, device=None) -> np.ndarray:
    """RandomWalk(Graph(walk_matrix), seed).get_random_walk_matrices(...) -> (N, N, L) float64 numpy."""
    return dense_step_tensor_device(walk_matrix, num_walks, p_halt, max_walk_length, seed, n_processes, ablation,
                                    rng, device).cpu().numpy()


def dense_kernel(adj, modulator_vector, walks_per_node=50, p_halt=0.1, max_walk_length=10, *, seed=42,
                 n_processes=None, rng=None, device=None, laplacian_mode=C.LAP_NUMPY, method="auto") -> np.ndarray:
    """fast_general_grf_kernel (dense, graph_kernels/fast_grf_kernel_general.py:31-39) -> (N, N) float64."""
    f = _check_len(modulator_vector, max_walk_length)
    eng = get_engine(device)
    G = dense_walk_matrix(adj, laplacian_mode, device)
    slots = _dense_slots(eng, G, walks_per_node, p_halt, max_walk_length, seed, n_processes, False, rng)
    phi = eng.compact(eng.phi(eng.steps(slots, C.NORM_DIV), f))
    return eng.gram(phi, method).cpu().numpy().astype(np.float64)


def diffusion_modulator(length: int, beta: float) -> float:
    """(-beta)^l / (2^l l!)  (modulation_functions/diffusion_modulator.py:3-6)."""
    import math
    return (-beta) ** length / (2 ** length * math.factorial(length))


def gram_from_features(F: np.ndarray, f: Sequence[float], device=None) -> np.ndarray:
    """K = (F f)(F f)^T for a precomputed (N, N, L) step tensor (GPflow wrappers' grf_kernel)."""
    eng = get_engine(device)
    F = np.asarray(F, dtype=np.float64)
    f = np.asarray(f, dtype=np.float64).reshape(-1)
    if F.shape[2] != f.shape[0]:
        raise ValueError("modulator length must equal the step tensor's last dimension")
    from .features import DenseSteps
    return DenseSteps(F, eng).gram(torch.from_numpy(f)).cpu().numpy().astype(np.float64)
