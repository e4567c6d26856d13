"""Diffusion fast GRF kernel: mirror of gpflow_kernels/diffusion_kernel_fast_grf.py:8-60.

``beta`` and ``sigma_f`` are learnable positive parameters (the reference's
``gpflow.Parameter(..., transform=positive())``, :29-30): raw ``torch.nn.Parameter``s under a
softplus, initialised so that ``beta`` / ``sigma_f`` start at the given values.
K = sigma_f^2 (F f(beta))(F f(beta))^T on the MFMA Gram, cached per (beta, sigma_f); ``K_torch``
is differentiable w.r.t. both parameters (autograd through the modulator formula into
``grf_amd.features.DenseGramFunction``)."""
import math
from typing import Optional

import numpy as np
import torch

from grf_amd import _lib as C
from grf_amd import api
from grf_amd.engine import get_engine
from grf_amd.features import DenseGramFunction, DenseSteps

from .general_kernel_fast_grf import _indices


def _softplus_inverse(y: float) -> float:
    return y + math.log(-math.expm1(-y))


class GraphDiffusionFastGRFKernel(torch.nn.Module):
    def __init__(self, adjacency_matrix, walks_per_node: int = 50, p_halt: float = 0.1, max_walk_length: int = 10,
                 beta: float = 2.0, sigma_f: float = 1.0, random_walk_seed: int = 42, normalize_laplacian: bool = True,
                 use_tqdm: bool = False, *, rng: Optional[str] = None, device=None, **kwargs):
        super().__init__()
        adjacency_matrix = np.asarray(adjacency_matrix, dtype=np.float64)
        assert adjacency_matrix.shape[0] == adjacency_matrix.shape[1], "Adjacency matrix must be square."
        if beta <= 0 or sigma_f <= 0:
            raise ValueError("beta and sigma_f must be positive")
        self.adjacency_matrix = adjacency_matrix
        self.walks_per_node = walks_per_node
        self.p_halt = p_halt
        self.max_walk_length = max_walk_length
        self.device = get_engine(device).device
        self.raw_beta = torch.nn.Parameter(torch.tensor(_softplus_inverse(float(beta)), dtype=torch.float64,
                                                        device=self.device))
        self.raw_sigma_f = torch.nn.Parameter(torch.tensor(_softplus_inverse(float(sigma_f)), dtype=torch.float64,
                                                           device=self.device))
        self._lap_mode = C.LAP_NUMPY_SAFE if normalize_laplacian else C.LAP_COMBINATORIAL
        # the walks run on that Laplacian, built and walked on the device (no host round trip)
        F = api.dense_step_tensor_device(adjacency_matrix, walks_per_node, p_halt, max_walk_length,
                                         seed=random_walk_seed, rng=rng, device=device, laplacian_mode=self._lap_mode)
        self._steps = DenseSteps(F, get_engine(device))

    @property
    def feature_matrices_device(self) -> torch.Tensor:
        """The (N, N, L) step tensor (the reference's ``feature_matrices_tf``), resident on the device."""
        return self._steps.F

    @property
    def feature_matrices(self) -> np.ndarray:
        """Host copy of the step tensor (made on access only; the kernel never reads it)."""
        return self._steps.F.cpu().numpy()

    @property
    def laplacian(self) -> np.ndarray:
        """The Laplacian the walks ran on (reference attribute; computed on access)."""
        return api.dense_laplacian(self.adjacency_matrix, self._lap_mode, self.device)

    @property
    def beta(self) -> torch.Tensor:
        return torch.nn.functional.softplus(self.raw_beta)

    @property
    def sigma_f(self) -> torch.Tensor:
        return torch.nn.functional.softplus(self.raw_sigma_f)

    def modulator(self, beta) -> torch.Tensor:
        """(-beta)^l / (2^l l!) for l < max_walk_length (diffusion_modulator_tf.py:3-9)."""
        beta = torch.as_tensor(beta, dtype=torch.float64, device=self.device)
        l = torch.arange(self.max_walk_length, dtype=torch.float64, device=self.device)
        return torch.pow(-beta, l) / (torch.pow(torch.tensor(2.0, dtype=torch.float64, device=self.device), l)
                                      * torch.exp(torch.lgamma(l + 1.0)))

    def grf_kernel(self, beta, sigma_f) -> np.ndarray:
        """The whole K (reference :46-60), fp64 numpy."""
        b = float(beta)
        return float(sigma_f) ** 2 * self._steps.gram(self.modulator(b), key=("beta", b)).cpu().numpy().astype(np.float64)

    def K_torch(self, X1, X2=None) -> torch.Tensor:
        Kf = self.sigma_f ** 2 * DenseGramFunction.apply(self.modulator(self.beta), self._steps)
        i1 = _indices(X1).to(Kf.device)
        i2 = i1 if X2 is None else _indices(X2).to(Kf.device)
        return Kf[i1][:, i2]

    def invalidate(self) -> None:
        """Drop the cached K (the calls here key it by the host value of beta; K_torch by tensor)."""
        self._steps.invalidate()

    def _cached(self) -> torch.Tensor:
        b = float(self.beta.detach())
        return float(self.sigma_f.detach()) ** 2 * self._steps.gram(self.modulator(b), key=("beta", b))

    def K(self, X1, X2=None) -> np.ndarray:
        Kf = self._cached()
        i1 = _indices(X1).to(Kf.device)
        i2 = i1 if X2 is None else _indices(X2).to(Kf.device)
        return Kf[i1][:, i2].cpu().numpy().astype(np.float64)

    def K_diag(self, X) -> np.ndarray:
        Kf = self._cached()
        return Kf.diagonal()[_indices(X).to(Kf.device)].cpu().numpy().astype(np.float64)

    def __call__(self, X1, X2=None, full_cov=True):
        return self.K(X1, X2) if full_cov else self.K_diag(X1)
