"""Diffusion GRF kernel for GPyTorch: mirror of gptorch_kernels_sparse/sparse_diffusion_kernel.py:6-96.

f_l = sigma_f (-beta)^l / (2^l l!) with learnable positive beta and sigma_f; K and its gradient
run on the HIP kernels behind ``grf_amd.features.GRFKernelFunction`` (autograd carries dK/df to
beta and sigma_f through the modulator formula)."""
import torch

from grf_amd.features import StepMatrices, feature_matrix, grf_kernel

try:
    import gpytorch
    from gpytorch.constraints import Positive
    _Base = gpytorch.kernels.Kernel
except ImportError:  # pragma: no cover - depends on the environment
    gpytorch = None
    _Base = torch.nn.Module


def diffusion_modulator_torch(length: torch.Tensor, beta: torch.Tensor) -> torch.Tensor:
    """(-beta)^l / (2^l Gamma(l + 1)) (reference :6-24)."""
    length = length.to(dtype=beta.dtype, device=beta.device)
    two = torch.tensor(2.0, dtype=beta.dtype, device=beta.device)
    return torch.pow(-beta, length) / (torch.pow(two, length) * torch.exp(torch.lgamma(length + 1.0)))


class SparseDiffusionKernel(_Base):
    def __init__(self, max_walk_length, step_matrices_torch, **kwargs):
        super().__init__(**kwargs) if _Base is not torch.nn.Module else super().__init__()
        self.register_parameter("raw_beta", torch.nn.Parameter(torch.tensor(1.0)))
        self.register_parameter("raw_sigma_f", torch.nn.Parameter(torch.tensor(1.0)))
        if gpytorch is not None:
            self.register_constraint("raw_beta", Positive())
            self.register_constraint("raw_sigma_f", Positive())
        self.step_matrices = step_matrices_torch
        self.max_walk_length = max_walk_length
        self._steps = None

    @property
    def beta(self):
        if gpytorch is not None:
            return self.raw_beta_constraint.transform(self.raw_beta)
        return torch.nn.functional.softplus(self.raw_beta)  # gpytorch Positive() = softplus

    @property
    def sigma_f(self):
        if gpytorch is not None:
            return self.raw_sigma_f_constraint.transform(self.raw_sigma_f)
        return torch.nn.functional.softplus(self.raw_sigma_f)

    @property
    def modulator_vector(self):
        lengths = torch.arange(self.max_walk_length, dtype=self.raw_beta.dtype, device=self.raw_beta.device)
        return self.sigma_f * diffusion_modulator_torch(lengths, self.beta)

    def _step_set(self) -> StepMatrices:
        if self._steps is None:
            self._steps = StepMatrices(self.step_matrices)
        return self._steps

    def forward(self, x1_idx=None, x2_idx=None, diag=False, **params):
        return grf_kernel(self.modulator_vector, self._step_set(), x1_idx, x2_idx, diag)

    def _get_feature_matrix(self):
        return feature_matrix(self.modulator_vector, self._step_set())
