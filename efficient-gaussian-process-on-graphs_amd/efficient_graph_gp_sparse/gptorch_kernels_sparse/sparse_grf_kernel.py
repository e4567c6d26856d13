"""GRF kernel for GPyTorch: mirror of gptorch_kernels_sparse/sparse_grf_kernel.py:5-61.

K[x1, x2] = Phi[x1] Phi[x2]^T with Phi = sum_l f_l M_l and a learnable modulator f.
Subclasses ``gpytorch.kernels.Kernel`` when gpytorch is installed, else
``torch.nn.Module`` with the same ``forward(x1_idx, x2_idx, diag)`` signature.
Step matrices stay on the GPU; Phi is rebuilt differentiably from them.
"""
import torch

from ._features import StepUnion, kernel_from_phi

try:
    import gpytorch
    _Base = gpytorch.kernels.Kernel
except ImportError:  # pragma: no cover - depends on the environment
    _Base = torch.nn.Module


class SparseGRFKernel(_Base):
    def __init__(self, max_walk_length, step_matrices_torch, **kwargs):
        super().__init__(**kwargs) if _Base is not torch.nn.Module else super().__init__()
        self.register_parameter("raw_modulator_vector",
                                torch.nn.Parameter(torch.randn(max_walk_length)))
        self.step_matrices = step_matrices_torch
        self._union = None

    @property
    def modulator_vector(self):
        return self.raw_modulator_vector

    def _phi_values(self):
        if self._union is None:
            self._union = StepUnion(self.step_matrices)
        return self._union.values(self.modulator_vector.to(self._union.vals[0].device))

    def forward(self, x1_idx=None, x2_idx=None, diag=False, **params):
        """K[x1, x2] (or its diagonal) = Phi[x1] Phi[x2]^T."""
        return kernel_from_phi(self._union_or_build(), self._phi_values(), x1_idx, x2_idx, diag)

    def _union_or_build(self):
        if self._union is None:
            self._union = StepUnion(self.step_matrices)
        return self._union

    def _get_feature_matrix(self):
        """Phi as a sparse COO tensor (values differentiable w.r.t. the modulator)."""
        u = self._union_or_build()
        return torch.sparse_coo_tensor(torch.stack([u.rows, u.cols]), self._phi_values(), u.shape)
