"""GRF kernel for GPyTorch: mirror of gptorch_kernels_sparse/sparse_grf_kernel.py:5-61.

K[x1, x2] = Phi[x1] Phi[x2]^T with Phi = sum_l f_l M_l and a learnable modulator f.  The step
matrices stay on the GPU; Phi, the row selections, K (the exact fixed-point sparse Gram) and the
gradient w.r.t. f run on the HIP kernels behind ``grf_amd.features.GRFKernelFunction`` -- Phi is
never densified.  Subclasses ``gpytorch.kernels.Kernel`` when gpytorch is installed, else
``torch.nn.Module`` with the same ``forward(x1_idx, x2_idx, diag)`` signature.
"""
import torch

from grf_amd.features import StepMatrices, feature_matrix, grf_kernel

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
        self._steps = None

    @property
    def modulator_vector(self):
        return self.raw_modulator_vector

    def _step_set(self) -> StepMatrices:
        if self._steps is None:
            self._steps = StepMatrices(self.step_matrices)
        return self._steps

    def forward(self, x1_idx=None, x2_idx=None, diag=False, **params):
        """K[x1, x2] (or its diagonal) = Phi[x1] Phi[x2]^T (reference :24-49)."""
        return grf_kernel(self.modulator_vector, self._step_set(), x1_idx, x2_idx, diag)

    def _get_feature_matrix(self):
        """Phi as a torch sparse CSR tensor on the device (reference :51-61; not differentiable:
        gradients flow through ``forward``)."""
        return feature_matrix(self.modulator_vector, self._step_set())
