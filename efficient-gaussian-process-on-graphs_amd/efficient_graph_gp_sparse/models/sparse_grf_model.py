"""SparseGraphGP: mirror of efficient_graph_gp_sparse/models/sparse_grf_model.py:10-45.

``predict`` is the pathwise-conditioning step after the GRF path:
    f_test  = eps1 Phi_test^T,  f_train = eps1 Phi_train^T,
    V       = linear_cg(K_train_train + s2 I, y - f_train - eps2)
    samples = f_test + (K_test_train V)^T
Here K is never formed: every product is Phi[rows] (Phi[cols]^T X) on the GPU
(``grf_spmm_csr`` / ``grf_cg_gram_solve*`` in libgrf_amd.so), and the CG runs the
same linear_cg rule (per-column normalisation, eps guards, stop at k >= 10 once the
mean residual < ``gpytorch.settings.cg_tolerance`` = 1) in fp64 by default
(``cg_dtype=torch.float32`` keeps the reference's fp32 recurrence).

The random draws are taken exactly as the reference takes them (same shapes, same
order, on the test inputs' device), so a seeded torch generator gives the same eps.
Subclasses ``gpytorch.models.ExactGP`` when gpytorch is installed; otherwise a
``torch.nn.Module`` whose ``forward`` returns (mean, covariance).
"""
import torch

from grf_amd.engine import DeviceCSR, get_engine  # noqa: F401

from ..gptorch_kernels_sparse.sparse_grf_kernel import SparseGRFKernel

try:
    import gpytorch
    _Base = gpytorch.models.ExactGP
except ImportError:  # pragma: no cover - depends on the environment
    gpytorch = None
    _Base = torch.nn.Module


def _noise_value(likelihood) -> float:
    noise = likelihood.noise if hasattr(likelihood, "noise") else likelihood
    return float(noise.item() if torch.is_tensor(noise) else noise)


class SparseGraphGP(_Base):
    def __init__(self, x_train, y_train, likelihood, step_matrices, max_walk_length):
        if gpytorch is not None:
            super().__init__(x_train, y_train, likelihood)
            self.mean_module = gpytorch.means.ZeroMean()
        else:
            super().__init__()
            self.likelihood = likelihood
        self.x_train, self.y_train = x_train, y_train
        self.covar_module = SparseGRFKernel(max_walk_length=max_walk_length, step_matrices_torch=step_matrices)
        self.num_nodes = step_matrices[0].shape[0]

    def forward(self, x):
        if gpytorch is not None:
            return gpytorch.distributions.MultivariateNormal(self.mean_module(x), self.covar_module(x))
        K = self.covar_module(x, x)
        return torch.zeros(K.shape[0], dtype=K.dtype, device=K.device), K

    def _phi_csr(self, device) -> DeviceCSR:
        """Phi = sum_l f_l M_l (current modulator) as a device CSR (rows ascending, columns
        ascending within a row, fp32 values; grf_phi_steps_csr on the kernel's step matrices)."""
        phi = self.covar_module._step_set().phi(self.covar_module.modulator_vector)
        if phi.ptr.device != torch.device(device):
            raise ValueError("predict: the step matrices live on another device than x_test")
        return phi

    @torch.no_grad()
    def predict(self, x_test, n_samples=64, cg_dtype=torch.float64, max_iter=1000, tolerance=None):
        """(n_samples x n_test) posterior samples (float32, like the reference)."""
        dev = x_test.device
        train_indices = self.x_train.int().flatten()
        test_indices = x_test.int().flatten()
        eng = get_engine(dev if dev.type == "cuda" else None)
        phi = self._phi_csr(eng.device)

        noise_variance = _noise_value(self.likelihood)
        noise_std = torch.sqrt(torch.tensor(noise_variance, device=dev))
        # the reference's draws, same shapes and order (sparse_grf_model.py:36-37)
        eps1_batch = torch.randn(n_samples, self.num_nodes, device=dev)
        eps2_batch = noise_std * torch.randn(n_samples, len(train_indices), device=dev)
        if tolerance is None:
            tolerance = gpytorch.settings.cg_tolerance.value() if gpytorch is not None else 1.0
        out, self.last_cg_iterations = eng.pathwise_predict(
            phi, train_indices.to(eng.device), test_indices.to(eng.device), self.y_train, noise_variance,
            eps1_batch, eps2_batch, tolerance=tolerance, max_iter=max_iter, dtype=cg_dtype)
        return out.to(torch.float32)
