"""General-modulator fast GRF kernel: mirror of gpflow_kernels/general_kernel_fast_grf.py:9-77.

The (N, N, L) step tensor is sampled once at construction on the GPU (Laplacian with safe
degrees as in preprocessing/laplacian_np.py, or the raw adjacency with the ablation rule) and
stays on the device.  ``modulator_vector`` is a learnable parameter (``torch.nn.Parameter``, fp64:
the reference's ``gpflow.Parameter(tf.float64)``, :31-41); K = (F f)(F f)^T runs on the MFMA Gram
(fp32 result, ``GRFEngine.gram_dense``) once per modulator value and is cached, so ``K`` / ``K_diag`` only gather
from it.  ``K_torch`` returns the same block as a torch tensor that is differentiable w.r.t. the
modulator (``grf_amd.features.DenseGramFunction``).  GPflow / TensorFlow are not installed here:
the class is a ``torch.nn.Module`` and ``K`` / ``K_diag`` return numpy arrays.
"""
from typing import Optional

import numpy as np
import torch

from grf_amd import _lib as C
from grf_amd import api
from grf_amd.engine import get_engine
from grf_amd.features import DenseGramFunction, DenseSteps


def _indices(X) -> torch.Tensor:
    if torch.is_tensor(X):
        return X.reshape(-1).long()
    return torch.from_numpy(np.asarray(X).reshape(-1).astype(np.int64))


class GraphGeneralFastGRFKernel(torch.nn.Module):
    def __init__(self, adjacency_matrix, walks_per_node: int = 50, p_halt: float = 0.1, max_walk_length: int = 10,
                 random_walk_seed: int = 42, modulator_vector: np.ndarray = None, step_matrices: np.ndarray = None,
                 use_tqdm: bool = False, ablation: bool = False, *, rng: Optional[str] = None, device=None, **kwargs):
        super().__init__()
        adjacency_matrix = np.asarray(adjacency_matrix, dtype=np.float64)
        assert adjacency_matrix.shape[0] == adjacency_matrix.shape[1], "Adjacency matrix must be square."
        self.adjacency_matrix = adjacency_matrix
        self.walks_per_node = walks_per_node
        self.p_halt = p_halt
        self.max_walk_length = max_walk_length
        self.device = get_engine(device).device
        if modulator_vector is None:
            np.random.seed(42)
            init = np.random.randn(max_walk_length)
        else:
            if len(modulator_vector) != max_walk_length:
                raise ValueError("The length of the modulator vector must be equal to the max_walk_length.")
            init = np.asarray(modulator_vector, dtype=np.float64)
        self.modulator_vector = torch.nn.Parameter(torch.tensor(init, dtype=torch.float64, device=self.device))
        self._lap_mode = None
        if step_matrices is not None:
            F = torch.as_tensor(np.asarray(step_matrices, dtype=np.float64))
        elif ablation:
            F = api.dense_step_tensor_device(adjacency_matrix, walks_per_node, p_halt, max_walk_length,
                                             seed=random_walk_seed, ablation=True, rng=rng, device=device)
        else:
            # walks on the safe-degree normalised Laplacian, built and walked on the device
            self._lap_mode = C.LAP_NUMPY_SAFE
            F = api.dense_step_tensor_device(adjacency_matrix, walks_per_node, p_halt, max_walk_length,
                                             seed=random_walk_seed, rng=rng, device=device,
                                             laplacian_mode=C.LAP_NUMPY_SAFE)
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
        """The normalised Laplacian the walks ran on (reference attribute; computed on access)."""
        if self._lap_mode is None:
            raise AttributeError("laplacian: this kernel was built from given step matrices or the ablation walk")
        return api.dense_laplacian(self.adjacency_matrix, self._lap_mode, self.device)

    def grf_kernel(self, modulator_vector) -> np.ndarray:
        """The whole K (reference :74-77), fp64 numpy."""
        if torch.is_tensor(modulator_vector):
            return self._steps.gram(modulator_vector.detach()).cpu().numpy().astype(np.float64)
        fv = np.asarray(modulator_vector, dtype=np.float64)  # (host values: cached by value)
        return self._steps.gram(torch.as_tensor(fv), key=("f", fv.tobytes())).cpu().numpy().astype(np.float64)

    def K_torch(self, X1, X2=None) -> torch.Tensor:
        """K[X1, X2] on the device, differentiable w.r.t. ``modulator_vector``."""
        Kf = DenseGramFunction.apply(self.modulator_vector, self._steps)
        i1 = _indices(X1).to(Kf.device)
        i2 = i1 if X2 is None else _indices(X2).to(Kf.device)
        return Kf[i1][:, i2]

    def _gram_host_keyed(self) -> torch.Tensor:
        """The cached K keyed by the modulator's VALUES (these calls return host arrays, so reading the
        L values back costs nothing extra): a write through ``.data`` is seen too."""
        fv = self.modulator_vector.detach().to("cpu", torch.float64).numpy()
        return self._steps.gram(self.modulator_vector, key=("f", fv.tobytes()))

    def invalidate(self) -> None:
        """Drop the cached K (needed only by ``K_torch`` after a modulator write that bypasses its version
        counter, e.g. ``modulator_vector.data.copy_(...)``)."""
        self._steps.invalidate()

    def K(self, X1, X2=None) -> np.ndarray:
        """K[X1, X2] (reference :61-67): a gather from the cached K of the current modulator."""
        Kf = self._gram_host_keyed()
        i1 = _indices(X1).to(Kf.device)
        i2 = i1 if X2 is None else _indices(X2).to(Kf.device)
        return Kf[i1][:, i2].cpu().numpy().astype(np.float64)

    def K_diag(self, X) -> np.ndarray:
        """diag(K)[X] (reference :69-72), from the same cached K."""
        Kf = self._gram_host_keyed()
        i = _indices(X).to(Kf.device)
        return Kf.diagonal()[i].cpu().numpy().astype(np.float64)

    def __call__(self, X1, X2=None, full_cov=True):
        return self.K(X1, X2) if full_cov else self.K_diag(X1)
