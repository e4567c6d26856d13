from .sparse_diffusion_kernel import SparseDiffusionKernel
from .sparse_grf_kernel import SparseGRFKernel

__all__ = ["SparseGRFKernel", "SparseDiffusionKernel"]
