"""Graph kernels (mirror of efficient_graph_gp/graph_kernels/__init__.py).

Only the GRF path is accelerated; the exact-kernel helpers of the reference
(diffusion_kernel, feature_matrix_kernel, networkx grf_kernel) are outside the
hot-path scope of this engine and raise NotImplementedError.
"""
from .fast_grf_kernel_diffusion import fast_diffusion_grf_kernel
from .fast_grf_kernel_general import fast_general_grf_kernel
from .utils import generate_noisy_samples, get_normalized_laplacian


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"{name} is outside the GRF hot path this engine implements (see DESIGN.md)")
    f.__name__ = name
    return f


diffusion_kernel = _out_of_scope("diffusion_kernel")
feature_matrix_kernel = _out_of_scope("feature_matrix_kernel")
grf_kernel = _out_of_scope("grf_kernel")

__all__ = ["get_normalized_laplacian", "generate_noisy_samples", "diffusion_kernel", "feature_matrix_kernel",
           "grf_kernel", "fast_diffusion_grf_kernel", "fast_general_grf_kernel"]
