"""GPflow-style GRF kernels (mirror of efficient_graph_gp/gpflow_kernels/__init__.py).

GPflow / TensorFlow are not installed in this image, so the two fast-GRF kernels
are provided with the same constructor and ``K`` / ``K_diag`` / ``grf_kernel`` API
backed by the GPU engine (numpy in, numpy out).  The exact / PoFM / TF-walker
kernels of the reference are outside the GRF hot path and raise NotImplementedError.
"""
from .diffusion_kernel_fast_grf import GraphDiffusionFastGRFKernel
from .general_kernel_fast_grf import GraphGeneralFastGRFKernel


def _out_of_scope(name):
    class _Stub:
        def __init__(self, *a, **k):
            raise NotImplementedError(f"{name} is outside the GRF hot path this engine implements (see DESIGN.md)")
    _Stub.__name__ = name
    return _Stub


GraphDiffusionKernel = _out_of_scope("GraphDiffusionKernel")
GraphDiffusionPoFMKernel = _out_of_scope("GraphDiffusionPoFMKernel")
GraphDiffusionGRFKernel = _out_of_scope("GraphDiffusionGRFKernel")
GraphGeneralPoFMKernel = _out_of_scope("GraphGeneralPoFMKernel")

__all__ = ["GraphDiffusionKernel", "GraphDiffusionPoFMKernel", "GraphDiffusionGRFKernel",
           "GraphDiffusionFastGRFKernel", "GraphGeneralPoFMKernel", "GraphGeneralFastGRFKernel"]
