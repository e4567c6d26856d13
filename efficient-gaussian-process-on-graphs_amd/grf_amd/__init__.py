"""grf_amd -- MI355X-native Graph Random Features engine.

Core device pipeline: :class:`grf_amd.engine.GRFEngine`.  Drop-in mirrors of
the reference's Python API live in the sibling packages ``efficient_graph_gp``
and ``efficient_graph_gp_sparse``.
"""
from . import _lib
from ._lib import (LAP_COMBINATORIAL, LAP_NONE, LAP_NUMPY, LAP_NUMPY_SAFE, LAP_SCIPY, LOAD_ABLATION,
                   LOAD_CUMULATIVE, LOAD_NONCUMULATIVE, NORM_DIV, NORM_MUL_RECIP, RNG_PCG64, RNG_PHILOX)

__all__ = ["_lib", "RNG_PCG64", "RNG_PHILOX", "LOAD_CUMULATIVE", "LOAD_NONCUMULATIVE", "LOAD_ABLATION", "NORM_DIV",
           "NORM_MUL_RECIP", "LAP_SCIPY", "LAP_NUMPY", "LAP_NUMPY_SAFE", "LAP_COMBINATORIAL", "LAP_NONE",
           "GRFEngine", "get_engine"]


def __getattr__(name):
    if name in ("GRFEngine", "get_engine", "DeviceCSR"):
        from . import engine
        return getattr(engine, name)
    raise AttributeError(name)
