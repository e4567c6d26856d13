"""The reference's SparseGraphGP (models/sparse_grf_model.py) is a downstream GPyTorch model, outside the
GRF hot path; it is importable only when gpytorch is installed."""
try:
    from .sparse_grf_model import SparseGraphGP  # noqa: F401
    __all__ = ["SparseGraphGP"]
except ImportError:  # pragma: no cover
    __all__ = []
