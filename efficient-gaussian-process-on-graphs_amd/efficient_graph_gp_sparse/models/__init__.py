from .sparse_grf_model import SparseGraphGP

__all__ = ["SparseGraphGP"]
