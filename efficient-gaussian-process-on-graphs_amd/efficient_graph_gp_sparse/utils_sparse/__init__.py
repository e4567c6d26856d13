from .graph_utils import get_normalized_laplacian
from .sparse_lo import SparseLinearOperator

__all__ = ["get_normalized_laplacian", "SparseLinearOperator"]
