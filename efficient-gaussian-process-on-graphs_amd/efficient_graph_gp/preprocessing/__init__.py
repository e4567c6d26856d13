from .laplacian_np import get_laplacian, get_normalized_laplacian

__all__ = ["get_normalized_laplacian", "get_laplacian"]
