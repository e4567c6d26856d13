"""Dense Laplacians used by the GPflow wrappers (mirror of preprocessing/laplacian_np.py:3-35), on the GPU."""
from grf_amd import _lib as C
from grf_amd import api


def get_normalized_laplacian(W):
    """I - D^-1/2 W D^-1/2 with zero degrees treated as 1 (bit-identical to the reference)."""
    return api.dense_laplacian(W, C.LAP_NUMPY_SAFE)


def get_laplacian(W):
    """D - W (bit-identical to the reference)."""
    return api.dense_laplacian(W, C.LAP_COMBINATORIAL)
