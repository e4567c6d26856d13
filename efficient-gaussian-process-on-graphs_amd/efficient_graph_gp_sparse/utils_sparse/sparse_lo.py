"""SparseLinearOperator: mirror of utils_sparse/sparse_lo.py:4-25.

Subclasses ``linear_operator.operators.LinearOperator`` when that package is
installed (as in the reference); otherwise a minimal stand-in with the same
methods (``_matmul``, ``_size``, ``_transpose_nonbatch``, ``@``, ``shape``) so the
preprocessor and kernels work without gpytorch.
"""
import torch

try:
    from linear_operator.operators import LinearOperator as _Base
    _HAVE_LO = True
except ImportError:  # pragma: no cover - depends on the environment
    _Base = object
    _HAVE_LO = False


class SparseLinearOperator(_Base):
    """Wraps a torch sparse CSR tensor (device resident)."""

    def __init__(self, sparse_csr_tensor):
        if not sparse_csr_tensor.is_sparse_csr:
            raise ValueError("Input tensor must be a sparse CSR tensor")
        self.sparse_csr_tensor = sparse_csr_tensor
        if _HAVE_LO:
            super().__init__(sparse_csr_tensor)

    def _matmul(self, rhs):
        return self.sparse_csr_tensor.matmul(rhs)

    def _size(self):
        return self.sparse_csr_tensor.size()

    def _transpose_nonbatch(self):
        return SparseLinearOperator(self.sparse_csr_tensor.t().to_sparse_csr())

    if not _HAVE_LO:
        def __matmul__(self, rhs):
            return self._matmul(rhs)

        def size(self, dim=None):
            s = self._size()
            return s if dim is None else s[dim]

        @property
        def shape(self):
            return self._size()

        def t(self):
            return self._transpose_nonbatch()

        def to_dense(self):
            return self.sparse_csr_tensor.to_dense()
