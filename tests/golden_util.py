"""Helpers to read CSR triples out of the golden .npz files."""
import numpy as np
import scipy.sparse as sp


def csr(d, prefix, n):
    return sp.csr_matrix((d[prefix + "_data"], d[prefix + "_indices"], d[prefix + "_indptr"]), shape=(n, n))


def same_csr(a, b) -> bool:
    """Bitwise equality of structure and values (explicit zeros included)."""
    a, b = sp.csr_matrix(a), sp.csr_matrix(b)
    return (a.shape == b.shape and np.array_equal(np.asarray(a.indptr, np.int64), np.asarray(b.indptr, np.int64))
            and np.array_equal(a.indices, b.indices)
            and np.array_equal(a.data.view(np.uint64), np.asarray(b.data, np.float64).view(np.uint64)))


def digest(M) -> str:
    import hashlib
    M = sp.csr_matrix(M)
    h = hashlib.sha256()
    for x in (np.asarray(M.indptr, np.int64), np.asarray(M.indices, np.int32), np.asarray(M.data, np.float64)):
        h.update(np.ascontiguousarray(x).tobytes())
    return h.hexdigest()


def snap_adjacency(d, name):
    """Unit-weight CSR adjacency of a SNAP fixture (tests/golden/make_snap.py)."""
    ip, ix = d[name + "_indptr"], d[name + "_indices"]
    n = len(ip) - 1
    return sp.csr_matrix((np.ones(len(ix)), ix, ip), shape=(n, n))


def snap_k_rows(d, name, n):
    """The fixture's K rows (the reference's fp64 Phi[rows] Phi^T) as a dense array."""
    ip, ix, dx = d[name + "_K_rows_indptr"], d[name + "_K_rows_indices"], d[name + "_K_rows_data"]
    return sp.csr_matrix((dx, ix, ip), shape=(len(ip) - 1, n)).toarray()
