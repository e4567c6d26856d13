"""Differentiable Phi = sum_l f_l M_l over device-resident step matrices (shared by the GPyTorch kernels).

The union sparsity pattern of the step matrices is computed once; Phi's values are
an index_add of f[l] * M_l values onto it, so autograd flows to the modulator.
"""
import torch


def _csr_parts(mat):
    t = getattr(mat, "sparse_csr_tensor", mat)
    if t.is_sparse_csr:
        crow, col, val = t.crow_indices(), t.col_indices(), t.values()
        rows = torch.repeat_interleave(torch.arange(t.shape[0], device=crow.device), crow[1:] - crow[:-1])
        return rows, col, val, t.shape
    t = t.coalesce()
    return t.indices()[0], t.indices()[1], t.values(), t.shape


class StepUnion:
    """Union pattern of the step matrices and the scatter map of every step entry."""

    def __init__(self, step_matrices):
        parts = [_csr_parts(m) for m in step_matrices]
        self.shape = tuple(parts[0][3])
        n_cols = self.shape[1]
        keys = torch.cat([r.long() * n_cols + c.long() for r, c, _, _ in parts])
        self.vals = [v for _, _, v, _ in parts]
        self.step_of = torch.cat([torch.full((v.numel(),), l, device=keys.device, dtype=torch.long)
                                  for l, v in enumerate(self.vals)])
        uniq, inv = torch.unique(keys, sorted=True, return_inverse=True)
        self.inv = inv
        self.rows = uniq // n_cols
        self.cols = uniq % n_cols
        self.nnz = uniq.numel()

    def values(self, modulator):
        L = len(self.vals)
        f = modulator[:L].to(self.vals[0].dtype)
        contrib = torch.cat([f[l] * v for l, v in enumerate(self.vals[:f.shape[0]])])
        inv = self.inv[:contrib.numel()]
        out = torch.zeros(self.nnz, dtype=contrib.dtype, device=contrib.device)
        return out.index_add(0, inv, contrib)

    def rows_dense(self, values, idx):
        """Dense rows Phi[idx, :] (len(idx) x N); idx may repeat."""
        n_rows, n_cols = self.shape
        uniq, back = torch.unique(idx, return_inverse=True)
        pos = torch.full((n_rows,), -1, dtype=torch.long, device=values.device)
        pos[uniq] = torch.arange(uniq.numel(), device=values.device)
        sel = pos[self.rows]
        keep = sel >= 0
        out = torch.zeros((uniq.numel(), n_cols), dtype=values.dtype, device=values.device)
        out = out.index_put((sel[keep], self.cols[keep]), values[keep], accumulate=True)
        return out[back]


def kernel_from_phi(union, values, x1_idx, x2_idx, diag):
    n = union.shape[0]
    dev = values.device
    i1 = torch.arange(n, device=dev) if x1_idx is None else x1_idx.long().flatten().to(dev)
    i2 = torch.arange(n, device=dev) if x2_idx is None else x2_idx.long().flatten().to(dev)
    p1 = union.rows_dense(values, i1)
    if diag:
        p2 = p1 if x2_idx is None or torch.equal(i1, i2) else union.rows_dense(values, i2)
        return (p1 * p2).sum(dim=-1)
    p2 = p1 if torch.equal(i1, i2) else union.rows_dense(values, i2)
    return p1 @ p2.transpose(-1, -2)
