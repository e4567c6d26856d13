"""Device-resident GRF features and a differentiable K[x1, x2] for the GPyTorch surface.

Replaces the tensor algebra of the reference's GPyTorch kernels
(``efficient_graph_gp_sparse/gptorch_kernels_sparse/sparse_grf_kernel.py:24-61``,
``sparse_diffusion_kernel.py:74-96``)::

    phi = sum(f_l * M_l)                      # grf_phi_steps_csr_count / _fill
    phi[x1], phi[x2]                          # grf_csr_row_lengths + grf_scan_counts + grf_csr_gather_rows
    K = phi[x1] @ phi[x2].T                   # banded transpose + grf_gram_sparse_cols (exact fixed point)
    diag = (phi[x1] * phi[x2]).sum(-1)        # grf_csr_rowdot

with the modulator gradient of ``K`` in ``backward`` (``GRFKernelFunction``):

    dL/df_l = sum_{r,s} G[r,s] (M_l[x1_r] . Phi[x2_s] + Phi[x1_r] . M_l[x2_s])
            = sum_r (M_l[x1] Z1)[r, r] + sum_s (M_l[x2] Z2)[s, s],
    Z1 = Phi[x2]^T G^T,  Z2 = Phi[x1]^T G       # grf_csr_transpose + grf_spmm_csr, then grf_csr_rows_dot_cols

Nothing here densifies Phi, and the step matrices never leave the device.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _lib as C
from .engine import DeviceCSR, GRFEngine, _p, cols_band_width, get_engine


def _torch_csr(mat) -> torch.Tensor:
    t = getattr(mat, "sparse_csr_tensor", mat)
    if not (torch.is_tensor(t) and t.is_sparse_csr):
        raise ValueError("step matrices must be torch sparse CSR tensors (or SparseLinearOperator over them)")
    return t


class StepMatrices:
    """The L step matrices of one graph on one device: int64 row pointers, int32 columns and the
    preprocessor's float32 values (views of the torch CSR tensors where the dtypes already match)."""

    def __init__(self, mats: Sequence, engine: Optional[GRFEngine] = None):
        ts = [_torch_csr(m) for m in mats]
        if not ts:
            raise ValueError("no step matrices")
        self.engine = engine or get_engine(ts[0].device if ts[0].is_cuda else None)
        dev = self.engine.device
        self.shape = tuple(ts[0].shape)
        self.steps: List[DeviceCSR] = []
        for t in ts:
            if tuple(t.shape) != self.shape:
                raise ValueError("step matrices differ in shape")
            ptr = t.crow_indices().to(dev, torch.int64).contiguous()
            idx = t.col_indices().to(dev, torch.int32).contiguous()
            val = t.values().to(dev, torch.float32).contiguous()
            self.steps.append(DeviceCSR(self.shape[0], self.shape[1], ptr, idx, None, val, int(idx.numel())))
        # host arrays of the L device pointers (the C ABI's step_ptr / step_idx / step_val)
        self._arrays = [(ctypes.c_void_p * len(self.steps))(*[getattr(s, a).data_ptr() for s in self.steps])
                        for a in ("ptr", "idx", "val32")]
        self._ptrs = [ctypes.cast(a, ctypes.c_void_p) for a in self._arrays]

    @property
    def L(self) -> int:
        return len(self.steps)

    def phi(self, f: torch.Tensor, want64: bool = False) -> DeviceCSR:
        """Phi = sum_l f_l M_l (compact CSR, fp32 values [+ fp64]) for the modulator f (len >= 1)."""
        eng = self.engine
        n = self.shape[0]
        ft = f.detach().to(eng.device, torch.float64).contiguous().flatten()
        nf = min(int(ft.numel()), self.L)
        cnt = eng._empty(n, torch.int32)
        C.check(eng.lib.grf_phi_steps_csr_count(n, self.L, self._ptrs[0], self._ptrs[1], self._ptrs[2], _p(ft), nf,
                                                _p(cnt), eng.stream), "grf_phi_steps_csr_count")
        ptr = eng._empty(n + 1, torch.int64)
        ws = eng._ws(eng.lib.grf_scan_workspace_bytes(n))
        C.check(eng.lib.grf_scan_counts(n, _p(cnt), _p(ptr), _p(ws), ws.numel(), eng.stream), "grf_scan_counts")
        nnz = int(ptr[-1].item())
        idx = eng._empty(nnz, torch.int32)
        v32 = eng._empty(nnz, torch.float32)
        v64 = eng._empty(nnz, torch.float64) if want64 else None
        C.check(eng.lib.grf_phi_steps_csr_fill(n, self.L, self._ptrs[0], self._ptrs[1], self._ptrs[2], _p(ft), nf,
                                               _p(ptr), _p(idx), _p(v64), _p(v32), eng.stream),
                "grf_phi_steps_csr_fill")
        return DeviceCSR(n, self.shape[1], ptr, idx, v64, v32, nnz)


def gather_rows(eng: GRFEngine, A: DeviceCSR, rows: torch.Tensor) -> DeviceCSR:
    """A[rows] as a compact CSR (rows may repeat)."""
    rmap = rows.to(eng.device, torch.int32).contiguous()
    n_sel = rmap.numel()
    cnt = eng._empty(n_sel, torch.int32)
    C.check(eng.lib.grf_csr_row_lengths(n_sel, _p(A.ptr), _p(rmap), _p(cnt), eng.stream), "grf_csr_row_lengths")
    ptr = eng._empty(n_sel + 1, torch.int64)
    ws = eng._ws(eng.lib.grf_scan_workspace_bytes(n_sel))
    C.check(eng.lib.grf_scan_counts(n_sel, _p(cnt), _p(ptr), _p(ws), ws.numel(), eng.stream), "grf_scan_counts")
    nnz = int(ptr[-1].item()) if n_sel else 0
    idx = eng._empty(nnz, torch.int32)
    val = eng._empty(nnz, torch.float32)
    C.check(eng.lib.grf_csr_gather_rows(n_sel, _p(A.ptr), _p(A.idx), _p(A.val32), _p(rmap), _p(ptr), _p(idx),
                                        _p(val), eng.stream), "grf_csr_gather_rows")
    return DeviceCSR(n_sel, A.n_cols, ptr, idx, None, val, nnz)


def rowdot(eng: GRFEngine, A: DeviceCSR, rows_a: Optional[torch.Tensor], B: DeviceCSR,
           rows_b: Optional[torch.Tensor], n_pairs: int) -> torch.Tensor:
    """out[r] = A[rows_a[r]] . B[rows_b[r]] (fp64)."""
    ra = None if rows_a is None else rows_a.to(eng.device, torch.int32).contiguous()
    rb = None if rows_b is None else rows_b.to(eng.device, torch.int32).contiguous()
    out = eng._empty(n_pairs, torch.float64)
    C.check(eng.lib.grf_csr_rowdot(n_pairs, _p(A.ptr), _p(A.idx), _p(A.val32), _p(ra), _p(B.ptr), _p(B.idx),
                                   _p(B.val32), _p(rb), _p(out), eng.stream), "grf_csr_rowdot")
    return out


def rows_dot_cols(eng: GRFEngine, M: DeviceCSR, rows: Optional[torch.Tensor], Z: torch.Tensor) -> torch.Tensor:
    """out[r] = sum_e M[rows[r], e] Z[col_e, r] (fp64), Z float32 (n_cols x >= n_sel) row-major."""
    rmap = None if rows is None else rows.to(eng.device, torch.int32).contiguous()
    n_sel = M.n_rows if rmap is None else rmap.numel()
    if Z.dtype != torch.float32 or Z.stride(1) != 1 or Z.shape[0] != M.n_cols:
        raise ValueError("rows_dot_cols: Z must be a float32 (n_cols x S) row-major matrix")
    out = eng._empty(n_sel, torch.float64)
    C.check(eng.lib.grf_csr_rows_dot_cols(n_sel, _p(M.ptr), _p(M.idx), _p(M.val32), _p(rmap), _p(Z), Z.stride(0),
                                          _p(out), eng.stream), "grf_csr_rows_dot_cols")
    return out


def kernel_block(eng: GRFEngine, phi: DeviceCSR, x1: Optional[torch.Tensor], x2: Optional[torch.Tensor],
                 same: bool) -> torch.Tensor:
    """K[x1, x2] = Phi[x1] Phi[x2]^T (float32, |x1| x |x2|) on the sparse Gram kernels: the
    column-block Gram of Phi[x1]'s rows against the banded transpose of Phi[x2] (exact fixed-point
    sums; with x1 == x2 the symmetric enumeration + mirror, so K comes out exactly symmetric)."""
    P1 = phi if x1 is None else gather_rows(eng, phi, x1)
    P2 = P1 if same else (phi if x2 is None else gather_rows(eng, phi, x2))
    n1, n2 = P1.n_rows, P2.n_rows
    if n1 == 0 or n2 == 0:
        return torch.zeros((n1, n2), dtype=torch.float32, device=eng.device)
    tr = eng.transpose_banded(P2, cols_band_width(n2))
    return eng.gram_sparse_cols(P1, eng.phi_row_shifts(P1), tr, 0, n1, sym_row0=0 if same else None)


def _index(x: Optional[torch.Tensor], dev) -> Optional[torch.Tensor]:
    return None if x is None else x.long().flatten().to(dev)


class GRFKernelFunction(torch.autograd.Function):
    """K[x1, x2] (or its diagonal) = Phi(f)[x1] Phi(f)[x2]^T, differentiable w.r.t. the modulator f."""

    @staticmethod
    def forward(ctx, f: torch.Tensor, steps: StepMatrices, x1, x2, diag: bool):
        eng = steps.engine
        dev = eng.device
        n = steps.shape[0]
        i1, i2 = _index(x1, dev), _index(x2, dev)
        same = (i1 is None and i2 is None) or (i1 is not None and i2 is not None and i1.shape == i2.shape
                                               and bool(torch.equal(i1, i2)))
        phi = steps.phi(f)
        if diag:
            n1 = n if i1 is None else i1.numel()
            n2 = n if i2 is None else i2.numel()
            if n1 != n2:
                raise ValueError("diag=True needs x1 and x2 of the same length")
            out = rowdot(eng, phi, i1, phi, i2, n1).to(f.dtype)
        else:
            out = kernel_block(eng, phi, i1, i2, same)
            out = out.to(f.dtype) if out.dtype != f.dtype else out
        ctx.steps, ctx.phi, ctx.i1, ctx.i2, ctx.diag, ctx.n_f = steps, phi, i1, i2, diag, f.numel()
        ctx.f_dtype = f.dtype
        return out

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        steps, phi, i1, i2 = ctx.steps, ctx.phi, ctx.i1, ctx.i2
        eng = steps.engine
        L = min(steps.L, ctx.n_f)
        grad = torch.zeros(ctx.n_f, dtype=torch.float64, device=eng.device)
        n = steps.shape[0]
        if ctx.diag:
            gd = g.to(eng.device, torch.float64)
            m = gd.numel()
            for l in range(L):
                M = steps.steps[l]
                d = rowdot(eng, M, i1, phi, i2, m) + rowdot(eng, phi, i1, M, i2, m)
                grad[l] = (gd * d).sum()
        else:
            G = g.to(eng.device, torch.float32).contiguous()
            n1 = n if i1 is None else i1.numel()
            n2 = n if i2 is None else i2.numel()
            if n1 and n2:
                Z1 = eng.spmm(eng.csr_transpose(phi, i2), G.t().contiguous())  # N x n1: Phi[x2]^T G^T
                Z2 = eng.spmm(eng.csr_transpose(phi, i1), G)                   # N x n2: Phi[x1]^T G
                for l in range(L):
                    M = steps.steps[l]
                    grad[l] = rows_dot_cols(eng, M, i1, Z1).sum() + rows_dot_cols(eng, M, i2, Z2).sum()
        return grad.to(ctx.f_dtype), None, None, None, None


def grf_kernel(f: torch.Tensor, steps: StepMatrices, x1=None, x2=None, diag: bool = False) -> torch.Tensor:
    """K[x1, x2] = Phi[x1] Phi[x2]^T with Phi = sum_l f_l M_l (differentiable in f)."""
    return GRFKernelFunction.apply(f, steps, x1, x2, diag)


def feature_matrix(f: torch.Tensor, steps: StepMatrices) -> torch.Tensor:
    """Phi as a torch sparse CSR tensor (float32 values, int64 indices) on the device (not differentiable)."""
    phi = steps.phi(f)
    return torch.sparse_csr_tensor(phi.ptr, phi.idx[:phi.nnz].long(), phi.val32[:phi.nnz], steps.shape,
                                   dtype=torch.float32)


# ----------------------------------------------------------------- dense step tensors (GPflow surface)
class DenseSteps:
    """A dense (N, N, L) step tensor F resident on the device once (the GPflow wrappers'
    ``feature_matrices_tf``, gpflow_kernels/general_kernel_fast_grf.py:44-59), with K = (F f)(F f)^T
    on the MFMA Gram (grf_gram_dense) cached per modulator value."""

    def __init__(self, F, engine: Optional[GRFEngine] = None):
        self.engine = engine or get_engine()
        Ft = F if torch.is_tensor(F) else torch.from_numpy(np.ascontiguousarray(F, dtype=np.float64))
        self.F = Ft.to(self.engine.device, torch.float64).contiguous()
        if self.F.dim() != 3 or self.F.shape[0] != self.F.shape[1]:
            raise ValueError("step tensor must be (N, N, L)")
        self.n, self.L = self.F.shape[0], self.F.shape[2]
        self._key = None
        self._K = None

    def phi(self, f: torch.Tensor) -> torch.Tensor:
        """Phi = F f (N x N, fp64 on the device): ``tf.linalg.matmul(F, f[:, None])`` (:76)."""
        return self.F @ f.detach().to(self.engine.device, torch.float64).reshape(-1)

    def gram(self, f: torch.Tensor) -> torch.Tensor:
        """K = Phi Phi^T (fp32, N x N) on the MFMA Gram, cached for the last modulator value."""
        key = f.detach().to("cpu", torch.float64).reshape(-1).numpy().tobytes()
        if key != self._key:
            n = self.n
            lda = max(16, -(-n // 16) * 16)
            A = torch.zeros((n, lda), dtype=torch.float32, device=self.engine.device)
            A[:, :n] = self.phi(f).to(torch.float32)
            self._K = self.engine.gram_dense(A, n)
            self._key = key
        return self._K


class DenseGramFunction(torch.autograd.Function):
    """K = (F f)(F f)^T with dK/df_l = F_l Phi^T + Phi F_l^T: the backward contracts the upstream
    G with it, dL/df_l = <F_l, (G + G^T) Phi> (one plain N x N GEMM + a reduction over F)."""

    @staticmethod
    def forward(ctx, f: torch.Tensor, steps: DenseSteps):
        ctx.steps = steps
        ctx.save_for_backward(f)
        return steps.gram(f).to(f.dtype)

    @staticmethod
    def backward(ctx, g: torch.Tensor):
        (f,) = ctx.saved_tensors
        steps = ctx.steps
        phi = steps.phi(f)
        G = g.to(steps.engine.device, torch.float64)
        H = (G + G.t()) @ phi
        grad = torch.einsum("ijl,ij->l", steps.F, H)
        return grad.to(f.dtype), None
