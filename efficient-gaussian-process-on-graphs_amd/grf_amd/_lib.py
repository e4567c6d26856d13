"""ctypes binding of ``libgrf_amd.so`` (the C ABI declared in ``include/grf.h``).

The shared library is built in-tree by ``csrc/Makefile`` (hipcc, gfx950).  If
it is missing this module raises -- there is no CPU fallback anywhere in the
product path.  ``torch`` is imported first so that the HIP runtime torch ships
(SONAME ``libamdhip64.so.7``) is the one the library binds to: device
pointers and streams are then shared between torch and the engine.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch  # noqa: F401  (load torch's HIP runtime before ours)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_PKG, "libgrf_amd.so")
if os.environ.get("GRF_AMD_LIB"):  # (same-box A/B of two builds of the library: tools/gpu_*.sh)
    LIB_PATH = os.path.abspath(os.environ["GRF_AMD_LIB"])
CSRC = os.path.join(os.path.dirname(_PKG), "csrc")

GRF_OK, GRF_EINVAL, GRF_EHIP, GRF_ECAPACITY, GRF_EUNSUPPORTED = 0, -1, -2, -3, -4
LAP_SCIPY, LAP_NUMPY, LAP_NUMPY_SAFE, LAP_COMBINATORIAL, LAP_NONE = 0, 1, 2, 3, 4
RNG_PCG64, RNG_PHILOX = 0, 1
LOAD_CUMULATIVE, LOAD_NONCUMULATIVE, LOAD_ABLATION = 0, 1, 2
NORM_DIV, NORM_MUL_RECIP = 0, 1
REC_LINE, REC_PACKED, REC_SLOT = 128, 12, 32
ABI_VERSION = 8  # include/grf.h GRF_ABI_VERSION: argument lists change between revisions


class GrfWalkParams(ctypes.Structure):
    _fields_ = [
        ("walks_per_node", ctypes.c_int64),
        ("p_halt", ctypes.c_double),
        ("max_walk_length", ctypes.c_int32),
        ("load_rule", ctypes.c_int32),
        ("rng", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("n_chunks", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
    ]


_i32, _i64, _u64, _dbl, _vp, _sz = (ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double,
                                    ctypes.c_void_p, ctypes.c_size_t)

# name -> (restype, argtypes); mirrors include/grf.h exactly
SIGNATURES = {
    "grf_last_error": (ctypes.c_char_p, []),
    "grf_version": (_i32, []),
    "grf_device_count": (_i32, []),
    "grf_set_device": (_i32, [_i32]),
    "grf_laplacian_csr": (_i32, [_i64, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _sz, _vp]),
    "grf_laplacian_csr_workspace_bytes": (_sz, [_i64]),
    "grf_laplacian_dense": (_i32, [_i64, _vp, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _sz, _vp]),
    "grf_laplacian_dense_workspace_bytes": (_sz, [_i64]),
    "grf_walk": (_i32, [_i64, _vp, _vp, _vp, ctypes.POINTER(GrfWalkParams), _i64, _i64, _vp, _vp, _vp]),
    "grf_walk_ex": (_i32, [_i64, _vp, _vp, _vp, _vp, ctypes.POINTER(GrfWalkParams), _i64, _i64, _vp, _vp, _vp]),
    "grf_chunk_bounds": (_i64, [_i64, _i64, _i64]),
    "grf_steps": (_i32, [_i64, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "grf_steps_densify": (_i32, [_i64, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "grf_phi": (_i32, [_i64, _i64, _i32, _vp, _vp, _vp, _vp, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "grf_walk_aug": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp]),
    "grf_walk_aug_bytes": (_sz, [_i64]),
    "grf_walk_phi": (_i32, [_i64, _vp, _vp, _vp, _vp, ctypes.POINTER(GrfWalkParams), _i64, _i64, _i32, _vp, _i32, _i64,
                             _vp, _vp, _vp, _vp, _vp, _i64, _i64, _vp]),
    "grf_phi_fused": (_i32, [_i64, _i64, _i32, _i32, _vp, _vp, _vp, _i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "grf_scan_counts": (_i32, [_i64, _vp, _vp, _vp, _sz, _vp]),
    "grf_scan_workspace_bytes": (_sz, [_i64]),
    "grf_concat_segments": (_i32, [_i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "grf_compact_rows": (_i32, [_i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "grf_compact_rows_stats": (_i32, [_i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "grf_transpose_banded_plan": (_i32, [_i64, _i64, _i64, _i32, _vp, _vp, _vp, _i32, _vp, _sz, _vp]),
    "grf_transpose_banded_fill": (_i32, [_i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _sz,
                                         _vp]),
    "grf_transpose_workspace_bytes": (_sz, [_i64]),
    "grf_gram_sparse": (_i32, [_i64, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _i64, _vp, _sz, _vp]),
    "grf_gram_workspace_bytes": (_sz, []),
    "grf_gram_sparse_cols": (_i32, [_i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp,
                                    _i64, _vp, _sz, _vp]),
    "grf_phi_row_shifts_workspace_bytes": (_sz, [_i64]),
    "grf_phi_row_shifts": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "grf_phi_row_shifts_stats": (_i32, [_i64, _vp, _vp, _vp, _vp]),
    "grf_phi_row_shifts_padded": (_i32, [_i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "grf_gram_sparse_cols_padded": (_i32, [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _i64,
                                           _vp]),
    "grf_gram_sparse_sym": (_i32, [_i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _sz, _vp]),
    "grf_gram_mirror": (_i32, [_i64, _vp, _i64, _i64, _vp]),
    "grf_gram_sparse_upper": (_i32, [_i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _i32,
                                     _i32, _vp, _sz, _vp]),
    "grf_gram_row_cuts": (_i32, [_i64, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp]),
    "grf_gram_sparse_upper_ex": (_i32, [_i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i32,
                                        _i32, _i32, _i32, _vp]),
    "grf_gram_sparse_upper_add": (_i32, [_i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _i32,
                                         _i32, _i32, _vp, _sz, _vp]),
    "grf_hub_panel": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    "grf_transpose_drop_columns": (_i32, [_i64, _i64, _vp, _vp, _i32, _vp]),
    "grf_gram_dense_upper": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "grf_transpose_banded_fill_staged": (_i32, [_i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                                _sz, _i64, _vp, _sz, _vp]),
    "grf_transpose_staging_bytes": (_sz, [_i64, _i64, _i64, _i64]),
    "grf_transpose_banded_self": (_i32, [_i64, _i64, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp,
                                         _sz, _i64, _vp, _sz, _vp]),
    "grf_transpose_self_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "grf_transpose_self_units_bound": (_i64, [_i64, _i64, _i64, _i32, _i64]),
    "grf_csr_transpose_workspace_bytes": (_sz, [_i64, _i64, _i64]),
    "grf_csr_transpose": (_i32, [_i64, _vp, _vp, _vp, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _sz, _vp]),
    "grf_spmm_csr": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp]),
    "grf_spmm_csr_f64": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _i64, _i32, _vp, _i64, _vp]),
    "grf_cg_gram_solve_f64": (_i32, [_i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _dbl, _vp, _i64, _i32, _dbl,
                                     _i32, _vp, _i64, _vp, _sz, _vp, _vp, _vp]),
    "grf_cg_workspace_bytes": (_sz, [_i64, _i64, _i32]),
    "grf_cg_gram_solve": (_i32, [_i64, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp, _dbl, _vp, _i64, _i32, _dbl, _i32,
                                 _vp, _i64, _vp, _sz, _vp, _vp, _vp]),
    "grf_gram_sparse_kslice": (_i32, [_i64, _i64, _i64, _i64, _i64, _vp, _vp, _vp, _i64, _i32, _vp, _vp, _vp, _vp,
                                      _i64, _vp, _sz, _vp]),
    "grf_gram_dense": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "grf_gram_dense_workspace_bytes": (_sz, [_i64, _i64]),
    "grf_gram_dense_ws": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp, _sz, _vp]),
    "grf_gram_dense_split_workspace_bytes": (_sz, [_i64, _i64]),
    "grf_gram_dense_split": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp, _sz, _vp]),
    "grf_gram_dense_split_upper": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "grf_densify": (_i32, [_i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "grf_densify_padded": (_i32, [_i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "grf_planes_row_bytes": (_i64, [_i64]),
    "grf_split_planes": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "grf_densify_padded_planes": (_i32, [_i64, _i64, _i64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "grf_gram_dense_planes": (_i32, [_i64, _i64, _vp, _i64, _vp, _i64, _vp, _sz, _vp]),
    # the GPyTorch surface's feature algebra (step_* are host arrays of device pointers)
    "grf_phi_steps_csr_count": (_i32, [_i64, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp]),
    "grf_phi_steps_csr_fill": (_i32, [_i64, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "grf_csr_row_lengths": (_i32, [_i64, _vp, _vp, _vp, _vp]),
    "grf_csr_gather_rows": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "grf_csr_rowdot": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "grf_csr_rows_dot_cols": (_i32, [_i64, _vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "grf_dense_to_csr_count": (_i32, [_i64, _i64, _vp, _i64, _vp, _vp]),
    "grf_dense_to_csr_fill": (_i32, [_i64, _i64, _vp, _i64, _vp, _vp, _vp, _vp]),
    # the GPflow surface's algebra on a dense (N, N, L) step tensor
    "grf_dense_steps_phi": (_i32, [_i64, _i32, _vp, _vp, _vp, _vp, _i64, _vp]),
    "grf_dense_steps_grad_workspace_bytes": (_sz, [_i64, _i32]),
    "grf_dense_steps_grad": (_i32, [_i64, _i32, _vp, _vp, _vp, _i64, _vp, _vp, _sz, _vp]),
}

_lib = None


def build(force: bool = False) -> str:
    """Compile libgrf_amd.so for gfx950 with hipcc (make -C csrc)."""
    cmd = ["make", "-s", "-C", CSRC, f"-j{min(16, os.cpu_count() or 1)}"]
    if force:
        subprocess.run(["make", "-s", "-C", CSRC, "clean"], check=True)
    subprocess.run(cmd, check=True)
    return LIB_PATH


def load():
    """Load the engine library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"grf_amd: native library {LIB_PATH} is missing; build it with "
            f"`make -C {CSRC}` (or __graft_entry__.build()).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    lib.grf_version.restype = ctypes.c_int32
    lib.grf_version.argtypes = []
    got = int(lib.grf_version())
    if got != ABI_VERSION:
        raise ImportError(f"grf_amd: {LIB_PATH} implements ABI revision {got}, this binding needs {ABI_VERSION} "
                          f"(rebuild it with `make -C {CSRC}`)")
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class GrfError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    """Map a grf_status to the reference's exception types (SURVEY.md §8b Errors)."""
    if rc == GRF_OK:
        return
    msg = f"{what}: {load().grf_last_error().decode(errors='replace')}"
    if rc == GRF_EINVAL:
        raise ValueError(msg)
    if rc == GRF_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise GrfError(msg)


def exported_symbols() -> list[str]:
    return sorted(SIGNATURES)
