"""SparseGraphGP (reference models/sparse_grf_model.py:10-45): needs gpytorch and linear_operator."""
import gpytorch  # noqa: F401  (ImportError when absent)

raise ImportError("SparseGraphGP is outside this engine's scope (downstream GP model); see DESIGN.md")
