from .sparse_sampler import SparseRandomWalk

__all__ = ["SparseRandomWalk"]
