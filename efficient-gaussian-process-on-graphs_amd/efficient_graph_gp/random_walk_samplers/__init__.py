from .sampler import Graph, RandomWalk

__all__ = ["RandomWalk", "Graph"]
