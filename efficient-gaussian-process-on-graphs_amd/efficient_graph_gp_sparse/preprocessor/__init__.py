from .graph_preprocessor import GraphPreprocessor

__all__ = ["GraphPreprocessor"]
