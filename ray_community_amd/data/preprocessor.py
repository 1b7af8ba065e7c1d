"""``ray.data.preprocessor`` (reference module path of the Preprocessor base class)."""
from .preprocessors import Preprocessor

__all__ = ["Preprocessor"]
