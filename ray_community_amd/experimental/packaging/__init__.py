"""Runtime packages (reference: ``python/ray/experimental/packaging``)."""
from .load_package import load_package  # noqa: F401

__all__ = ["load_package"]
