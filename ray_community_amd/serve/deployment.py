"""``ray.serve.deployment`` import path."""
from .api import Application, Deployment

__all__ = ["Deployment", "Application"]
