"""``ray.util.debugpy`` import path: see ``util/ray_debugpy.py``."""
from .ray_debugpy import *  # noqa: F401,F403
