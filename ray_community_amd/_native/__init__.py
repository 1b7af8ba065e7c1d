"""Native runtime core loader (builds in-tree on first import if needed)."""
import importlib
import os

from . import build as _build


def load():
    if _build.is_stale() and os.environ.get("RCA_NO_REBUILD") != "1":
        _build.build()
    return importlib.import_module("ray_community_amd._native._rca_native")
