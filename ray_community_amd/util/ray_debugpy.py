"""Post-mortem / breakpoint debugging over debugpy (reference ``python/ray/util/debugpy.py``):
``set_trace()`` waits for a DAP client (VS Code) when ``debugpy`` is importable; without it the
framework's socket pdb (``util/pdb.py``) serves the breakpoint instead."""
from __future__ import annotations

import os


def _debugpy():
    try:
        import debugpy  # noqa: F401

        return debugpy
    except ImportError:
        return None


def set_trace(breakpoint_uuid=None):
    dbg = _debugpy()
    if dbg is None:
        from .pdb import set_trace as _pdb_trace

        return _pdb_trace()
    port = int(os.environ.get("RCA_DEBUGPY_PORT", "0") or 0)
    host, port = dbg.listen(("127.0.0.1", port))
    print(f"debugpy waiting on {host}:{port}", flush=True)
    dbg.wait_for_client()
    dbg.breakpoint()


def post_mortem():
    dbg = _debugpy()
    if dbg is None:
        from .pdb import post_mortem as _pm

        return _pm()
    set_trace()
