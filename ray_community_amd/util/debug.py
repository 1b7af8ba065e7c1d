"""Debug helpers (reference: ``python/ray/util/debug.py``)."""
from __future__ import annotations

_logged = set()
_disabled = False


def log_once(key: str) -> bool:
    """True the first time ``key`` is seen in this process."""
    if _disabled or key in _logged:
        return False
    _logged.add(key)
    return True


def disable_log_once_globally():
    global _disabled
    _disabled = True


def enable_periodic_logging():
    _logged.clear()
