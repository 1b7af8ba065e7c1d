"""Garbage-collector settings for the control-plane processes (head and workers)."""
from __future__ import annotations

import gc
import os
from typing import Optional


def tune_gc(config: Optional[dict] = None, freeze: bool = True) -> Optional[tuple]:
    """Raise the young-generation GC threshold of a control-plane process (head / workers).

    Every task allocates a few dozen short-lived containers (specs, messages, futures); with the
    default threshold (700) CPython runs a generation-0 pass every few tasks, and the occasional
    older-generation pass walks every live task/object record of the session. 50k (override:
    ``_system_config={"gc_threshold": n}`` or ``RCA_GC_THRESHOLD``) measured 1.2-2.1x on the core
    microbenchmark rows (bench_core.py); ``gc_threshold=0`` disables the tuning.

    ``freeze`` additionally moves startup objects to the permanent generation -- only for
    processes the framework owns (standalone head, workers). A head living inside the user's
    driver passes ``freeze=False`` (frozen unreachable cycles of user objects, e.g. torch modules
    holding GPU tensors, would never be reclaimed) and restores the returned previous threshold
    with ``restore_gc`` at shutdown. Returns the previous threshold, or None if nothing changed.
    """
    v = (config or {}).get("gc_threshold")
    if v is None:
        v = os.environ.get("RCA_GC_THRESHOLD", 50000)
    n = int(v)
    if n <= 0:
        return None
    prev = gc.get_threshold()
    _, g1, g2 = prev
    gc.set_threshold(max(n, 700), max(g1, 20), max(g2, 100))
    if freeze:
        gc.collect()
        gc.freeze()
    return prev


def restore_gc(prev: Optional[tuple]) -> None:
    if prev is not None:
        gc.set_threshold(*prev)
