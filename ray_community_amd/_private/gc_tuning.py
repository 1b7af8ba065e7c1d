"""Garbage-collector settings for the control-plane processes (head and workers)."""
from __future__ import annotations

import gc
import os
from typing import Optional


def tune_gc(config: Optional[dict] = None) -> None:
    """Raise the young-generation GC threshold of a control-plane process (head / workers).

    Every task allocates a few dozen short-lived containers (specs, messages, futures); with the
    default threshold (700) CPython runs a generation-0 pass every few tasks, and the occasional
    older-generation pass walks every live task/object record of the session. 50k (override:
    ``_system_config={"gc_threshold": n}`` or ``RCA_GC_THRESHOLD``) measured 1.2-2.1x on the core
    microbenchmark rows (bench_core.py). Startup objects are frozen out of later passes.
    """
    n = int((config or {}).get("gc_threshold") or os.environ.get("RCA_GC_THRESHOLD", 50000))
    if n > 0:
        _, g1, g2 = gc.get_threshold()
        gc.set_threshold(max(n, 700), max(g1, 20), max(g2, 100))
        gc.freeze()
