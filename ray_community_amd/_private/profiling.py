"""Custom profiling events for the timeline (reference: ``python/ray/_private/profiling.py``
``profile(event_type, extra_data)``): a span recorded whether or not tracing is enabled, shown by
``ray.timeline()`` on the process's row next to the task events."""
from __future__ import annotations

import contextlib
from typing import Dict, Optional


@contextlib.contextmanager
def profile(event_type: str, extra_data: Optional[Dict] = None):
    from ..util.tracing import start_span

    with start_span(event_type, attributes=extra_data, kind="profile") as span:
        yield span


def chrome_tracing_dump(events, filename: Optional[str] = None):
    import json

    if filename:
        with open(filename, "w") as f:
            json.dump(events, f)
        return None
    return events
