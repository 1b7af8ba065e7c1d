"""Serve exceptions (reference: ``python/ray/serve/exceptions.py``)."""
from __future__ import annotations


class RayServeException(Exception):
    pass


class BackPressureError(RayServeException):
    """A request was rejected because the caller already holds ``max_queued_requests`` requests
    that no replica has accepted yet (HTTP 503, gRPC UNAVAILABLE)."""

    def __init__(self, *, num_queued_requests: int, max_queued_requests: int):
        self.num_queued_requests = num_queued_requests
        self.max_queued_requests = max_queued_requests
        self._message = (f"Request dropped due to backpressure (num_queued_requests={num_queued_requests}, "
                         f"max_queued_requests={max_queued_requests}).")
        super().__init__(self._message)

    @property
    def message(self) -> str:
        return self._message

    def __reduce__(self):
        return (_rebuild_backpressure, (self.num_queued_requests, self.max_queued_requests))


def _rebuild_backpressure(n, m):
    return BackPressureError(num_queued_requests=n, max_queued_requests=m)
