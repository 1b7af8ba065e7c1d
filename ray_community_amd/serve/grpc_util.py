"""``RayServegRPCContext`` (reference: ``python/ray/serve/grpc_util.py``): the gRPC servicer
context of a request, as a picklable object that travels with the request to the replica.

A deployment method that declares a ``grpc_context`` parameter receives it; what the method sets
on it (status code, details, trailing metadata, compression) is carried back with the result and
applied to the real ``grpc.ServicerContext`` by the gRPC proxy, so a deployment can answer e.g.
``NOT_FOUND`` with details, or attach trailing metadata, without raising.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple


class RayServegRPCContext:
    def __init__(self, grpc_context=None):
        self._auth_context: Dict[str, Any] = {}
        self._invocation_metadata: List[Tuple[str, str]] = []
        self._peer = ""
        self._peer_identities = None
        self._peer_identity_key = None
        if grpc_context is not None:
            try:
                self._auth_context = dict(grpc_context.auth_context() or {})
            except Exception:  # noqa - not every context type implements every accessor
                pass
            self._invocation_metadata = [(k, v) for k, v in (grpc_context.invocation_metadata() or ())]
            for attr, name in (("_peer", "peer"), ("_peer_identities", "peer_identities"),
                               ("_peer_identity_key", "peer_identity_key")):
                try:
                    setattr(self, attr, getattr(grpc_context, name)())
                except Exception:  # noqa
                    pass
        self._code = None  # grpc.StatusCode set by the deployment (None: OK)
        self._details = ""
        self._trailing_metadata: List[Tuple[str, str]] = []
        self._compression = None
        self._touched = False

    # ------------------------------------------------------------------ read
    def auth_context(self) -> Dict[str, Any]:
        return self._auth_context

    def invocation_metadata(self) -> List[Tuple[str, str]]:
        return list(self._invocation_metadata)

    def peer(self) -> str:
        return self._peer

    def peer_identities(self) -> Optional[Sequence[bytes]]:
        return self._peer_identities

    def peer_identity_key(self) -> Optional[str]:
        return self._peer_identity_key

    def code(self):
        return self._code

    def details(self) -> str:
        return self._details

    def trailing_metadata(self) -> List[Tuple[str, str]]:
        return list(self._trailing_metadata)

    # ------------------------------------------------------------------ write (carried back)
    def set_code(self, code) -> None:
        self._code, self._touched = code, True

    def set_details(self, details: str) -> None:
        self._details, self._touched = str(details), True

    def set_trailing_metadata(self, trailing_metadata: Sequence[Tuple[str, str]]) -> None:
        self._trailing_metadata, self._touched = [(k, v) for k, v in trailing_metadata], True

    def set_compression(self, compression) -> None:
        self._compression, self._touched = compression, True

    def _apply(self, grpc_context) -> None:
        """Copy what the deployment set onto the proxy's real servicer context."""
        if not self._touched:
            return
        if self._trailing_metadata:
            grpc_context.set_trailing_metadata(tuple(self._trailing_metadata))
        if self._compression is not None:
            grpc_context.set_compression(self._compression)
        if self._code is not None:
            grpc_context.set_code(self._code)
        if self._details:
            grpc_context.set_details(self._details)


class _GrpcReply:
    """A gRPC request's result together with the context the deployment may have modified."""

    __slots__ = ("value", "context")

    def __init__(self, value, context):
        self.value, self.context = value, context


def _wants_context(fn) -> bool:
    import inspect

    try:
        params = inspect.signature(fn).parameters
    except (TypeError, ValueError):
        return False
    return "grpc_context" in params
