"""Binary IDs (reference: ``src/ray/common/id.h``, ``python/ray/includes/unique_ids.pxi``).

IDs are 16 random-prefix bytes + an 8-byte counter rendered as fixed-size ``bytes``; the hex
form is used for display. A process-local counter makes generation ~100 ns (no urandom per id).
"""
from __future__ import annotations

import itertools
import os
import struct
import threading

_PREFIX = os.urandom(12)
_COUNTER = itertools.count(1)
_LOCK = threading.Lock()
ID_LEN = 20


def _reseed_after_fork():
    global _PREFIX, _COUNTER
    _PREFIX = os.urandom(12)
    _COUNTER = itertools.count(1)


if hasattr(os, "register_at_fork"):
    os.register_at_fork(after_in_child=_reseed_after_fork)


def new_id() -> bytes:
    return _PREFIX + struct.pack("<Q", next(_COUNTER))


def return_ids(tid: bytes, n: int) -> list:
    """Object ids of a task's ``n`` returns: the task id's first 16 bytes + a 1-based index
    (reference: ``ObjectID::FromIndex``). ``new_id`` values keep bytes 16..20 zero (< 2**32 ids
    per process), so these never collide with a put id or another task's returns."""
    head = tid[:16]
    return [head + struct.pack("<I", i + 1) for i in range(n)]


def task_id_of(oid: bytes):
    """The id of the task that returns ``oid`` (None for ``put`` objects)."""
    if len(oid) == ID_LEN and oid[16:] != b"\0\0\0\0":
        return oid[:16] + b"\0\0\0\0"
    return None


class BaseID:
    __slots__ = ("_b",)
    size = ID_LEN

    def __init__(self, b: bytes):
        if isinstance(b, str):
            b = bytes.fromhex(b)
        self._b = bytes(b)

    @classmethod
    def from_random(cls):
        return cls(new_id())

    @classmethod
    def from_hex(cls, h: str):
        return cls(bytes.fromhex(h))

    @classmethod
    def nil(cls):
        return cls(b"\xff" * ID_LEN)

    def is_nil(self):
        return self._b == b"\xff" * ID_LEN

    def binary(self) -> bytes:
        return self._b

    def hex(self) -> str:
        return self._b.hex()

    def __hash__(self):
        return hash(self._b)

    def __eq__(self, other):
        return type(other) is type(self) and other._b == self._b

    def __lt__(self, other):
        return self._b < other._b

    def __repr__(self):
        return f"{type(self).__name__}({self.hex()})"

    def __reduce__(self):
        return (type(self), (self._b,))


class JobID(BaseID):
    __slots__ = ()


class TaskID(BaseID):
    __slots__ = ()


class ActorID(BaseID):
    __slots__ = ()


class ActorClassID(BaseID):
    __slots__ = ()


class NodeID(BaseID):
    __slots__ = ()


class WorkerID(BaseID):
    __slots__ = ()


class FunctionID(BaseID):
    __slots__ = ()


class PlacementGroupID(BaseID):
    __slots__ = ()


class UniqueID(BaseID):
    __slots__ = ()


class ObjectID(BaseID):
    __slots__ = ()
