"""Python face of the native shared-memory object store (``_native/shm_store.cpp``)."""
from __future__ import annotations

import os

from .. import _native
from .serialization import Serialized

_mod = None


def native():
    global _mod
    if _mod is None:
        _mod = _native.load()
    return _mod


class ObjectStore:
    def __init__(self, name: str, capacity: int = 0, create: bool = False, table_cap: int = 1 << 18):
        self.name = name
        self._s = native().ShmStore(name, capacity, create, table_cap)
        self.created = create

    # -------------------------------------------------------------- writes
    def put_serialized(self, oid: bytes, ser: Serialized) -> bool:
        """Create+write+seal. False if the store is full (caller spills or falls back)."""
        off = self._s.create(oid, ser.total_size)
        if off == -2:
            return True  # already present (idempotent retries)
        if off < 0:
            return False
        try:
            mv = self._s.view(off, ser.total_size, False)
            ser.write_into(mv)
            mv.release()
        except BaseException:
            self._s.abort(oid)
            raise
        self._s.seal(oid)
        return True

    def put_bytes(self, oid: bytes, data) -> bool:
        n = len(data)
        off = self._s.create(oid, n)
        if off == -2:
            return True
        if off < 0:
            return False
        self._s.write(off, data)
        self._s.seal(oid)
        return True

    # -------------------------------------------------------------- reads
    def pin(self, oid: bytes):
        """A pinned buffer-protocol view of the object, or None. The pin is released when the
        view (and every memoryview/array aliasing it) is garbage collected."""
        return native().pin_view(self._s, oid, True)

    def contains(self, oid: bytes) -> bool:
        return self._s.contains(oid)

    def read_bytes(self, oid: bytes):
        v = self.pin(oid)
        if v is None:
            return None
        return bytes(memoryview(v))

    # -------------------------------------------------------------- lifetime
    def delete(self, oid: bytes):
        self._s.remove(oid)

    def lru_candidates(self, n: int = 64):
        return self._s.lru_candidates(n)

    def stats(self):
        return self._s.stats()

    def unlink(self):
        try:
            self._s.unlink()
        except Exception:
            pass


def default_store_capacity() -> int:
    """30% of system memory by default (the reference's default), capped at /dev/shm free space."""
    try:
        import psutil

        mem = psutil.virtual_memory().total
    except Exception:
        mem = 8 << 30
    cap = int(mem * 0.3)
    try:
        st = os.statvfs("/dev/shm")
        cap = min(cap, int(st.f_bavail * st.f_frsize * 0.9))
    except Exception:
        pass
    return max(cap, 64 << 20)
