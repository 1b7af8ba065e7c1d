"""Object serialization (reference: ``python/ray/_private/serialization.py``).

Wire format (one contiguous region — either inline bytes or one shm-store object):

    | "RCA1" | flags u32 | nbuf u32 | inband_len u64 | buf_len u64 * nbuf | pad64 | inband | pad64 | buf0 | pad64 | buf1 ...

* cloudpickle protocol 5 with out-of-band buffers: numpy arrays / CPU torch tensors are written
  raw (64-B aligned) and deserialised as zero-copy views of the shm object.
* ObjectRefs inside a value are recorded (``SerializationContext.contained``) so the head keeps
  them alive while the container lives (borrowing).
* CUDA tensors are NOT copied through the host: they become persistent-id slots of the pickle,
  the owning process keeps them in its GPU object store (``_private/gpu_store.py``) and the wire
  bytes carry a table of HIP IPC export records as the last out-of-band buffer (``FLAG_GPU``);
  readers map the owner's HBM (same GPU: zero-copy; another GPU of the node: peer mapping over
  xGMI).
"""
from __future__ import annotations

import io
import itertools
import os
import pickle
import struct
import sys
import threading
import weakref
from typing import Any, List, Optional, Tuple

import cloudpickle

MAGIC = b"RCA1"
FLAG_ERROR = 1
FLAG_GPU = 2
ALIGN = 64
_HDR = struct.Struct("<4sIIQ")

_tls = threading.local()


def _pad(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class SerializationContext:
    def __init__(self):
        self.contained: List[bytes] = []
        self.gpu_tensors: List[Any] = []


def current_context() -> Optional[SerializationContext]:
    return getattr(_tls, "ctx", None)


# ------------------------------------------------------------------ custom serializers
_CUSTOM = {}


def register_serializer(cls, *, serializer, deserializer):
    _CUSTOM[cls] = (serializer, deserializer)


def deregister_serializer(cls):
    _CUSTOM.pop(cls, None)


def _rebuild_custom(deserializer, state):
    return deserializer(state)


def _rebuild_np_torch(arr, dtype_name, shape):
    import warnings

    import torch

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        t = torch.from_numpy(arr)
    if dtype_name == "bfloat16":
        t = t.view(torch.bfloat16)
    elif dtype_name == "float8_e4m3fn":
        t = t.view(torch.float8_e4m3fn)
    elif dtype_name == "float8_e5m2":
        t = t.view(torch.float8_e5m2)
    return t.reshape(shape)


def _reduce_cpu_tensor(t):
    import torch

    if t.layout != torch.strided or t.requires_grad or t.is_quantized or t.is_sparse:
        return None
    c = t.detach().contiguous()
    name = str(c.dtype).replace("torch.", "")
    if c.dtype in (torch.bfloat16, torch.float16) or name.startswith("float8"):
        view_dt = {1: torch.uint8, 2: torch.int16}[c.element_size()]
        arr = c.view(view_dt).numpy()
    else:
        try:
            arr = c.numpy()
        except Exception:
            return None
    return (_rebuild_np_torch, (arr, name, tuple(t.shape)))


_TENSOR_TYPES: frozenset = frozenset()


def _tensor_types() -> frozenset:
    global _TENSOR_TYPES
    if not _TENSOR_TYPES and "torch" in sys.modules:
        import torch

        _TENSOR_TYPES = frozenset({torch.Tensor, torch.nn.Parameter})
    return _TENSOR_TYPES


class _Pickler(cloudpickle.CloudPickler):
    def persistent_id(self, obj):
        # CUDA tensors become slots resolved against the object's GPU export table (called for
        # every pickled object: one set lookup on the hot path)
        if type(obj) in _tensor_types():
            if obj.is_cuda:
                ctx = current_context()
                if ctx is None:
                    raise TypeError("CUDA tensors can only be serialized into objects")
                ctx.gpu_tensors.append(obj)
                return ("rca_gpu", len(ctx.gpu_tensors) - 1)
        return None

    def reducer_override(self, obj):
        t = type(obj)
        if t in _CUSTOM:
            ser, des = _CUSTOM[t]
            return (_rebuild_custom, (des, ser(obj)))
        if t in _tensor_types() and not obj.is_cuda:
            r = _reduce_cpu_tensor(obj)
            if r is not None:
                return r
        return super().reducer_override(obj)


def _dumps(value, buffers: list) -> bytes:
    f = io.BytesIO()
    p = _Pickler(f, protocol=5, buffer_callback=buffers.append)
    p.dump(value)
    return f.getvalue()


_BULK = 8 << 20  # buffers this large are copied by the native multi-threaded memcpy
# drivers copy with up to half the cores; worker processes (many of them put at once) copy alone
_COPY_THREADS = int(os.environ.get("RCA_MEMCOPY_THREADS", 1 if os.environ.get("RCA_WORKER_ID") else
                                   max(1, min(8, (os.cpu_count() or 2) // 2))))
_COPY_FN = []


def _bulk_copy():
    if not _COPY_FN:
        try:
            from .._native import load

            _COPY_FN.append(getattr(load(), "copy_into", None))
        except Exception:  # native core unavailable: plain slice assignment
            _COPY_FN.append(None)
    return _COPY_FN[0]


class Serialized:
    """A serialised value: inband pickle + raw out-of-band buffers, ready to be written."""

    __slots__ = ("inband", "buffers", "flags", "contained", "gpu_tensors", "total_size", "_lens")

    def __init__(self, inband: bytes, buffers: list, flags: int, contained, gpu_tensors):
        self.inband = inband
        self.buffers = [b.raw() if isinstance(b, pickle.PickleBuffer) else memoryview(b) for b in buffers]
        self.flags = flags
        self.contained = contained
        self.gpu_tensors = gpu_tensors
        self._lens = [mv.nbytes for mv in self.buffers]
        size = _pad(_HDR.size + 8 * len(self.buffers)) + _pad(len(self.inband))
        for n in self._lens:
            size += _pad(n)
        self.total_size = size

    def write_into(self, mv: memoryview):
        """Write the wire format into a writable buffer of ``total_size`` bytes."""
        mv = mv.cast("B") if mv.format != "B" else mv
        hdr = _HDR.pack(MAGIC, self.flags, len(self.buffers), len(self.inband))
        off = 0
        mv[off:off + len(hdr)] = hdr
        off += len(hdr)
        for n in self._lens:
            mv[off:off + 8] = struct.pack("<Q", n)
            off += 8
        off = _pad(off)
        mv[off:off + len(self.inband)] = self.inband
        off = _pad(off + len(self.inband))
        for b, n in zip(self.buffers, self._lens):
            if n:
                src = b.cast("B") if b.format != "B" or b.ndim != 1 else b
                if n >= _BULK and _bulk_copy() is not None:
                    _bulk_copy()(mv[off:off + n], src, _COPY_THREADS)
                else:
                    mv[off:off + n] = src
            off = _pad(off + n)

    def to_bytes(self) -> bytes:
        buf = bytearray(self.total_size)
        self.write_into(memoryview(buf))
        return bytes(buf)

    def to_bytes_with_table(self, table: bytes) -> bytes:
        """Wire bytes of a GPU object: the host parts plus the IPC export table as the last
        out-of-band buffer (``FLAG_GPU``)."""
        t = Serialized(self.inband, [], self.flags | FLAG_GPU, self.contained, [])
        t.buffers = list(self.buffers) + [memoryview(table)]
        t._lens = list(self._lens) + [len(table)]
        size = _pad(_HDR.size + 8 * len(t.buffers)) + _pad(len(t.inband))
        for n in t._lens:
            size += _pad(n)
        t.total_size = size
        return t.to_bytes()


_ESCAPE_HOOK = [None]


def set_escape_hook(fn):
    """``fn(oids)`` runs whenever a serialized value contains ObjectRefs (the refs may leave this
    process with it): the core worker waits there for the head to have registered its own
    not-yet-acknowledged puts among them (``CoreWorker.sync_puts``)."""
    _ESCAPE_HOOK[0] = fn


def serialize(value: Any, error: bool = False) -> Serialized:
    ctx = SerializationContext()
    prev = getattr(_tls, "ctx", None)
    _tls.ctx = ctx
    buffers: list = []
    try:
        inband = _dumps(value, buffers)
    finally:
        _tls.ctx = prev
    if ctx.contained and _ESCAPE_HOOK[0] is not None:
        _ESCAPE_HOOK[0](ctx.contained)
    flags = (FLAG_ERROR if error else 0) | (FLAG_GPU if ctx.gpu_tensors else 0)
    return Serialized(inband, buffers, flags, ctx.contained, ctx.gpu_tensors)


def parse(mv) -> Tuple[int, bytes, list]:
    """Return (flags, inband memoryview, [buffer memoryviews]) — all views alias ``mv``."""
    mv = memoryview(mv)
    if mv.format != "B":
        mv = mv.cast("B")
    magic, flags, nbuf, inlen = _HDR.unpack_from(mv, 0)
    if magic != MAGIC:
        raise ValueError("corrupt object (bad magic)")
    off = _HDR.size
    lens = struct.unpack_from(f"<{nbuf}Q", mv, off) if nbuf else ()
    off = _pad(off + 8 * nbuf)
    inband = mv[off:off + inlen]
    off = _pad(off + inlen)
    bufs = []
    for n in lens:
        bufs.append(mv[off:off + n])
        off = _pad(off + n)
    return flags, inband, bufs


def deserialize(mv) -> Tuple[Any, int]:
    flags, inband, bufs = parse(mv)
    if flags & FLAG_GPU:
        from .gpu_store import decode_table, import_tensor

        tensors = [import_tensor(r) for r in decode_table(bufs[-1])]
        up = pickle.Unpickler(io.BytesIO(inband), buffers=bufs[:-1])
        up.persistent_load = lambda pid: tensors[pid[1]]
        return up.load(), flags
    value = pickle.loads(inband, buffers=bufs)
    return value, flags


def dumps_function(fn) -> bytes:
    return cloudpickle.dumps(fn, protocol=5)


def loads_function(b: bytes):
    return pickle.loads(b)
