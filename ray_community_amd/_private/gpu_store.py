"""GPU object store: objects whose tensors stay in HBM, with an HBM budget and host spill.

Reference: Ray copies GPU tensors to host at ``put`` and has no device-resident store
(``python/ray/_private/serialization.py``); spilling of host objects is
``python/ray/_private/external_storage.py:185-293``. Here GPU tensors never leave the device on
the hot path:

  * ``ray.put`` / task returns of CUDA tensors: the owning process keeps the tensors in its
    ``GpuObjectStore`` (a ``put`` snapshots them with one device-to-device copy -- puts are
    immutable; a task's return value is taken over without a copy);
  * consumers map the owner's allocation with HIP IPC (``hipIpcGetMemHandle`` /
    ``hipIpcOpenMemHandle``: same GPU zero-copy, another GPU of the node peer-mapped over xGMI).
    The mapping is closed when the consumer's tensor dies; the owner frees its copy only when the
    head says the object has no holders left -- one lifetime protocol, no torch CUDA-IPC
    refcount files (so no "producer terminated before shared tensors released" at teardown);
  * the head accounts HBM bytes of GPU objects per physical GPU against
    ``gpu_object_store_memory`` (bytes per GPU, default 30 % of the device). Over budget it asks
    the owners of the least recently used objects to spill: the owner copies the tensors into
    pinned host memory with ``hipMemcpyAsync`` on a side stream and releases the HBM; a later
    ``get`` asks the owner to restore them (pinned H2D copy) and hands out fresh IPC handles;
  * an owner that dies takes its objects with it: readers get ``OwnerDiedError`` (an
    ``ObjectLostError``).

Wire format of a GPU object: the normal serialized value in which every CUDA tensor is a
persistent-id slot, plus (as the last out-of-band buffer) a pickled table of per-slot IPC
export records. Spill/restore only rewrites that table.
"""
from __future__ import annotations

import ctypes
import os
import pickle
import threading
import time
from typing import Dict, List, Optional

_HIP = None
_HIP_LOCK = threading.Lock()


class _IpcHandle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def _hip():
    """The HIP runtime torch itself loaded (one runtime per process)."""
    global _HIP
    if _HIP is None:
        with _HIP_LOCK:
            if _HIP is None:
                import torch

                path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
                L = ctypes.CDLL(path if os.path.exists(path) else "libamdhip64.so")
                L.hipIpcGetMemHandle.argtypes = [ctypes.POINTER(_IpcHandle), ctypes.c_void_p]
                L.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), _IpcHandle, ctypes.c_uint]
                L.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
                L.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                                    ctypes.c_void_p]
                _HIP = L
    return _HIP


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (hipError {rc})")


def physical_gpu(local_index: int) -> str:
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES") or \
        os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        ids = [x.strip() for x in vis.split(",") if x.strip()]
        if 0 <= local_index < len(ids):
            return ids[local_index]
    return str(local_index)


def _local_index(phys: str) -> Optional[int]:
    import torch

    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES") or \
        os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        ids = [x.strip() for x in vis.split(",") if x.strip()]
        return ids.index(phys) if phys in ids else None
    i = int(phys) if phys.isdigit() else None
    return i if i is not None and i < torch.cuda.device_count() else None


# ====================================================================== export / import
def export_tensor(t, oid: bytes = b"", slot: int = 0) -> dict:
    """IPC export record of a (store-owned, contiguous) CUDA tensor."""
    import torch

    L = _hip()
    with torch.cuda.device(t.device):
        base = ctypes.c_void_p()
        size = ctypes.c_size_t()
        _check(L.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(t.data_ptr())),
               "hipMemGetAddressRange")
        h = _IpcHandle()
        _check(L.hipIpcGetMemHandle(ctypes.byref(h), base), "hipIpcGetMemHandle")
    # raw 64 bytes (reading the c_char field would stop at the first NUL byte)
    return {"handle": ctypes.string_at(ctypes.addressof(h), ctypes.sizeof(h)), "offset": t.data_ptr() - base.value, "nbytes": t.numel() * t.element_size(),
            "dtype": str(t.dtype).replace("torch.", ""), "shape": tuple(t.shape), "stride": tuple(t.stride()),
            "gpu": physical_gpu(t.device.index), "pid": os.getpid(), "oid": oid, "slot": slot}


class _Mapped:
    """A peer allocation opened by HIP IPC, exposed through ``__cuda_array_interface__`` so torch
    wraps it zero-copy; closed when the last tensor viewing it dies."""


    def __init__(self, rec, dev_index):
        import torch

        self.dev = dev_index
        self.oid = rec.get("oid")
        h = _IpcHandle()
        ctypes.memmove(ctypes.addressof(h), rec["handle"], ctypes.sizeof(h))
        ptr = ctypes.c_void_p()
        with torch.cuda.device(dev_index):
            _check(_hip().hipIpcOpenMemHandle(ctypes.byref(ptr), h, 1), "hipIpcOpenMemHandle")
        self.base = ptr.value
        # raw bytes; import_tensor reinterprets them as the record's dtype / shape (contiguous)
        self.__cuda_array_interface__ = {"shape": (rec["nbytes"],), "typestr": "|u1",
                                         "data": (self.base + rec["offset"], False), "version": 2, "strides": None}

    def __del__(self):
        try:
            import torch

            with torch.cuda.device(self.dev):
                _hip().hipIpcCloseMemHandle(ctypes.c_void_p(self.base))
        except Exception:
            pass
        try:  # tell the head this reader no longer maps the owner's HBM (spill eligibility)
            from .core_worker import _core

            if _core is not None and self.oid:
                _core.client.call_async("gpu_unmapped", self.oid)
        except Exception:
            pass


def _dense_layout(t) -> bool:
    """Dense layouts the store keeps as they are (a permutation of a contiguous block):
    row-major and channels-last; anything else is snapshotted row-major."""
    import torch

    if t.is_contiguous():
        return True
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return True
    return t.dim() == 5 and t.is_contiguous(memory_format=torch.channels_last_3d)


def import_tensor(rec):
    import torch

    if rec["pid"] == os.getpid():
        t = _local_store().local_tensor(rec)
        if t is not None:
            return t
    dev = _local_index(rec["gpu"])
    if dev is None:
        dev = torch.cuda.current_device()
    torch.cuda.init()
    m = _Mapped(rec, dev)
    raw = torch.as_tensor(m, device=f"cuda:{dev}").view(getattr(torch, rec["dtype"]))
    # dense record: same bytes, the exporter's strides (e.g. channels-last activations keep their
    # memory format, so the consumer's kernels see the layout the producer chose)
    stride = rec.get("stride")
    return raw.as_strided(tuple(rec["shape"]), tuple(stride)) if stride else raw.view(rec["shape"])


# ====================================================================== owner side
class _Entry:
    __slots__ = ("tensors", "host", "host_bufs", "nbytes", "gpus", "tensor_gpus", "last", "state", "serialized")

    def __init__(self, tensors, serialized):
        self.tensors = tensors            # store-owned device tensors (None while spilled)
        self.host = None                  # pinned host copies while spilled
        self.host_bufs = None             # the pool buffers under them (returned on restore)
        self.nbytes = sum(t.numel() * t.element_size() for t in tensors)
        self.tensor_gpus = [physical_gpu(t.device.index) for t in tensors]
        self.gpus = sorted(set(self.tensor_gpus))
        self.last = time.time()
        self.state = "hbm"
        self.serialized = serialized      # the value with its CUDA tensors as slots (host parts)


class _PinnedPool:
    """Reusable pinned (page-locked) host buffers for spills, by size class. ``hipHostMalloc`` is
    slow (it maps and pins every page) and used to run once per spilled tensor under the store
    lock; buffers now come from this pool and go back to it on restore. Cached bytes are bounded
    by ``RCA_GPU_SPILL_POOL_BYTES`` (default 8 GiB)."""

    def __init__(self, cap_bytes: Optional[int] = None):
        import os

        self.cap = int(cap_bytes if cap_bytes is not None else os.environ.get("RCA_GPU_SPILL_POOL_BYTES", 8 << 30))
        self.free_lists: Dict[int, list] = {}
        self.cached = 0
        self.hits = 0
        self.misses = 0
        self.lock = threading.Lock()

    @staticmethod
    def size_class(n: int) -> int:
        if n <= (1 << 20):
            return 1 << 20
        return 1 << (int(n - 1).bit_length())  # next power of two: <= 2x slack, few classes

    def take(self, nbytes: int):
        import torch

        c = self.size_class(max(1, nbytes))
        with self.lock:
            fl = self.free_lists.get(c)
            if fl:
                self.cached -= c
                self.hits += 1
                return fl.pop()
            self.misses += 1
        return torch.empty(c, dtype=torch.uint8, pin_memory=True)

    def give(self, buf):
        c = buf.numel()
        with self.lock:
            if self.cached + c <= self.cap:
                self.free_lists.setdefault(c, []).append(buf)
                self.cached += c


def _host_view(buf, t):
    """A host tensor shaped / strided like device tensor ``t`` over pinned byte buffer ``buf``."""
    span = 1 + sum((n - 1) * st for n, st in zip(t.shape, t.stride())) if t.numel() else 0
    flat = buf[: max(span, 1) * t.element_size()].view(t.dtype)
    return flat.as_strided(t.shape, t.stride())


class GpuObjectStore:
    """Device-resident objects owned by this process.

    Spill / restore copy outside the store lock: an entry moves hbm -> spilling -> host (and
    host -> restoring -> hbm) under the lock, the copies run on a per-device side stream with ONE
    event per object, and pinned host buffers come from ``_PinnedPool``. Readers of other objects
    never wait behind a copy; a restore of an object that is being spilled waits for that spill."""

    def __init__(self):
        self.entries: Dict[bytes, _Entry] = {}
        self.lock = threading.RLock()
        self.cond = threading.Condition(self.lock)
        self._stream = None
        self.pool = _PinnedPool()
        self.num_spilled = 0
        self.num_restored = 0
        self.spilled_bytes = 0

    def _side_stream(self, dev):
        import torch

        if self._stream is None:
            self._stream = {}
        s = self._stream.get(dev)
        if s is None:
            s = torch.cuda.Stream(device=dev)
            self._stream[dev] = s
        return s

    # -------------------------------------------------------------- registration
    def add(self, oid: bytes, serialized, copy: bool) -> bytes:
        """Take ownership of the CUDA tensors of a serialized value for object ``oid`` (one
        device-to-device snapshot when ``copy``); returns the object's wire bytes (host parts +
        IPC export table)."""
        import torch

        owned = []
        for t in serialized.gpu_tensors:
            c = t.detach()
            dense = _dense_layout(c)
            if copy:
                # keep a dense layout (row-major or channels-last) as it is: a consumer that gets
                # NCHW bytes for an NHWC producer would silently run different (slower) kernels
                c = c.clone(memory_format=torch.preserve_format) if dense else c.clone(
                    memory_format=torch.contiguous_format)
            elif not dense:
                c = c.contiguous()
            owned.append(c)
        if owned:
            torch.cuda.current_stream(owned[0].device).synchronize()
        serialized.gpu_tensors = []  # the store, not the skeleton, references the tensors now
        with self.lock:
            self.entries[oid] = _Entry(owned, serialized)
        return serialized.to_bytes_with_table(encode_table([export_tensor(t, oid, i) for i, t in enumerate(owned)]))

    def info(self, oid):
        e = self.entries.get(oid)
        return None if e is None else {"nbytes": e.nbytes, "gpus": e.gpus}

    def local_tensor(self, rec):
        """Same-process reader: the store's own tensor (HIP cannot IPC-open its own allocation)."""
        with self.lock:
            e = self.entries.get(rec.get("oid"))
            if e is None or e.tensors is None or rec.get("slot", 0) >= len(e.tensors):
                return None
            e.last = time.time()
            return e.tensors[rec["slot"]]

    # -------------------------------------------------------------- spill / restore
    def spill(self, oid) -> int:
        """Copy the object's tensors into pinned host memory (async copies on a side stream, one
        event) and release its HBM. Returns the bytes released."""
        import torch

        with self.lock:
            e = self.entries.get(oid)
            if e is None or e.state != "hbm":
                return 0
            e.state = "spilling"
            tensors = list(e.tensors)
        try:
            host, bufs, last = [], [], {}
            for t in tensors:
                s = self._side_stream(t.device)
                if t.device not in last:
                    s.wait_stream(torch.cuda.current_stream(t.device))
                buf = self.pool.take(t.numel() * t.element_size())
                h = _host_view(buf, t)
                with torch.cuda.stream(s):
                    h.copy_(t, non_blocking=True)
                last[t.device] = s
                host.append(h)
                bufs.append(buf)
            for s in last.values():  # one wait per device, not per tensor
                ev = torch.cuda.Event()
                ev.record(s)
                ev.synchronize()
        except BaseException:
            with self.lock:
                e.state = "hbm"
                self.cond.notify_all()
            raise
        with self.lock:
            e.host, e.host_bufs = host, bufs
            e.tensors = None
            e.state = "host"
            self.num_spilled += 1
            self.spilled_bytes += e.nbytes
            self.cond.notify_all()
        return e.nbytes

    def restore(self, oid) -> Optional[bytes]:
        """Bring a spilled object back into HBM (pinned H2D copies on a side stream, one event);
        returns the object's fresh wire bytes."""
        import torch

        with self.lock:
            e = self.entries.get(oid)
            if e is None:
                return None
            while e.state in ("spilling", "restoring"):
                self.cond.wait(timeout=1.0)
                if self.entries.get(oid) is not e:
                    return None
            mine = e.state == "host"
            if mine:
                e.state = "restoring"
                host, bufs = e.host, e.host_bufs
        if mine:
            try:
                out, last = [], {}
                for h, g in zip(host, e.tensor_gpus):
                    dev = _local_index(g)
                    dev = torch.cuda.current_device() if dev is None else dev
                    d = torch.device("cuda", dev)
                    s = self._side_stream(d)
                    with torch.cuda.stream(s):
                        t = torch.empty_strided(h.shape, h.stride(), dtype=h.dtype, device=d)
                        t.copy_(h, non_blocking=True)
                    last[d] = s
                    out.append(t)
                for d, s in last.items():
                    ev = torch.cuda.Event()
                    ev.record(s)
                    ev.synchronize()
                    # tensors allocated on the side stream are used on the default stream next
                    for t in out:
                        if t.device == d:
                            t.record_stream(torch.cuda.current_stream(d))
            except BaseException:
                with self.lock:
                    e.state = "host"
                    self.cond.notify_all()
                raise
            for b in bufs or ():
                self.pool.give(b)
            with self.lock:
                e.tensors = out
                e.host = e.host_bufs = None
                e.state = "hbm"
                self.num_restored += 1
                self.cond.notify_all()
        with self.lock:
            if e.tensors is None:
                return None
            e.last = time.time()
            table = encode_table([export_tensor(t, oid, i) for i, t in enumerate(e.tensors)])
            return e.serialized.to_bytes_with_table(table)

    def free(self, oids):
        bufs = []
        with self.lock:
            for o in oids:
                e = self.entries.pop(o, None)
                if e is not None and e.state == "host" and e.host_bufs:
                    bufs += e.host_bufs
        for b in bufs:
            self.pool.give(b)

    def stats(self):
        with self.lock:
            hbm = sum(e.nbytes for e in self.entries.values() if e.state == "hbm")
            host = sum(e.nbytes for e in self.entries.values() if e.state == "host")
        return {"objects": len(self.entries), "hbm_bytes": hbm, "host_bytes": host, "num_spilled": self.num_spilled,
                "num_restored": self.num_restored, "pinned_pool_cached_bytes": self.pool.cached,
                "pinned_pool_hits": self.pool.hits, "pinned_pool_misses": self.pool.misses}


_STORE: Optional[GpuObjectStore] = None


def _local_store() -> GpuObjectStore:
    global _STORE
    if _STORE is None:
        _STORE = GpuObjectStore()
    return _STORE


def local_store() -> GpuObjectStore:
    return _local_store()


def encode_table(records: List[dict]) -> bytes:
    return pickle.dumps(records, protocol=5)


def decode_table(b) -> List[dict]:
    return pickle.loads(bytes(b))
