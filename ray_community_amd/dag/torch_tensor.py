"""Device-resident tensor edges for compiled DAGs (reference: ``python/ray/experimental/channel/
torch_tensor_type.py`` + ``torch_tensor_nccl_channel.py``: ``node.with_type_hint(TorchTensorType(
transport="nccl"))`` sends tensors GPU-to-GPU with NCCL send/recv).

MI355X-first design: a compiled DAG's actors live on one node, so the tensor never needs a
collective. The producer copies each output tensor into a persistent device slot it owns (one per
(node, position, shape, dtype)), exports the slot ONCE through HIP IPC and writes only a small
descriptor into the shared-memory channel; a consumer maps the slot once (peer access over xGMI
when the GPUs differ) and copies it into its own memory with one device-to-device copy before it
releases the channel. The channel's read/release protocol is the flow control: the producer
cannot overwrite a slot before every reader has released the previous value.
"""
from __future__ import annotations

import os
import uuid
from typing import Any, Dict, Optional


class TorchTensorType:
    """Type hint for a compiled-DAG edge carrying (structures of) torch tensors on the GPU.
    ``transport``: "auto" / "nccl" / "ipc" all select the device-resident path here."""

    AUTO = "auto"
    NCCL = "nccl"
    IPC = "ipc"

    def __init__(self, transport: str = "auto", device: Optional[str] = None, _static_shape: bool = False, **kw):
        if transport not in ("auto", "nccl", "ipc", "cpu"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport
        self.device = device

    @property
    def on_device(self) -> bool:
        return self.transport != "cpu"


class _GpuSlotRef:
    """What travels through the shared-memory channel instead of the tensor bytes."""
    __slots__ = ("slot", "rec")

    def __init__(self, slot: str, rec: dict):
        self.slot = slot
        self.rec = rec

    def __reduce__(self):
        return (_GpuSlotRef, (self.slot, self.rec))


def _map_tensors(x, fn):
    import torch

    if isinstance(x, torch.Tensor):
        return fn(x)
    if isinstance(x, tuple):
        return tuple(_map_tensors(v, fn) for v in x)
    if isinstance(x, list):
        return [_map_tensors(v, fn) for v in x]
    if isinstance(x, dict):
        return {k: _map_tensors(v, fn) for k, v in x.items()}
    return x


class DeviceSender:
    """Producer side of one typed edge (lives in the producing actor's DAG loop)."""

    def __init__(self):
        self._slots: Dict[tuple, tuple] = {}  # key -> (device tensor, export record, slot id)

    def pack(self, value: Any) -> Any:
        import torch

        counter = [0]
        copied = []

        def put(t: "torch.Tensor"):
            pos = counter[0]
            counter[0] += 1
            if not t.is_cuda:
                return t
            key = (pos, tuple(t.shape), t.dtype, t.device.index)
            ent = self._slots.get(key)
            if ent is None:
                from .._private.gpu_store import export_tensor

                buf = torch.empty(t.shape, dtype=t.dtype, device=t.device)
                ent = (buf, export_tensor(buf), uuid.uuid4().hex)
                self._slots[key] = ent
            buf, rec, sid = ent
            buf.copy_(t)
            copied.append(buf.device)
            return _GpuSlotRef(sid, rec)

        out = _map_tensors(value, put)
        for dev in set(copied):
            torch.cuda.current_stream(dev).synchronize()  # the slot holds the value before it is announced
        return out


class DeviceReceiver:
    """Consumer side: maps each producer slot once, copies values out before release."""

    def __init__(self):
        self._mapped: Dict[str, Any] = {}

    def unpack(self, value: Any) -> Any:
        import torch

        if not _has_slot(value):
            return value
        devs = set()

        def get(x):
            if not isinstance(x, _GpuSlotRef):
                return x
            src = self._mapped.get(x.slot)
            if src is None:
                from .._private.gpu_store import import_tensor

                src = import_tensor(x.rec)
                self._mapped[x.slot] = src
            dev = torch.device("cuda", torch.cuda.current_device())
            out = torch.empty_like(src, device=dev)
            out.copy_(src)  # peer read over xGMI when the slot lives on another GPU
            devs.add(dev)
            return out

        out = _walk(value, get)
        for d in devs:
            torch.cuda.current_stream(d).synchronize()  # done with the slot before the channel is released
        return out


def _walk(x, fn):
    if isinstance(x, _GpuSlotRef):
        return fn(x)
    if isinstance(x, tuple):
        return tuple(_walk(v, fn) for v in x)
    if isinstance(x, list):
        return [_walk(v, fn) for v in x]
    if isinstance(x, dict):
        return {k: _walk(v, fn) for k, v in x.items()}
    return x


def _has_slot(x) -> bool:
    if isinstance(x, _GpuSlotRef):
        return True
    if isinstance(x, (tuple, list)):
        return any(_has_slot(v) for v in x)
    if isinstance(x, dict):
        return any(_has_slot(v) for v in x.values())
    return False


_RECEIVER: Optional[DeviceReceiver] = None


def receiver() -> DeviceReceiver:
    """The process-wide receiver (mapped slots are shared by every DAG edge read here)."""
    global _RECEIVER
    if _RECEIVER is None or _RECEIVER_PID != os.getpid():
        _set_receiver()
    return _RECEIVER


_RECEIVER_PID = None


def _set_receiver():
    global _RECEIVER, _RECEIVER_PID
    _RECEIVER = DeviceReceiver()
    _RECEIVER_PID = os.getpid()
