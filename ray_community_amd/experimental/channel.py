"""Shared-memory channels for compiled DAGs (reference: ``python/ray/experimental/channel.py``).

A channel is one POSIX shared-memory segment: a header of u64 words ``[write_seq, nbytes,
ack[0..R)]`` followed by the payload. ``write`` waits until every reader has acknowledged the
previous value, copies the pickled value in and publishes it by bumping ``write_seq`` (x86 keeps
stores in order, and the header words are single aligned 8-byte stores). Readers poll
``write_seq``; ``end_read`` acknowledges. No broker, no RPC: a driver->actor->actor->driver hop is
a handful of memory copies. GPU tensors inside values travel as HIP IPC handles (the object
serializer's GPU path), so HBM payloads are not copied either.
"""
from __future__ import annotations

import pickle
import time
from multiprocessing import resource_tracker, shared_memory
from typing import Any, Optional

import numpy as np

DEFAULT_BUFFER = 10 * 1024 * 1024


class ChannelTimeoutError(TimeoutError):
    pass


class _Closed:
    """Sentinel written into channels at teardown."""

    def __reduce__(self):
        return (_Closed, ())


def _wait(cond, timeout: Optional[float]):
    deadline = None if timeout is None else time.monotonic() + timeout
    spins = 0
    while not cond():
        spins += 1
        if spins < 2000:
            continue
        if deadline is not None and time.monotonic() > deadline:
            raise ChannelTimeoutError("channel operation timed out")
        time.sleep(0 if spins < 20000 else 50e-6)


class Channel:
    def __init__(self, buffer_size_bytes: Optional[int] = None, num_readers: int = 1, _name: Optional[str] = None):
        self.num_readers = int(num_readers)
        self.capacity = int(buffer_size_bytes or DEFAULT_BUFFER)
        self._hdr_words = 2 + self.num_readers
        self._data_off = ((self._hdr_words * 8 + 63) // 64) * 64
        if _name is None:
            self._shm = shared_memory.SharedMemory(create=True, size=self._data_off + self.capacity)
            self._owner = True
        else:
            self._shm = shared_memory.SharedMemory(name=_name)
            try:  # attached segments must not be unlinked by this process's resource tracker
                resource_tracker.unregister(self._shm._name, "shared_memory")
            except Exception:
                pass
            self._owner = False
        self.name = self._shm.name
        self._hdr = np.ndarray((self._hdr_words,), dtype=np.uint64, buffer=self._shm.buf, offset=0)
        if self._owner:
            self._hdr[:] = 0
        self._read_seq = [0] * self.num_readers

    def __reduce__(self):
        return (_attach, (self.name, self.capacity, self.num_readers))

    # ------------------------------------------------------------------ writer
    def write(self, value: Any, timeout: Optional[float] = None):
        data = pickle.dumps(value, protocol=5) if not isinstance(value, _Closed) else b"\x00CLOSED"
        if len(data) > self.capacity:
            raise ValueError(f"value of {len(data)} bytes exceeds the channel buffer ({self.capacity} bytes); "
                             f"compile with a larger buffer_size_bytes")
        hdr = self._hdr
        seq = int(hdr[0])
        _wait(lambda: all(int(hdr[2 + r]) >= seq for r in range(self.num_readers)), timeout)
        self._shm.buf[self._data_off:self._data_off + len(data)] = data
        hdr[1] = len(data)
        hdr[0] = seq + 1

    def can_write(self) -> bool:
        """Every reader has acknowledged the current value, so ``write`` would not block."""
        hdr = self._hdr
        seq = int(hdr[0])
        return all(int(hdr[2 + r]) >= seq for r in range(self.num_readers))

    def close(self):
        try:
            self.write(_Closed(), timeout=5.0)
        except Exception:
            pass

    # ------------------------------------------------------------------ reader
    def begin_read(self, reader: int = 0, timeout: Optional[float] = None) -> Any:
        hdr = self._hdr
        want = self._read_seq[reader] + 1
        _wait(lambda: int(hdr[0]) >= want, timeout)
        n = int(hdr[1])
        data = bytes(self._shm.buf[self._data_off:self._data_off + n])
        self._read_seq[reader] = want
        if data == b"\x00CLOSED":
            return _Closed()
        return pickle.loads(data)

    def end_read(self, reader: int = 0):
        self._hdr[2 + reader] = self._read_seq[reader]

    def read(self, reader: int = 0, timeout: Optional[float] = None) -> Any:
        v = self.begin_read(reader, timeout)
        self.end_read(reader)
        return v

    def destroy(self):
        try:
            self._hdr = None
            self._shm.close()
        except Exception:
            pass
        if self._owner:
            try:
                self._shm.unlink()
            except Exception:
                pass


class ReaderInterface:
    """Reads one value per execution from a list of input channels (reference
    experimental/channel/common.py). ``read()`` returns the values in channel order."""

    def __init__(self, input_channels, reader_index: int = 0):
        self._channels = list(input_channels)
        self._idx = reader_index
        self._closed = False

    def start(self):
        pass

    def read(self, timeout: Optional[float] = None) -> list:
        if self._closed:
            raise RayChannelErrorClosed("reader is closed")
        return [c.read(self._idx, timeout) for c in self._channels]

    def close(self):
        self._closed = True


class SynchronousReader(ReaderInterface):
    pass


class AwaitableBackgroundReader(ReaderInterface):
    """Reads on a background thread; ``read()`` / ``await read_async()`` hand out the values."""

    def __init__(self, input_channels, reader_index: int = 0):
        super().__init__(input_channels, reader_index)
        import queue
        import threading

        self._q: "queue.Queue" = queue.Queue(maxsize=1)
        self._t = threading.Thread(target=self._loop, daemon=True)

    def start(self):
        self._t.start()

    def _loop(self):
        import queue

        while not self._closed:
            try:
                v = ReaderInterface.read(self, timeout=0.5)
            except ChannelTimeoutError:
                continue
            except Exception as e:  # noqa
                v = e
            while not self._closed:  # a bounded hand-off that still notices close()
                try:
                    self._q.put(v, timeout=0.5)
                    break
                except queue.Full:
                    continue
            if isinstance(v, Exception):
                return

    def read(self, timeout: Optional[float] = None) -> list:
        import queue

        try:
            v = self._q.get(timeout=timeout)
        except queue.Empty:
            raise ChannelTimeoutError("channel read timed out")
        if isinstance(v, Exception):
            raise v
        return v

    async def read_async(self) -> list:
        import asyncio

        return await asyncio.get_running_loop().run_in_executor(None, self.read)

    def close(self):
        """Stop the background thread (it re-checks within its 0.5 s read timeout) before the
        channels can be torn down."""
        self._closed = True
        if self._t.is_alive():
            self._t.join(timeout=5.0)


class WriterInterface:
    def __init__(self, output_channels):
        self._channels = list(output_channels)
        self._closed = False

    def start(self):
        pass

    def write(self, value, timeout: Optional[float] = None):
        for c in self._channels:
            c.write(value, timeout)

    def close(self):
        self._closed = True
        for c in self._channels:
            c.close()


class SynchronousWriter(WriterInterface):
    pass


class AwaitableBackgroundWriter(WriterInterface):
    """``await write_async(v)`` hands the value to a background thread that writes it."""

    async def write_async(self, value):
        import asyncio

        await asyncio.get_running_loop().run_in_executor(None, self.write, value)


class RayChannelErrorClosed(RuntimeError):
    pass


def _attach(name, capacity, num_readers):
    return Channel(capacity, num_readers, _name=name)


def __getattr__(name):  # reference import path: ray.experimental.channel.torch_tensor_type.TorchTensorType
    if name in ("TorchTensorType", "torch_tensor_type"):
        from ..dag import torch_tensor

        return torch_tensor.TorchTensorType if name == "TorchTensorType" else torch_tensor
    raise AttributeError(name)
