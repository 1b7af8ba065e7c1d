"""Length-prefixed message framing over Unix sockets (head <-> workers / client drivers).

Reference: the raylet/core-worker gRPC + flatbuffers protocols (``src/ray/protobuf``,
``src/ray/raylet/format``). Here one persistent AF_UNIX stream per process carries pickled
tuples ``(msg_type, *fields)``; small frames are coalesced into a single ``sendall``.
"""
from __future__ import annotations

import pickle
import socket
import struct
import threading

_LEN = struct.Struct("<Q")

# worker/client -> head
REGISTER = 1
TASK_DONE = 2
RPC = 3            # (RPC, req_id, method, args, kwargs)
REF_DELTA = 4      # (REF_DELTA, adds, removes)
GEN_ITEM = 5       # (GEN_ITEM, task_id, index, desc)
BLOCKED = 6        # (BLOCKED, flag)
LOG = 7
# head -> worker
EXECUTE = 20       # (EXECUTE, task_spec_dict)
REPLY = 21         # (REPLY, req_id, ok, value)
EXIT = 22
CANCEL = 23        # (CANCEL, task_id, force)
FREE_GPU = 24      # (FREE_GPU, [object_ids])
PING = 25
GPU_CMD = 26       # (GPU_CMD, "spill" | "restore", [object_ids])  head -> GPU-object owner
LOG_BATCH = 27     # (LOG_BATCH, [{pid, label, node, lines}])       head -> log_to_driver drivers
# worker -> head: batched records of directly transported actor calls
DIRECT_EVENTS = 30  # (DIRECT_EVENTS, [(tid, name, actor_id, start, end, failed, error_type)])
# caller <-> actor worker (direct transport, _private/direct_transport.py)
DEXEC = 40         # (DEXEC, task_spec_dict)              caller -> actor worker
DDONE = 41         # (DDONE, task_id, [desc], head_managed) actor worker -> caller
DCANCEL = 42       # (DCANCEL, task_id, force)             caller -> actor worker


def dumps(msg) -> bytes:
    return pickle.dumps(msg, protocol=5)


def loads(b):
    return pickle.loads(b)


def _native_send_frame():
    try:
        from .._native import load

        return load().send_frame
    except Exception:  # noqa  (no native module: pure-Python framing)
        return None


_SEND_FRAME = _native_send_frame()


class Connection:
    """Blocking framed connection with a send lock (many threads may send). Frames go out
    through the native ``send_frame`` (header + payload in one ``sendmsg``, GIL released for
    large payloads) when the runtime core is built."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self._send_lock = threading.Lock()
        self._closed = False

    def send(self, msg):
        data = dumps(msg)
        with self._send_lock:
            if _SEND_FRAME is not None:
                _SEND_FRAME(self.sock.fileno(), data)
                return
            hdr = _LEN.pack(len(data))
            if len(data) < 65536:
                self.sock.sendall(hdr + data)
            else:
                self.sock.sendall(hdr)
                self.sock.sendall(data)

    def recv(self):
        hdr = self._recv_exact(8)
        (n,) = _LEN.unpack(hdr)
        return loads(self._recv_exact(n))

    def _recv_exact(self, n):
        buf = bytearray(n)
        mv = memoryview(buf)
        got = 0
        while got < n:
            k = self.sock.recv_into(mv[got:], n - got)
            if k == 0:
                raise ConnectionError("connection closed")
            got += k
        return buf

    def close(self):
        if not self._closed:
            self._closed = True
            try:
                self.sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            self.sock.close()

    def fileno(self):
        return self.sock.fileno()


class FrameReader:
    """Incremental non-blocking reader used by the head's selector loop."""

    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes):
        buf = self.buf
        buf += data
        out = []
        off = 0
        L = len(buf)
        while L - off >= 8:
            (n,) = _LEN.unpack_from(buf, off)
            if L - off < 8 + n:
                break
            out.append(pickle.loads(bytes(buf[off + 8: off + 8 + n])))
            off += 8 + n
        if off:
            del buf[:off]
        return out
