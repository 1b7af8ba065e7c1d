"""WebSocket server protocol for the Serve HTTP proxy (RFC 6455), plugged into uvicorn as its
``ws`` protocol class (reference: the proxy serves ``websocket`` ASGI scopes through uvicorn's
websocket backends, ``python/ray/serve/_private/proxy.py:856-1103``).

uvicorn only speaks WebSocket through the ``websockets`` / ``wsproto`` packages, which this image
does not have; without a protocol class it answers every upgrade with 400. This one handles the
upgrade handshake and the framing itself: uvicorn's HTTP protocol detects the upgrade request and
hands the connection over (``handle_websocket_upgrade``: the request head is replayed into
``data_received``), and this class runs the ASGI app with a ``websocket`` scope:

  * handshake: the app's ``websocket.accept`` answers ``101 Switching Protocols`` with
    ``Sec-WebSocket-Accept`` (and the chosen subprotocol / extra headers); a ``websocket.close``
    before accepting answers ``403``;
  * frames: text / binary (fragmented messages reassembled), ping -> pong, close (echoed with the
    client's code); client frames must be masked (1002 otherwise), server frames are not;
    messages over ``max_message_bytes`` close with 1009;
  * ASGI: ``websocket.connect`` first, then ``websocket.receive`` per message and
    ``websocket.disconnect`` (with the close code) when the peer closes or the socket drops.
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import struct
from typing import Optional
from urllib.parse import unquote

_GUID = b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11"
_OP_CONT, _OP_TEXT, _OP_BIN, _OP_CLOSE, _OP_PING, _OP_PONG = 0x0, 0x1, 0x2, 0x8, 0x9, 0xA


def accept_key(key: bytes) -> bytes:
    return base64.b64encode(hashlib.sha1(key.strip() + _GUID).digest())


def encode_frame(opcode: int, payload: bytes, fin: bool = True, mask: Optional[bytes] = None) -> bytes:
    """One frame (server frames unmasked; ``mask`` for client-side use in tests)."""
    head = bytearray([(0x80 if fin else 0) | opcode])
    n = len(payload)
    mbit = 0x80 if mask else 0
    if n < 126:
        head.append(mbit | n)
    elif n < 1 << 16:
        head.append(mbit | 126)
        head += struct.pack("!H", n)
    else:
        head.append(mbit | 127)
        head += struct.pack("!Q", n)
    if mask:
        head += mask
        payload = bytes(b ^ mask[i & 3] for i, b in enumerate(payload))
    return bytes(head) + payload


class FrameParser:
    """Incremental RFC 6455 frame decoder: ``feed(bytes)`` -> list of (fin, opcode, payload)."""

    def __init__(self, require_mask: bool = True):
        self.buf = bytearray()
        self.require_mask = require_mask

    def feed(self, data: bytes):
        self.buf += data
        out = []
        while True:
            b = self.buf
            if len(b) < 2:
                return out
            fin, opcode = bool(b[0] & 0x80), b[0] & 0x0F
            masked, n = bool(b[1] & 0x80), b[1] & 0x7F
            pos = 2
            if n == 126:
                if len(b) < 4:
                    return out
                n = struct.unpack_from("!H", b, 2)[0]
                pos = 4
            elif n == 127:
                if len(b) < 10:
                    return out
                n = struct.unpack_from("!Q", b, 2)[0]
                pos = 10
            if self.require_mask and not masked:
                raise ValueError("unmasked client frame")
            key = b""
            if masked:
                if len(b) < pos + 4:
                    return out
                key = bytes(b[pos:pos + 4])
                pos += 4
            if len(b) < pos + n:
                return out
            payload = bytes(b[pos:pos + n])
            if masked:
                payload = _unmask(payload, key)
            del self.buf[:pos + n]
            out.append((fin, opcode, payload))


def _unmask(payload: bytes, key: bytes) -> bytes:
    if not payload:
        return payload
    # XOR with the 4-byte key repeated: one big-int XOR instead of a per-byte Python loop
    reps = (len(payload) + 3) // 4
    k = int.from_bytes(key * reps, "big") >> (8 * (4 * reps - len(payload)))
    return (int.from_bytes(payload, "big") ^ k).to_bytes(len(payload), "big")


class RFC6455Protocol(asyncio.Protocol):
    max_message_bytes = 16 << 20

    def __init__(self, config, server_state, app_state=None, _loop=None):
        self.config = config
        self.app = config.loaded_app
        self.root_path = getattr(config, "root_path", "") or ""
        self.server_state = server_state
        self.connections = server_state.connections
        self.transport = None
        self.head = bytearray()
        self.parser = FrameParser()
        self.queue: "asyncio.Queue[dict]" = asyncio.Queue()
        self.scope = None
        self.key = b""
        self.accepted = False
        self.closed_by_app = False
        self.disconnected = False
        self.frag_op: Optional[int] = None
        self.frag: bytearray = bytearray()
        self.task = None

    # ------------------------------------------------------------------ asyncio.Protocol
    def connection_made(self, transport):
        self.transport = transport
        self.connections.add(self)

    def connection_lost(self, exc):
        self.connections.discard(self)
        self._disconnect(1006)

    def data_received(self, data: bytes):
        if self.scope is None:
            self.head += data
            end = self.head.find(b"\r\n\r\n")
            if end < 0:
                return
            rest = bytes(self.head[end + 4:])
            if not self._handshake(bytes(self.head[:end])):
                return
            if not rest:
                return
            data = rest
        try:
            frames = self.parser.feed(data)
        except ValueError:
            self._close_frame(1002)
            return
        for fin, op, payload in frames:
            self._on_frame(fin, op, payload)

    def shutdown(self):  # uvicorn's graceful shutdown
        if self.accepted and not self.closed_by_app:
            self._close_frame(1012)
        elif self.transport is not None:
            self.transport.close()

    # ------------------------------------------------------------------ handshake / frames
    def _handshake(self, head: bytes) -> bool:
        lines = head.split(b"\r\n")
        try:
            method, target, _ = lines[0].split(b" ", 2)
        except ValueError:
            self._http_error(400)
            return False
        headers = []
        hmap = {}
        for line in lines[1:]:
            if b":" not in line:
                continue
            k, v = line.split(b":", 1)
            k, v = k.strip().lower(), v.strip()
            headers.append((k, v))
            hmap[k] = v
        self.key = hmap.get(b"sec-websocket-key", b"")
        if method != b"GET" or b"websocket" not in hmap.get(b"upgrade", b"").lower() or not self.key:
            self._http_error(400)
            return False
        path, _, query = target.partition(b"?")
        sub = [s.strip().decode() for s in hmap.get(b"sec-websocket-protocol", b"").split(b",") if s.strip()]
        peer = self.transport.get_extra_info("peername")
        sock = self.transport.get_extra_info("sockname")
        self.scope = {"type": "websocket", "asgi": {"version": "3.0", "spec_version": "2.3"}, "http_version": "1.1",
                      "scheme": "ws", "path": unquote(path.decode("latin-1")), "raw_path": path,
                      "query_string": query, "root_path": self.root_path, "headers": headers,
                      "client": tuple(peer[:2]) if peer else None, "server": tuple(sock[:2]) if sock else None,
                      "subprotocols": sub, "state": {}}
        self.queue.put_nowait({"type": "websocket.connect"})
        self.task = asyncio.get_running_loop().create_task(self._run())
        return True

    def _on_frame(self, fin: bool, op: int, payload: bytes):
        if op == _OP_PING:
            self._write(encode_frame(_OP_PONG, payload))
            return
        if op == _OP_PONG:
            return
        if op == _OP_CLOSE:
            code = struct.unpack("!H", payload[:2])[0] if len(payload) >= 2 else 1005
            if not self.closed_by_app:  # echo the close; the app's later sends are dropped
                self._write(encode_frame(_OP_CLOSE, payload[:2]))
                self.closed_by_app = True
            self._disconnect(code)
            if self.transport is not None:
                self.transport.close()
            return
        if op in (_OP_TEXT, _OP_BIN):
            self.frag_op, self.frag = op, bytearray(payload)
        elif op == _OP_CONT and self.frag_op is not None:
            self.frag += payload
        else:
            self._close_frame(1002)
            return
        if len(self.frag) > self.max_message_bytes:
            self._close_frame(1009)
            return
        if fin:
            msg = {"type": "websocket.receive"}
            if self.frag_op == _OP_TEXT:
                msg["text"] = bytes(self.frag).decode("utf-8", "replace")
            else:
                msg["bytes"] = bytes(self.frag)
            self.frag_op, self.frag = None, bytearray()
            self.queue.put_nowait(msg)

    def _disconnect(self, code: int):
        if not self.disconnected:
            self.disconnected = True
            self.queue.put_nowait({"type": "websocket.disconnect", "code": code})

    def _write(self, data: bytes):
        if self.transport is not None and not self.transport.is_closing():
            self.transport.write(data)

    def _close_frame(self, code: int, reason: str = ""):
        self._write(encode_frame(_OP_CLOSE, struct.pack("!H", code) + reason.encode()[:120]))
        self.closed_by_app = True
        self._disconnect(code)
        if self.transport is not None:
            self.transport.close()

    def _http_error(self, status: int):
        reason = {400: b"Bad Request", 403: b"Forbidden", 500: b"Internal Server Error"}.get(status, b"Error")
        self._write(b"HTTP/1.1 %d %s\r\ncontent-length: 0\r\nconnection: close\r\n\r\n" % (status, reason))
        if self.transport is not None:
            self.transport.close()

    # ------------------------------------------------------------------ ASGI
    async def _run(self):
        try:
            await self.app(self.scope, self.receive, self.send)
        except Exception:  # noqa - the app failed: 500 before the handshake, 1011 after
            if not self.accepted:
                self._http_error(500)
            elif not self.closed_by_app:
                self._close_frame(1011)
            return
        if not self.accepted:
            self._http_error(403 if not self.disconnected else 500)
        elif not self.closed_by_app:
            self._close_frame(1000)

    async def receive(self):
        return await self.queue.get()

    async def send(self, message):
        t = message["type"]
        if t == "websocket.accept":
            if self.accepted:
                return
            self.accepted = True
            lines = [b"HTTP/1.1 101 Switching Protocols", b"upgrade: websocket", b"connection: Upgrade",
                     b"sec-websocket-accept: " + accept_key(self.key)]
            if message.get("subprotocol"):
                lines.append(b"sec-websocket-protocol: " + message["subprotocol"].encode())
            for k, v in message.get("headers") or []:
                lines.append((k if isinstance(k, bytes) else k.encode()) + b": "
                             + (v if isinstance(v, bytes) else v.encode()))
            self._write(b"\r\n".join(lines) + b"\r\n\r\n")
        elif t == "websocket.send":
            if not self.accepted or self.closed_by_app:
                return
            if message.get("bytes") is not None:
                self._write(encode_frame(_OP_BIN, bytes(message["bytes"])))
            else:
                self._write(encode_frame(_OP_TEXT, (message.get("text") or "").encode()))
        elif t == "websocket.close":
            if not self.accepted:
                self.closed_by_app = True
                self._http_error(403)
            elif not self.closed_by_app:
                self._close_frame(int(message.get("code") or 1000), message.get("reason") or "")
