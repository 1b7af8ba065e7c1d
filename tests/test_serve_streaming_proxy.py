"""Serve proxy: request bodies streamed to the replica as the app consumes them, and WebSocket
sessions (reference python/ray/serve/_private/proxy.py:430,856-1103 receive_asgi_messages;
tests/test_streaming_response.py, test_websockets.py). WebSocket sessions are driven two ways: through the proxy's ASGI app with
a scripted client (``HTTPProxy.run_asgi_session``), and end to end over a raw socket with a
minimal RFC 6455 client against the proxy's own protocol (``serve/_private/ws_protocol.py``;
uvicorn's websockets / wsproto backends are not installed here)."""
import hashlib

import pytest
import requests

import ray_community_amd as ray
from ray_community_amd import serve

PORT = 18131


@pytest.fixture
def serve_instance():
    ray.init(num_cpus=8, log_to_driver=False)
    serve.start(http_options={"port": PORT})
    yield
    serve.shutdown()
    ray.shutdown()


def _proxy():
    from ray_community_amd.serve.api import _STATE

    return _STATE["proxy"]


def test_large_upload_streams_with_bounded_proxy_memory(serve_instance):
    from fastapi import FastAPI, Request

    app = FastAPI()

    @serve.deployment
    @serve.ingress(app)
    class Sink:
        @app.post("/upload")
        async def upload(self, request: Request):
            h = hashlib.sha256()
            n = chunks = 0
            async for chunk in request.stream():  # consumed as it arrives
                h.update(chunk)
                n += len(chunk)
                chunks += 1
            return {"bytes": n, "sha": h.hexdigest(), "chunks": chunks}

    serve.run(Sink.bind(), route_prefix="/s")
    total, piece = 200 << 20, 1 << 20
    block = bytes(range(256)) * (piece // 256)
    ref = hashlib.sha256()
    for _ in range(total // piece):
        ref.update(block)

    def gen():
        for _ in range(total // piece):
            yield block

    r = requests.post(f"http://127.0.0.1:{PORT}/s/upload", data=gen(), timeout=300)
    assert r.status_code == 200, r.text
    out = r.json()
    assert out["bytes"] == total and out["sha"] == ref.hexdigest()
    st = ray.get(_proxy().stats.remote())
    assert st["streamed_requests"] >= 1 and st["streamed_bytes"] >= total - piece
    # the proxy never held more than one pull's budget (1 MiB) plus one client chunk at a time
    assert st["max_pull_bytes"] <= (1 << 20) + (256 << 10), st
    assert st["pulls"] >= total // ((1 << 20) + (256 << 10))
    import time

    deadline = time.time() + 10
    while st["open_streams"] and time.time() < deadline:  # closed right after the last body message
        time.sleep(0.05)
        st = ray.get(_proxy().stats.remote())
    assert st["open_streams"] == 0


def test_small_body_stays_inline_and_function_deployment_reads_stream(serve_instance):
    @serve.deployment
    async def echo_len(request):
        body = await request.body()
        return {"n": len(body), "head": body[:4].decode()}

    serve.run(echo_len.bind(), route_prefix="/e")
    before = ray.get(_proxy().stats.remote())["streamed_requests"]
    r = requests.post(f"http://127.0.0.1:{PORT}/e", data=b"abcd" * 10, timeout=60)
    assert r.json() == {"n": 40, "head": "abcd"}
    assert ray.get(_proxy().stats.remote())["streamed_requests"] == before  # one message: inline

    def gen():
        for i in range(40):
            yield (b"wxyz" if i == 0 else b"-") * 4096

    r = requests.post(f"http://127.0.0.1:{PORT}/e", data=gen(), timeout=60)
    assert r.json() == {"n": 4 * 4096 + 39 * 4096, "head": "wxyz"}


def test_websocket_echo_session_through_proxy_app(serve_instance):
    from fastapi import FastAPI, WebSocket, WebSocketDisconnect

    app = FastAPI()

    @serve.deployment
    @serve.ingress(app)
    class Echo:
        @app.websocket("/ws")
        async def ws(self, websocket: WebSocket):
            await websocket.accept()
            try:
                while True:
                    text = await websocket.receive_text()
                    await websocket.send_text(f"echo:{text}")
                    if text == "bye":
                        await websocket.close(code=1000)
                        return
            except WebSocketDisconnect:
                return

    serve.run(Echo.bind(), route_prefix="/chat")
    scope = {"type": "websocket", "path": "/chat/ws", "query_string": b"", "headers": [], "subprotocols": []}
    msgs = [{"type": "websocket.connect"}, {"type": "websocket.receive", "text": "hi"},
            {"type": "websocket.receive", "text": "there"}, {"type": "websocket.receive", "text": "bye"}]
    sent = ray.get(_proxy().run_asgi_session.remote(scope, msgs))
    kinds = [m["type"] for m in sent]
    assert kinds[0] == "websocket.accept"
    texts = [m.get("text") for m in sent if m["type"] == "websocket.send"]
    assert texts == ["echo:hi", "echo:there", "echo:bye"]
    assert kinds[-1] == "websocket.close" and sent[-1].get("code", 1000) == 1000
    assert ray.get(_proxy().stats.remote())["websocket_sessions"] >= 1

    # client disconnects first: the app sees WebSocketDisconnect, the proxy closes normally
    sent = ray.get(_proxy().run_asgi_session.remote(scope, [{"type": "websocket.connect"},
                                                             {"type": "websocket.receive", "text": "x"},
                                                             {"type": "websocket.disconnect", "code": 1001}]))
    assert [m.get("text") for m in sent if m["type"] == "websocket.send"] == ["echo:x"]

    # no route: the handshake is refused with a close
    sent = ray.get(_proxy().run_asgi_session.remote(dict(scope, path="/nope/ws"), [{"type": "websocket.connect"}]))
    assert sent == [{"type": "websocket.close", "code": 1000}] or sent[0]["type"] == "websocket.close"


def _ws_connect(path, protocols=None):
    """A minimal RFC 6455 client over a raw socket (no websocket client library is installed)."""
    import base64
    import os
    import socket

    from ray_community_amd.serve._private.ws_protocol import FrameParser, accept_key

    s = socket.create_connection(("127.0.0.1", PORT), timeout=60)
    key = base64.b64encode(os.urandom(16))
    req = (f"GET {path} HTTP/1.1\r\nHost: 127.0.0.1:{PORT}\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
           f"Sec-WebSocket-Key: {key.decode()}\r\nSec-WebSocket-Version: 13\r\n")
    if protocols:
        req += f"Sec-WebSocket-Protocol: {', '.join(protocols)}\r\n"
    s.sendall((req + "\r\n").encode())
    head = b""
    while b"\r\n\r\n" not in head:
        chunk = s.recv(4096)
        if not chunk:
            break
        head += chunk
    status_line, _, rest = head.partition(b"\r\n")
    hdrs, _, extra = rest.partition(b"\r\n\r\n")
    return s, status_line, hdrs, extra, key, FrameParser(require_mask=False), accept_key


def _ws_send(s, op, payload, fin=True):
    import os

    from ray_community_amd.serve._private.ws_protocol import encode_frame

    s.sendall(encode_frame(op, payload, fin=fin, mask=os.urandom(4)))


def _ws_recv(s, parser, pending):
    while not pending:
        data = s.recv(65536)
        if not data:
            return None
        pending.extend(parser.feed(data))
    return pending.pop(0)


def test_websocket_over_a_real_socket(serve_instance):
    """End to end: RFC 6455 handshake and framing in the proxy (serve/_private/ws_protocol.py),
    the session routed to a FastAPI ``@app.websocket`` ingress."""
    from fastapi import FastAPI, WebSocket, WebSocketDisconnect

    app = FastAPI()

    @serve.deployment
    @serve.ingress(app)
    class Echo:
        @app.websocket("/ws")
        async def ws(self, websocket: WebSocket):
            await websocket.accept(subprotocol="chat" if "chat" in websocket.scope.get("subprotocols", []) else None)
            try:
                while True:
                    msg = await websocket.receive()
                    if msg["type"] == "websocket.disconnect":
                        return
                    if msg.get("bytes") is not None:
                        await websocket.send_bytes(msg["bytes"][::-1])
                    else:
                        await websocket.send_text("echo:" + msg["text"])
                        if msg["text"] == "bye":
                            await websocket.close(code=4000)
                            return
            except WebSocketDisconnect:
                return

    serve.run(Echo.bind(), route_prefix="/chat")
    s, status, hdrs, extra, key, parser, accept_key = _ws_connect("/chat/ws", protocols=["chat"])
    assert status.startswith(b"HTTP/1.1 101"), status
    h = dict(l.split(b": ", 1) for l in hdrs.split(b"\r\n") if b": " in l)
    h = {k.lower(): v for k, v in h.items()}
    assert h[b"sec-websocket-accept"] == accept_key(key) and h[b"sec-websocket-protocol"] == b"chat"
    pending = parser.feed(extra) if extra else []
    _ws_send(s, 0x1, b"hello")
    assert _ws_recv(s, parser, pending) == (True, 0x1, b"echo:hello")
    _ws_send(s, 0x2, bytes(range(200)) * 400)  # 80 KB binary: 64-bit length field both ways
    fin, op, data = _ws_recv(s, parser, pending)
    assert op == 0x2 and data == (bytes(range(200)) * 400)[::-1]
    _ws_send(s, 0x1, b"frag", fin=False)  # a fragmented text message
    _ws_send(s, 0x0, b"mented", fin=True)
    assert _ws_recv(s, parser, pending)[2] == b"echo:fragmented"
    _ws_send(s, 0x9, b"ping!")
    assert _ws_recv(s, parser, pending) == (True, 0xA, b"ping!")
    _ws_send(s, 0x1, b"bye")
    assert _ws_recv(s, parser, pending)[2] == b"echo:bye"
    fin, op, data = _ws_recv(s, parser, pending)
    assert op == 0x8 and int.from_bytes(data[:2], "big") == 4000
    s.close()

    # client-initiated close: the app sees the disconnect, the proxy echoes the close frame
    s, status, _h, extra, _k, parser, _a = _ws_connect("/chat/ws")
    assert status.startswith(b"HTTP/1.1 101")
    pending = parser.feed(extra) if extra else []
    _ws_send(s, 0x8, (1000).to_bytes(2, "big"))
    fin, op, data = _ws_recv(s, parser, pending)
    assert op == 0x8 and int.from_bytes(data[:2], "big") == 1000
    s.close()

    # no such route: the handshake is refused
    s, status, *_ = _ws_connect("/nowhere/ws")
    assert status.startswith(b"HTTP/1.1 403"), status
    s.close()
