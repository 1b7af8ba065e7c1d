"""HTTP plumbing between the proxy and replicas (reference: ``serve/_private/http_util.py``,
``proxy.py``). The proxy serialises each request to a plain dict; the replica either runs the
deployment's ASGI app (``@serve.ingress(FastAPI)``) or calls ``__call__(request)`` with a
Starlette ``Request``, and returns ``(status, headers, body)``."""
from __future__ import annotations

import inspect
import json
from typing import Any, Dict, List, Tuple


def _to_response(result) -> Tuple[int, List, bytes]:
    try:
        from starlette.responses import Response
    except ImportError:  # pragma: no cover
        Response = None
    if Response is not None and isinstance(result, Response):
        return result.status_code, [(k.decode(), v.decode()) for k, v in result.raw_headers], result.body
    if isinstance(result, (bytes, bytearray)):
        return 200, [("content-type", "application/octet-stream")], bytes(result)
    if isinstance(result, str):
        return 200, [("content-type", "text/plain; charset=utf-8")], result.encode()
    try:
        import numpy as np

        if isinstance(result, np.ndarray):
            result = result.tolist()
    except ImportError:
        pass
    return 200, [("content-type", "application/json")], json.dumps(result, default=_jsonable).encode()


def _jsonable(o):
    try:
        import numpy as np

        if isinstance(o, np.generic):
            return o.item()
        if isinstance(o, np.ndarray):
            return o.tolist()
    except ImportError:
        pass
    return str(o)


def _scope(req: Dict) -> Dict:
    headers = [(k.encode() if isinstance(k, str) else k, v.encode() if isinstance(v, str) else v)
               for k, v in req.get("headers", [])]
    if req.get("type") == "websocket":
        return {"type": "websocket", "asgi": {"version": "3.0"}, "http_version": "1.1", "scheme": "ws",
                "path": req["path"], "raw_path": req["path"].encode(), "query_string": req.get("query_string", b""),
                "root_path": req.get("root_path", ""), "headers": headers,
                "subprotocols": list(req.get("subprotocols") or []),
                "client": ("127.0.0.1", 0), "server": ("127.0.0.1", 8000)}
    return {"type": "http", "asgi": {"version": "3.0"}, "http_version": "1.1", "method": req["method"],
            "scheme": "http", "path": req["path"], "raw_path": req["path"].encode(),
            "query_string": req.get("query_string", b""), "root_path": req.get("root_path", ""),
            "headers": headers, "client": ("127.0.0.1", 0), "server": ("127.0.0.1", 8000)}


class _StreamReceive:
    """The replica side of a streamed request (``req["stream"]``, serve/_private/proxy.py): ASGI
    ``receive()`` that hands out the inline first chunk, then pulls the next client messages from
    the proxy (``receive_asgi_messages``) only when the app asks for them. After the request body
    ended it parks like a real server's receive (an app listening for a disconnect must not see
    one); a WebSocket's ``websocket.disconnect`` is delivered and then repeated."""

    def __init__(self, req: Dict):
        from collections import deque

        self.ws = req.get("type") == "websocket"
        st = req.get("stream")
        self.proxy = st["proxy"] if st else None
        self.sid = st["id"] if st else None
        self.buf = deque()
        if not self.ws:
            self.buf.append({"type": "http.request", "body": req.get("body", b""), "more_body": st is not None})
        self.ended = st is None and not self.ws
        self.last = None

    async def __call__(self):
        import asyncio

        if self.buf:
            msg = self.buf.popleft()
            self._note(msg)
            return msg
        if self.ended:
            if self.ws:
                return self.last or {"type": "websocket.disconnect", "code": 1000}
            await asyncio.sleep(3600)  # no more request body: park like a real server
        msgs = await self.proxy.receive_asgi_messages.remote(self.sid)
        if not msgs:
            self.ended = True
            if self.ws:
                self.last = {"type": "websocket.disconnect", "code": 1006}
                return self.last
            return {"type": "http.disconnect"}
        self.buf.extend(msgs)
        msg = self.buf.popleft()
        self._note(msg)
        return msg

    def _note(self, msg):
        t = msg.get("type")
        if t == "websocket.disconnect":
            self.ended, self.last = True, msg
        elif t == "http.request" and not msg.get("more_body"):
            self.ended = True
        elif t == "http.disconnect":
            self.ended = True


async def run_asgi_or_call(replica, req: Dict):
    obj = replica.obj
    spec = getattr(type(obj), "_serve_ingress_spec", None) if not replica.is_function else None
    if spec is not None:
        app = getattr(replica, "_asgi_app", None)
        if app is None:
            from ..api import _build_ingress_app

            app = replica._asgi_app = _build_ingress_app(spec, obj)
        return await _run_asgi(app, req)
    from starlette.requests import Request

    body = req.get("body", b"")

    async def receive():
        return {"type": "http.request", "body": body, "more_body": False}

    request = Request(_scope(req), receive)
    res = await replica._call_user("__call__", (request,), {})
    return _to_response(res)


async def _run_asgi(app, req: Dict):
    body = req.get("body", b"")
    scope = _scope(req)
    sent = {"status": 500, "headers": [], "body": b""}
    done = {"v": False}

    async def receive():
        if done["v"]:
            return {"type": "http.disconnect"}
        done["v"] = True
        return {"type": "http.request", "body": body, "more_body": False}

    async def send(msg):
        if msg["type"] == "http.response.start":
            sent["status"] = msg["status"]
            sent["headers"] = [(k.decode(), v.decode()) for k, v in msg.get("headers", [])]
        elif msg["type"] == "http.response.body":
            sent["body"] += msg.get("body", b"")

    await app(scope, receive, send)
    return sent["status"], sent["headers"], sent["body"]


async def stream_asgi_or_call(replica, req: Dict):
    """Async generator of response messages: ("start", status, headers), ("body", chunk)*."""
    import asyncio

    obj = replica.obj
    spec = getattr(type(obj), "_serve_ingress_spec", None) if not replica.is_function else None
    ws = req.get("type") == "websocket"
    if ws and spec is None:
        # WebSockets need an ASGI ingress (reference: FastAPI @serve.ingress): refuse the handshake
        yield ("ws", {"type": "websocket.close", "code": 1003})
        return
    if spec is not None:
        app = getattr(replica, "_asgi_app", None)
        if app is None:
            from ..api import _build_ingress_app

            app = replica._asgi_app = _build_ingress_app(spec, obj)
        q: asyncio.Queue = asyncio.Queue()
        receive = _StreamReceive(req)

        async def send(msg):
            await q.put(msg)

        async def run():
            try:
                await app(_scope(req), receive, send)
            finally:
                await q.put(None)

        task = asyncio.ensure_future(run())
        try:
            while True:
                msg = await q.get()
                if msg is None:
                    break
                if ws:
                    yield ("ws", msg)
                    continue
                if msg["type"] == "http.response.start":
                    yield ("start", msg["status"], [(k.decode(), v.decode()) for k, v in msg.get("headers", [])])
                elif msg["type"] == "http.response.body":
                    if msg.get("body"):
                        yield ("body", msg["body"])
        finally:
            await task
        return
    from starlette.requests import Request

    request = Request(_scope(req), _StreamReceive(req))
    res = await replica._invoke_user("__call__", (request,), {})
    try:
        from starlette.responses import StreamingResponse
    except ImportError:  # pragma: no cover
        StreamingResponse = None
    if StreamingResponse is not None and isinstance(res, StreamingResponse):
        yield ("start", res.status_code, [(k.decode(), v.decode()) for k, v in res.raw_headers])
        async for chunk in res.body_iterator:
            yield ("body", chunk.encode() if isinstance(chunk, str) else chunk)
        return
    if inspect.isgenerator(res) or inspect.isasyncgen(res):
        from .replica import _aiter

        yield ("start", 200, [("content-type", "text/plain; charset=utf-8")])
        async for chunk in _aiter(res):
            yield ("body", chunk.encode() if isinstance(chunk, str) else bytes(chunk))
        return
    status, headers, out = _to_response(res)
    yield ("start", status, headers)
    yield ("body", out)
