"""HTTP proxy actor (reference: ``serve/_private/proxy.py``): a uvicorn ASGI server that matches
the longest route prefix, then forwards the request to the application's ingress deployment
through a DeploymentHandle (power-of-two-choices routing).

Request bodies and WebSocket traffic STREAM (reference ``proxy.py:430,856-1103``,
``receive_asgi_messages``): the proxy reads the first ASGI message itself; a body that fits in it
travels inline with the request, otherwise (``more_body``, or any ``websocket`` scope) the request
carries this proxy's actor handle and a stream id, and the replica's ASGI ``receive()`` pulls the
following messages with ``receive_asgi_messages`` as the app consumes them. The proxy reads from
the client only inside such a pull (at most ``pull_budget_bytes`` per pull), so a large upload is
never buffered here: uvicorn's own flow control pauses the socket between pulls. Response
messages -- ``http.response.*`` or ``websocket.*`` -- come back over the replica's streaming
generator and are forwarded the moment they are produced.
"""
from __future__ import annotations

import asyncio
import itertools
import threading
import time
from typing import Dict, List, Optional


class _RequestStream:
    """The client side of one streamed request: pulls ASGI messages from uvicorn's ``receive``
    on the server loop. A pull that stops early (budget or a short idle) keeps its pending
    ``receive()`` for the next pull, so no message is ever lost to a cancellation."""

    def __init__(self, receive, kind: str, budget: int):
        self.receive = receive
        self.kind = kind
        self.budget = budget
        self.pending: Optional[asyncio.Future] = None
        self.closed = False

    def _next(self):
        if self.pending is None:
            self.pending = asyncio.ensure_future(self.receive())
        return self.pending

    async def pull(self, idle_s: float = 0.02) -> List[Dict]:
        if self.closed:
            return []
        out: List[Dict] = []
        nbytes = 0
        while True:
            fut = self._next()
            if out:
                done, _ = await asyncio.wait({fut}, timeout=idle_s)
                if not done:
                    break  # nothing more right now: hand over what we have
            msg = await fut
            self.pending = None
            out.append(msg)
            t = msg.get("type", "")
            nbytes += len(msg.get("body") or b"") + len(msg.get("bytes") or b"") + len(msg.get("text") or "")
            if t in ("http.disconnect", "websocket.disconnect") or (t == "http.request" and not msg.get("more_body")):
                self.closed = True
                break
            if self.kind == "websocket" or nbytes >= self.budget:
                break  # websocket frames are delivered one by one, promptly
        return out


class HTTPProxy:
    def __init__(self, host: str = "127.0.0.1", port: int = 8000, request_timeout_s: Optional[float] = None,
                 keep_alive_timeout_s: int = 5, root_path: str = "", pull_budget_bytes: int = 1 << 20):
        self.host = host
        self.port = port
        self.keep_alive_timeout_s = int(keep_alive_timeout_s)
        self.root_path = root_path or ""
        # end-to-end request timeout (HTTPOptions.request_timeout_s): 408 if no response started
        self.request_timeout_s = request_timeout_s if request_timeout_s and request_timeout_s > 0 else None
        self.pull_budget_bytes = int(pull_budget_bytes)
        self.routes: Dict[str, tuple] = {}
        self.last_routes = 0.0
        self._streams: Dict[str, _RequestStream] = {}
        self._ids = itertools.count()
        self._self_handle = None
        self._stats = {"streamed_requests": 0, "websocket_sessions": 0, "pulls": 0, "max_pull_bytes": 0,
                       "streamed_bytes": 0}
        self._server = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        deadline = time.time() + 15
        while self._server is None or not getattr(self._server, "started", False):
            if time.time() > deadline:
                raise RuntimeError("HTTP proxy failed to start")
            time.sleep(0.02)

    def _run(self):
        import uvicorn

        from .ws_protocol import RFC6455Protocol

        # WebSocket upgrades go to the in-tree RFC 6455 protocol (uvicorn's own backends need the
        # websockets / wsproto packages)
        config = uvicorn.Config(self._app, host=self.host, port=self.port, log_level="warning", lifespan="off",
                                interface="asgi3", timeout_keep_alive=self.keep_alive_timeout_s,
                                root_path=self.root_path, ws=RFC6455Protocol)
        self._server = uvicorn.Server(config)
        # our own loop (not uvicorn's asyncio.run) so replicas' receive_asgi_messages pulls and
        # run_asgi_session can schedule onto it from other threads
        loop = asyncio.new_event_loop()
        asyncio.set_event_loop(loop)
        self._loop = loop
        loop.run_until_complete(self._server.serve())

    def ready(self):
        return {"host": self.host, "port": self.port}

    def stats(self) -> Dict:
        """Streaming counters: ``max_pull_bytes`` is the most request bytes this proxy ever held
        for one request at a time (the bound on proxy memory per streamed upload)."""
        return dict(self._stats, open_streams=len(self._streams))

    # ------------------------------------------------------------------ request streams
    async def receive_asgi_messages(self, stream_id: str) -> List[Dict]:
        """Called by the replica's ASGI ``receive()``: the next client messages of a streamed
        request ([] once the stream is over). Runs on the actor's event loop without blocking
        it (the pull itself runs on the HTTP server's loop), so pulls of concurrent requests
        overlap."""
        st = self._streams.get(stream_id)
        if st is None or self._loop is None:
            return []
        msgs = await asyncio.wrap_future(asyncio.run_coroutine_threadsafe(st.pull(), self._loop))
        n = sum(len(m.get("body") or b"") + len(m.get("bytes") or b"") + len(m.get("text") or "") for m in msgs)
        self._stats["pulls"] += 1
        self._stats["streamed_bytes"] += n
        self._stats["max_pull_bytes"] = max(self._stats["max_pull_bytes"], n)
        return msgs

    def _handle(self):
        if self._self_handle is None:
            from ..._private.worker import get_runtime_context

            try:
                self._self_handle = get_runtime_context().current_actor
            except RuntimeError:
                return None  # not running as an actor (an in-process proxy): no streaming
        return self._self_handle

    def _open_stream(self, receive, kind: str):
        h = self._handle()
        if h is None:
            return None, None
        sid = f"{id(self):x}-{next(self._ids)}"
        self._streams[sid] = _RequestStream(receive, kind, self.pull_budget_bytes)
        return sid, {"proxy": h, "id": sid}

    def _close_stream(self, sid):
        if sid is not None:
            st = self._streams.pop(sid, None)
            if st is not None and st.pending is not None and not st.pending.done():
                st.pending.cancel()

    # ------------------------------------------------------------------ routing
    async def _refresh_routes(self, force=False):
        if not force and time.time() - self.last_routes < 1.0:
            return
        from ..api import _get_controller

        self.routes = await _get_controller().list_routes.remote()
        self.last_routes = time.time()

    def _match(self, path):
        best = None
        for prefix, target in self.routes.items():
            p = prefix.rstrip("/")
            if path == p or path.startswith(p + "/") or prefix == "/":
                if best is None or len(prefix) > len(best[0]):
                    best = (prefix, target)
        return best

    async def _route(self, path):
        await self._refresh_routes()
        m = self._match(path)
        if m is None:
            await self._refresh_routes(force=True)
            m = self._match(path)
        return m

    async def _app(self, scope, receive, send):
        self._loop = asyncio.get_running_loop()
        if scope["type"] == "websocket":
            await self._websocket(scope, receive, send)
            return
        if scope["type"] != "http":
            return
        m = await self._route(scope["path"])
        if m is None:
            await _respond(send, 404, b"Path not found")
            return
        prefix, (app_name, ingress) = m
        first = await receive()
        body = first.get("body", b"") if first.get("type") == "http.request" else b""
        sid, stream = (None, None)
        if first.get("type") == "http.request" and first.get("more_body"):
            sid, stream = self._open_stream(receive, "http")
            if stream is None:  # no actor handle to pull through: buffer (in-process proxies only)
                while True:
                    msg = await receive()
                    body += msg.get("body", b"")
                    if not msg.get("more_body"):
                        break
            else:
                self._stats["streamed_requests"] += 1
        root = prefix.rstrip("/")
        sub = scope["path"][len(root):] if root else scope["path"]
        req = {"type": "http", "method": scope["method"], "path": sub or "/",
               "query_string": scope.get("query_string", b""),
               "headers": [(k.decode(), v.decode()) for k, v in scope.get("headers", [])], "body": body,
               "root_path": root}
        if stream is not None:
            req["stream"] = stream
        try:
            await self._forward_http(app_name, ingress, req, send)
        finally:
            self._close_stream(sid)

    async def _forward_http(self, app_name, ingress, req, send):
        from ..exceptions import BackPressureError
        from ..handle import _Router

        started = False
        deadline = None if self.request_timeout_s is None else time.monotonic() + self.request_timeout_s

        def left():
            return None if deadline is None else max(0.0, deadline - time.monotonic())

        try:
            router = _Router.get(app_name, ingress)
            loop = asyncio.get_running_loop()
            fut = await loop.run_in_executor(None, router.submit, None, (req,), {}, {}, "handle_http_stream")
            gen, _ = await asyncio.wait_for(asyncio.wrap_future(fut), left())
            # streamed response: each message is forwarded the moment the replica produces it
            it = gen.__aiter__()
            while True:
                try:
                    ref = await asyncio.wait_for(it.__anext__(), left())
                except StopAsyncIteration:
                    break
                msg = await asyncio.wait_for(ref, left())
                if msg[0] == "start":
                    await send({"type": "http.response.start", "status": msg[1],
                                "headers": [(k.encode(), v.encode()) for k, v in msg[2]]})
                    started = True
                else:
                    await send({"type": "http.response.body", "body": msg[1], "more_body": True})
            await asyncio.wait_for(gen.completed(), left())  # surfaces a replica-side failure
        except asyncio.TimeoutError:
            if not started:
                await _respond(send, 408, f"Request timed out after {self.request_timeout_s}s.".encode())
                return
        except BackPressureError as e:
            if not started:
                await _respond(send, 503, e.message.encode())
                return
        except Exception as e:  # noqa
            if not started:
                await _respond(send, 500, f"Internal Server Error: {e}".encode())
                return
        if not started:
            await _respond(send, 500, b"Internal Server Error: empty response")
            return
        await send({"type": "http.response.body", "body": b"", "more_body": False})

    async def _websocket(self, scope, receive, send):
        """A WebSocket session: every client frame is pulled by the replica's ASGI app through
        ``receive_asgi_messages``; every ``websocket.*`` message it sends comes back over the
        streaming generator and is sent to the client as is."""
        m = await self._route(scope["path"])
        if m is None:
            await send({"type": "websocket.close", "code": 1000})  # rejected handshake (HTTP 403)
            return
        prefix, (app_name, ingress) = m
        sid, stream = self._open_stream(receive, "websocket")
        if stream is None:
            await send({"type": "websocket.close", "code": 1011})
            return
        self._stats["websocket_sessions"] += 1
        root = prefix.rstrip("/")
        sub = scope["path"][len(root):] if root else scope["path"]
        req = {"type": "websocket", "path": sub or "/", "query_string": scope.get("query_string", b""),
               "headers": [(k.decode(), v.decode()) for k, v in scope.get("headers", [])], "body": b"",
               "root_path": root, "subprotocols": list(scope.get("subprotocols") or []), "stream": stream}
        closed = False
        try:
            from ..handle import _Router

            router = _Router.get(app_name, ingress)
            loop = asyncio.get_running_loop()
            fut = await loop.run_in_executor(None, router.submit, None, (req,), {}, {}, "handle_http_stream")
            gen, _ = await asyncio.wrap_future(fut)
            async for ref in gen:
                kind, msg = await ref
                if kind != "ws":
                    continue
                await send(msg)
                if msg.get("type") == "websocket.close":
                    closed = True
            await gen.completed()
        except Exception:  # noqa  (a failed replica ends the session with an internal-error close)
            if not closed:
                await send({"type": "websocket.close", "code": 1011})
                closed = True
        finally:
            self._close_stream(sid)
        if not closed:
            await send({"type": "websocket.close", "code": 1000})

    async def run_asgi_session(self, scope: Dict, messages: List[Dict], timeout_s: float = 60.0) -> List[Dict]:
        """Run ONE ASGI connection through this proxy with a scripted client: ``messages`` are
        what the client's ``receive()`` yields, in order (then it waits, like an idle peer); returns
        every message the proxy sent to the client. The same path uvicorn drives (used to exercise
        WebSocket sessions where no WebSocket server library is installed)."""
        if self._loop is None:
            raise RuntimeError("proxy event loop not started")
        script = list(messages)
        sent: List[Dict] = []

        async def receive():
            if script:
                return script.pop(0)
            await asyncio.sleep(3600)

        async def send(msg):
            sent.append(msg)

        await asyncio.wrap_future(asyncio.run_coroutine_threadsafe(
            asyncio.wait_for(self._app(dict(scope), receive, send), timeout_s), self._loop))
        return sent

    def shutdown(self):
        if self._server is not None:
            self._server.should_exit = True
        return True


async def _respond(send, status, body):
    await send({"type": "http.response.start", "status": status, "headers": [(b"content-type", b"text/plain")]})
    await send({"type": "http.response.body", "body": body})
