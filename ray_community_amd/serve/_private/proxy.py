"""HTTP proxy actor (reference: ``serve/_private/proxy.py``): a uvicorn ASGI server that matches
the longest route prefix, then forwards the request to the application's ingress deployment
through a DeploymentHandle (power-of-two-choices routing)."""
from __future__ import annotations

import asyncio
import threading
import time
from typing import Dict, Optional


class HTTPProxy:
    def __init__(self, host: str = "127.0.0.1", port: int = 8000, request_timeout_s: Optional[float] = None,
                 keep_alive_timeout_s: int = 5, root_path: str = ""):
        self.host = host
        self.port = port
        self.keep_alive_timeout_s = int(keep_alive_timeout_s)
        self.root_path = root_path or ""
        # end-to-end request timeout (HTTPOptions.request_timeout_s): 408 if no response started
        self.request_timeout_s = request_timeout_s if request_timeout_s and request_timeout_s > 0 else None
        self.routes: Dict[str, tuple] = {}
        self.last_routes = 0.0
        self._server = None
        self._thread = threading.Thread(target=self._run, daemon=True)
        self._thread.start()
        deadline = time.time() + 15
        while self._server is None or not getattr(self._server, "started", False):
            if time.time() > deadline:
                raise RuntimeError("HTTP proxy failed to start")
            time.sleep(0.02)

    def _run(self):
        import uvicorn

        config = uvicorn.Config(self._app, host=self.host, port=self.port, log_level="warning", lifespan="off",
                                interface="asgi3", timeout_keep_alive=self.keep_alive_timeout_s,
                                root_path=self.root_path)
        self._server = uvicorn.Server(config)
        self._server.run()

    def ready(self):
        return {"host": self.host, "port": self.port}

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

    async def _app(self, scope, receive, send):
        if scope["type"] != "http":
            return
        await self._refresh_routes()
        m = self._match(scope["path"])
        if m is None:
            await self._refresh_routes(force=True)
            m = self._match(scope["path"])
        if m is None:
            await _respond(send, 404, b"Path not found")
            return
        prefix, (app_name, ingress) = m
        body = b""
        while True:
            msg = await receive()
            body += msg.get("body", b"")
            if not msg.get("more_body"):
                break
        root = prefix.rstrip("/")
        sub = scope["path"][len(root):] if root else scope["path"]
        req = {"method": scope["method"], "path": sub or "/", "query_string": scope.get("query_string", b""),
               "headers": [(k.decode(), v.decode()) for k, v in scope.get("headers", [])], "body": body,
               "root_path": root}
        from ..handle import _Router

        from ..exceptions import BackPressureError

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

    def shutdown(self):
        if self._server is not None:
            self._server.should_exit = True
        return True


async def _respond(send, status, body):
    await send({"type": "http.response.start", "status": status, "headers": [(b"content-type", b"text/plain")]})
    await send({"type": "http.response.body", "body": body})
