"""Minimal dashboard HTTP server (reference: ``dashboard/`` — the web UI is out of scope): serves
the cluster-wide Prometheus exposition at ``/metrics`` and JSON state at ``/api/*``, backed by the
head's state RPCs. Started by ``init(include_dashboard=True, dashboard_port=...)``."""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class Dashboard:
    def __init__(self, head, host: str = "127.0.0.1", port: int = 8265):
        from .core_worker import DirectClient

        self.client = DirectClient(head)
        self.client.key = "dashboard"
        dash = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body, ctype):
                data = body.encode() if isinstance(body, str) else body
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                try:
                    path = self.path.split("?")[0].rstrip("/")
                    if path == "/metrics":
                        return self._send(200, dash._call("metrics_text"), "text/plain; version=0.0.4")
                    routes = {"/api/version": lambda: {"version": _version(), "ray_compatible": "3.0.0.dev0"},
                              "/api/cluster_status": lambda: {"total": dash._call("cluster_resources"),
                                                              "available": dash._call("available_resources")},
                              "/api/nodes": lambda: dash._call("nodes"),
                              "/api/actors": lambda: dash._call("list_actors"),
                              "/api/tasks": lambda: dash._call("list_tasks", 1000),
                              "/api/objects": lambda: dash._call("list_objects"),
                              "/api/workers": lambda: dash._call("list_workers"),
                              "/api/object_store": lambda: dash._call("store_stats"),
                              "/api/timeline": lambda: dash._call("timeline")}
                    if path in routes:
                        return self._send(200, json.dumps(routes[path](), default=str), "application/json")
                    return self._send(404, "not found", "text/plain")
                except Exception as e:  # noqa
                    return self._send(500, f"error: {e}", "text/plain")

        self.server = ThreadingHTTPServer((host, port), Handler)
        self.host, self.port = host, self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True, name="rca-dashboard")
        self.thread.start()

    def _call(self, method, *args):
        return self.client.call(method, *args)

    @property
    def url(self):
        return f"http://{self.host}:{self.port}"

    def stop(self):
        self.server.shutdown()
        self.server.server_close()


def _version():
    from .. import __version__

    return __version__
