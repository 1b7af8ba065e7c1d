"""Dashboard HTTP server (reference: ``dashboard/`` -- the web UI is out of scope): the cluster-wide
Prometheus exposition at ``/metrics``, JSON state at ``/api/*`` backed by the head's state RPCs, and
the job REST API of ``dashboard/modules/job/job_head.py`` (``/api/jobs/``) on the session's
JobManager actor, which ``JobSubmissionClient("http://host:port")`` speaks. Started by
``init(include_dashboard=True, dashboard_port=...)``."""
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

            def _json(self, code, obj):
                return self._send(code, json.dumps(obj, default=str), "application/json")

            def _body(self):
                n = int(self.headers.get("Content-Length") or 0)
                return json.loads(self.rfile.read(n) or b"{}") if n else {}

            def _jobs(self, method):
                """Job REST API: returns True if the path was a job route."""
                from urllib.parse import parse_qs, urlparse

                u = urlparse(self.path)
                parts = [p for p in u.path.split("/") if p]
                if parts[:2] != ["api", "jobs"]:
                    return False
                try:
                    out = dash._job_route(method, parts[2:], self._body() if method == "POST" else {},
                                          parse_qs(u.query))
                    self._json(*out)
                except Exception as e:  # noqa
                    self._json(500, {"error": f"{type(e).__name__}: {e}"})
                return True

            def do_POST(self):
                if not self._jobs("POST"):
                    self._send(404, "not found", "text/plain")

            def do_DELETE(self):
                if not self._jobs("DELETE"):
                    self._send(404, "not found", "text/plain")

            def do_GET(self):
                try:
                    if self._jobs("GET"):
                        return
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

    def _job_route(self, method, rest, body, query):
        """(status, json) for one job REST call."""
        from .. import job_submission as js
        from .worker import get

        mgr = js._job_manager()
        if method == "POST" and not rest:
            from ..runtime_env import validate

            res = {k: body.get(k) for k in ("entrypoint_num_cpus", "entrypoint_num_gpus", "entrypoint_resources")}
            try:
                sid = get(mgr.submit.remote(body["entrypoint"], body.get("submission_id") or body.get("job_id"),
                                            validate(body.get("runtime_env")), body.get("metadata"), res))
            except Exception as e:  # noqa
                return 400, {"error": str(getattr(e, "cause", None) or e)}
            return 200, {"submission_id": sid, "job_id": sid}
        if method == "GET" and not rest:
            return 200, [js._jsonable_job(d) for d in get(mgr.list.remote())]
        if not rest:
            return 405, {"error": "method not allowed"}
        sid = rest[0]
        info = get(mgr.info.remote(sid))
        if info is None:
            return 404, {"error": f"Job {sid} does not exist."}
        if method == "GET" and len(rest) == 1:
            return 200, js._jsonable_job(info)
        if method == "GET" and rest[1:] == ["logs"]:
            off = int((query.get("offset") or ["0"])[0])
            return 200, {"logs": get(mgr.logs.remote(sid, off)) or ""}
        if method == "POST" and rest[1:] == ["stop"]:
            return 200, {"stopped": bool(get(mgr.stop.remote(sid)))}
        if method == "DELETE" and len(rest) == 1:
            try:
                return 200, {"deleted": bool(get(mgr.delete.remote(sid)))}
            except Exception as e:  # noqa
                return 400, {"error": str(getattr(e, "cause", None) or e)}
        return 404, {"error": "unknown job route"}

    @property
    def url(self):
        return f"http://{self.host}:{self.port}"

    def stop(self):
        self.server.shutdown()
        self.server.server_close()


def _version():
    from .. import __version__

    return __version__
