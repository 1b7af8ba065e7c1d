"""Dashboard HTTP server (reference: ``dashboard/`` -- the web UI is out of scope): the cluster-wide
Prometheus exposition at ``/metrics``, JSON state at ``/api/*`` backed by the head's state RPCs, and
the job REST API of ``dashboard/modules/job/job_head.py`` (``/api/jobs/``) on the session's
JobManager actor, which ``JobSubmissionClient("http://host:port")`` speaks. Started by
``init(include_dashboard=True, dashboard_port=...)``."""
from __future__ import annotations

import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, urlparse


class Dashboard:
    def __init__(self, head, host: str = "127.0.0.1", port: int = 8265):
        from .core_worker import DirectClient

        self.client = DirectClient(head)
        self.client.key = "dashboard"
        self._serve_lock = threading.Lock()
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

            def _serve(self, method):
                """Serve applications REST API: returns True if the path was a serve route."""
                u = urlparse(self.path)
                parts = [p for p in u.path.split("/") if p]
                if parts[:3] != ["api", "serve", "applications"]:
                    return False
                try:
                    body = self._body() if method == "PUT" else None
                    self._json(*dash._serve_route(method, body))
                except Exception as e:  # noqa
                    self._json(500, {"error": f"{type(e).__name__}: {e}"})
                return True

            def do_PUT(self):
                if not self._serve("PUT"):
                    self._send(404, "not found", "text/plain")

            def do_POST(self):
                if not self._jobs("POST"):
                    self._send(404, "not found", "text/plain")

            def do_DELETE(self):
                if not self._jobs("DELETE") and not self._serve("DELETE"):
                    self._send(404, "not found", "text/plain")

            def do_GET(self):
                try:
                    if self._jobs("GET") or self._serve("GET"):
                        return
                    path = self.path.split("?")[0].rstrip("/")
                    query = parse_qs(urlparse(self.path).query)
                    if path in ("", "/index.html"):
                        return self._send(200, _INDEX_HTML, "text/html; charset=utf-8")
                    if path == "/api/logs/file":
                        lines = dash._call("get_log", (query.get("filename") or [None])[0], None, None, None, None,
                                           int((query.get("lines") or ["-1"])[0]))
                        return self._send(200, "\n".join(lines), "text/plain; charset=utf-8")
                    if path == "/metrics":
                        return self._send(200, dash._call("metrics_text"), "text/plain; version=0.0.4")
                    if path.startswith("/api/v0/"):
                        code, body = dash._state_route(path[len("/api/v0/"):].split("/"), query)
                        return self._send(code, json.dumps(body, default=str), "application/json")
                    routes = {"/api/version": lambda: {"version": _version(), "ray_compatible": "3.0.0.dev0"},
                              "/api/cluster_status": lambda: {"total": dash._call("cluster_resources"),
                                                              "available": dash._call("available_resources")},
                              "/api/nodes": lambda: dash._call("nodes"),
                              "/api/actors": lambda: dash._call("list_actors"),
                              "/api/tasks": lambda: dash._call("list_tasks", 1000),
                              "/api/objects": lambda: dash._call("list_objects"),
                              "/api/workers": lambda: dash._call("list_workers"),
                              "/api/object_store": lambda: dash._call("store_stats"),
                              "/api/timeline": lambda: dash._call("timeline"),
                              "/api/logs": lambda: dash._call("list_logs", None, None),
                              "/api/cluster_events": lambda: dash._call("cluster_events"),
                              "/api/placement_groups": lambda: list(dash._call("pg_table", None).values())}
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

    def _state_route(self, parts, query):
        """Reference state-API HTTP protocol (``dashboard/modules/state/state_head.py``):
        ``GET /api/v0/<resource>?limit=&detail=&filter_keys=&filter_predicates=&filter_values=`` and
        ``GET /api/v0/<tasks|actors|objects>/summarize``, answered in the reference envelope."""
        from ..util import state as st

        def env(ok, msg, data):
            return (200 if ok else 400), {"result": ok, "msg": msg, "data": data}

        res = parts[0] if parts else ""
        try:
            with st._using_client(self.client):
                if len(parts) == 2 and parts[1] == "summarize" and res in ("tasks", "actors", "objects"):
                    summary = getattr(st, f"summarize_{res}")()
                    return env(True, "", {"result": {"node_id_to_summary": summary}})
                if len(parts) != 1 or res not in st._RESOURCES:
                    return 404, {"result": False, "msg": f"unknown state resource {'/'.join(parts)!r}", "data": {}}
                keys = query.get("filter_keys", [])
                preds = query.get("filter_predicates", [])
                vals = query.get("filter_values", [])
                if not (len(keys) == len(preds) == len(vals)):
                    return env(False, "filter_keys, filter_predicates and filter_values must have equal lengths", {})
                filters = list(zip(keys, preds, vals))
                limit = int((query.get("limit") or ["100"])[0])
                rows = getattr(st, f"list_{res}")(filters=None)
                total = len(rows)
                rows = st._filter(rows, filters)
                out = rows[:limit]
                return env(True, "", {"result": {"total": total, "num_after_truncation": len(out),
                                                 "num_filtered": len(rows), "result": out,
                                                 "partial_failure_warning": "", "warnings": None}})
        except ValueError as e:
            return env(False, str(e), {})

    def _job_route(self, method, rest, body, query):
        """(status, json) for one job REST call."""
        from .. import job_submission as js
        from .worker import get

        mgr = js._job_manager()
        if method == "POST" and not rest:
            from ..runtime_env import validate

            res = {k: body.get(k) for k in ("entrypoint_num_cpus", "entrypoint_num_gpus", "entrypoint_resources",
                                            "entrypoint_memory")}
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

    def _serve_route(self, method, body):
        """(status, json) for ``/api/serve/applications/`` (reference:
        ``dashboard/modules/serve/serve_rest_api_impl.py``): GET the instance details, PUT a
        ``ServeDeploySchema`` (declarative: apps missing from it are deleted), DELETE = shutdown."""
        from ..serve import api as sapi
        from ..serve._private.controller import CONTROLLER_NAME, NAMESPACE
        from .worker import get, get_actor

        with self._serve_lock:
            sapi._STATE["controller"] = None  # another driver (the CLI) may have restarted Serve
            sapi._STATE["proxy"] = None
            try:
                ctrl = get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
            except ValueError:
                ctrl = None
            if method == "GET":
                empty = {"controller_info": None, "proxy_location": None, "http_options": None,
                         "grpc_options": None, "proxies": {}, "deploy_mode": "UNSET", "applications": {},
                         "target_capacity": None}
                if ctrl is None:
                    return 200, empty
                from .. import exceptions as rexc

                try:
                    return 200, get(ctrl.get_serve_instance_details.remote())
                except rexc.RayActorError:  # the controller is being shut down (DELETE just ran)
                    return 200, empty
            if method == "DELETE":
                if ctrl is not None:
                    sapi.shutdown()
                return 200, {}
            if method == "PUT":
                from pydantic import ValidationError

                from ..serve._private.config_deploy import deploy_config
                from ..serve.schema import ServeDeploySchema

                try:
                    cfg = ServeDeploySchema.model_validate(body or {})
                except ValidationError as e:
                    return 400, {"error": str(e)}
                try:
                    return 200, {"applications": deploy_config(cfg)}
                except Exception as e:  # noqa  (build / deploy errors are the caller's config)
                    return 400, {"error": f"{type(e).__name__}: {getattr(e, 'cause', None) or e}"}
            return 405, {"error": "method not allowed"}

    @property
    def url(self):
        return f"http://{self.host}:{self.port}"

    def stop(self):
        self.server.shutdown()
        self.server.server_close()


def _version():
    from .. import __version__

    return __version__


# One self-contained overview page (reference: the dashboard's React client, dashboard/client/):
# cluster resources, nodes, actors, recent tasks, workers, jobs, events and worker logs, refreshed
# from the /api/* routes above every two seconds.
_INDEX_HTML = """<!doctype html><html><head><meta charset="utf-8"><title>ray_community_amd dashboard</title>
<style>body{font:13px sans-serif;margin:16px;color:#222}h2{margin:18px 0 6px;font-size:15px}
table{border-collapse:collapse;width:100%}td,th{border:1px solid #ddd;padding:3px 6px;text-align:left;
vertical-align:top}th{background:#f3f3f3}pre{background:#f7f7f7;padding:8px;max-height:300px;overflow:auto}
.bar{display:flex;gap:24px}.k{color:#666}</style></head><body>
<h1>ray_community_amd</h1><div class="bar" id="res"></div>
<h2>Nodes</h2><div id="nodes"></div><h2>Actors</h2><div id="actors"></div>
<h2>Recent tasks</h2><div id="tasks"></div><h2>Workers</h2><div id="workers"></div>
<h2>Jobs</h2><div id="jobs"></div><h2>Cluster events</h2><div id="events"></div>
<h2>Logs</h2><div id="logs"></div><pre id="logview"></pre>
<script>
function esc(v){return String(v===null||v===undefined?"":(typeof v==="object"?JSON.stringify(v):v))
 .replace(/[&<>]/g,c=>({"&":"&amp;","<":"&lt;",">":"&gt;"}[c]))}
function table(rows,cols){if(!rows||!rows.length)return "<i>none</i>";
 return "<table><tr>"+cols.map(c=>"<th>"+c+"</th>").join("")+"</tr>"+rows.map(r=>"<tr>"+cols.map(
 c=>"<td>"+esc(r[c])+"</td>").join("")+"</tr>").join("")+"</table>"}
async function j(u){const r=await fetch(u);return r.ok?r.json():null}
async function showLog(f){const r=await fetch("/api/logs/file?lines=200&filename="+encodeURIComponent(f));
 document.getElementById("logview").textContent=await r.text()}
async function refresh(){
 const cs=await j("/api/cluster_status");if(cs){document.getElementById("res").innerHTML=Object.keys(cs.total)
  .filter(k=>!k.startsWith("node:")).map(k=>"<div><span class=k>"+esc(k)+"</span> "+esc(cs.available[k]||0)+" / "
  +esc(cs.total[k])+"</div>").join("")}
 document.getElementById("nodes").innerHTML=table(await j("/api/nodes"),["NodeID","Alive","IsHead","Resources"]);
 document.getElementById("actors").innerHTML=table(await j("/api/actors"),["actor_id","class_name","state","name",
  "pid","num_restarts","death_cause"]);
 const t=(await j("/api/tasks"))||[];document.getElementById("tasks").innerHTML=table(t.slice(-50).reverse(),
  ["task_id","name","state","type","worker_id","error_type"]);
 document.getElementById("workers").innerHTML=table(await j("/api/workers"),["worker_id","pid","state","is_actor",
  "gpu_ids","log_file"]);
 document.getElementById("jobs").innerHTML=table(await j("/api/jobs/"),["submission_id","status","entrypoint",
  "message"]);
 const ev=(await j("/api/cluster_events"))||[];document.getElementById("events").innerHTML=table(ev.slice(-30)
  .reverse(),["severity","source_type","message"]);
 const lg=(await j("/api/logs"))||{};document.getElementById("logs").innerHTML=Object.values(lg).flat().map(
  f=>"<a href='#' onclick='showLog(\\""+esc(f)+"\\");return false'>"+esc(f)+"</a>").join(" &middot; ")}
refresh();setInterval(refresh,2000);
</script></body></html>"""
