"""Dashboard HTTP server (reference: ``dashboard/`` -- the web UI is out of scope): the cluster-wide
Prometheus exposition at ``/metrics``, JSON state at ``/api/*`` backed by the head's state RPCs, and
the job REST API of ``dashboard/modules/job/job_head.py`` (``/api/jobs/``) on the session's
JobManager actor, which ``JobSubmissionClient("http://host:port")`` speaks. Started by
``init(include_dashboard=True, dashboard_port=...)``.

Per-node agents (reference ``dashboard/agent.py`` + ``modules/reporter`` / ``modules/log``): the
dashboard supervises one ``dashboard_agent`` process per alive node (``_AgentSupervisor``), which
reports that node's and its workers' stats through the head KV and serves that node's logs.
``/nodes?view=summary``, ``/nodes/<node_id>``, ``/api/v0/logs[/file]?node_id=`` and the
``ray_component_*`` / ``ray_node_agent_*`` lines of ``/metrics`` come from them.
``RCA_DASHBOARD_AGENTS=0`` turns the agents off."""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading
import time
import urllib.error
import urllib.request
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
                        text = dash._call("metrics_text")
                        if dash.agents is not None:
                            text = text.rstrip("\n") + "\n" + "\n".join(dash.agents.prometheus_lines()) + "\n"
                        return self._send(200, text, "text/plain; version=0.0.4")
                    if path == "/nodes" or path.startswith("/nodes/"):
                        code, body = dash._nodes_route(path.split("/")[2:], query)
                        return self._send(code, json.dumps(body, default=str), "application/json")
                    if path in ("/api/v0/logs", "/api/v0/logs/file") and query.get("node_id"):
                        code, body, ctype = dash._agent_log_route(path.endswith("/file"), query)
                        return self._send(code, body, ctype)
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
        self.agents = None
        if os.environ.get("RCA_DASHBOARD_AGENTS", "1") != "0" and getattr(head, "sock_path", None):
            self.agents = _AgentSupervisor(self, head.sock_path, getattr(head, "logs_dir", None),
                                           float(os.environ.get("RCA_DASHBOARD_AGENT_PERIOD_S", "1.0")))

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
        if self.agents is not None:
            self.agents.stop()
        self.server.shutdown()
        self.server.server_close()

    # ------------------------------------------------------------------ per-node agents
    def _nodes_route(self, rest, query):
        """``GET /nodes?view=summary`` and ``GET /nodes/<node_id>`` (reference
        ``modules/node/node_head.py`` get_all_nodes / get_node), in the reference envelope."""
        reports = self.agents.reports() if self.agents is not None else {}
        nodes = {n["NodeID"]: n for n in self._call("nodes")}

        def summary(nid, n):
            rep = reports.get(nid) or {}
            node = rep.get("node") or {}
            return {"raylet": {"nodeId": nid, "state": "ALIVE" if n.get("Alive") else "DEAD",
                               "isHeadNode": n.get("IsHead"), "resources": n.get("Resources"),
                               "labels": n.get("Labels")},
                    "hostname": rep.get("hostname"), "ip": n.get("NodeManagerAddress"),
                    "cpu": node.get("cpu_percent"), "cpus": [node.get("cpu_count"), node.get("cpu_count")],
                    "mem": [node.get("mem_total"), node.get("mem_available"),
                            (100.0 * node["mem_used"] / node["mem_total"]) if node.get("mem_total") else None,
                            node.get("mem_used")],
                    "disk": {"/tmp": {"total": node.get("disk_total"), "used": node.get("disk_used")}},
                    "gpus": rep.get("gpus", []), "numWorkers": rep.get("num_workers"),
                    "agent": {"pid": rep.get("agent_pid"), "http": rep.get("agent_http"),
                              "reportTime": rep.get("timestamp"), "reports": rep.get("reports")}}

        if not rest:
            view = (query.get("view") or ["summary"])[0]
            if view not in ("summary", "hostnamelist"):
                return 400, {"result": False, "msg": f"unknown view {view!r}", "data": {}}
            if view == "hostnamelist":
                hosts = sorted({(reports.get(nid) or {}).get("hostname") for nid in nodes} - {None})
                return 200, {"result": True, "msg": "", "data": {"hostNameList": hosts}}
            return 200, {"result": True, "msg": "Node summary fetched.",
                         "data": {"summary": [summary(nid, n) for nid, n in nodes.items()]}}
        nid = rest[0]
        if nid not in nodes:
            return 404, {"result": False, "msg": f"node {nid} not found", "data": {}}
        detail = summary(nid, nodes[nid])
        detail["workers"] = (reports.get(nid) or {}).get("workers", [])
        return 200, {"result": True, "msg": "Node details fetched.", "data": {"detail": detail}}

    def _agent_log_route(self, is_file, query):
        """``/api/v0/logs?node_id=`` and ``/api/v0/logs/file?node_id=&filename=&lines=``: answered
        by that node's agent (reference ``modules/log/log_manager.py`` -> the node's LogAgent)."""
        nid = query["node_id"][0]
        rep = (self.agents.reports() if self.agents is not None else {}).get(nid)
        if not rep or not rep.get("agent_http"):
            return 503, json.dumps({"result": False, "msg": f"no agent is reporting for node {nid}"}), \
                "application/json"
        base = rep["agent_http"]
        try:
            if is_file:
                name = (query.get("filename") or [""])[0]
                lines = int((query.get("lines") or ["-1"])[0])
                url = f"{base}/logs/{urllib.request.quote(os.path.basename(name))}?lines={lines}"
                with urllib.request.urlopen(url, timeout=10) as r:
                    return 200, r.read(), "text/plain; charset=utf-8"
            with urllib.request.urlopen(f"{base}/logs", timeout=10) as r:
                names = json.loads(r.read())
            return 200, json.dumps({"result": True, "msg": "", "data": {"result": {nid: names}}}), "application/json"
        except urllib.error.HTTPError as e:
            return e.code, e.read(), "application/json"


class _AgentSupervisor:
    """Keeps one ``dashboard_agent`` process per alive node: starts one for a node that has none
    (or whose agent exited: restarted, counted in ``restarts``), stops the agent of a removed
    node, stops them all with the dashboard. Reports are read back from the head KV."""

    def __init__(self, dash, sock_path, logs_dir, period_s=1.0):
        self.dash, self.sock_path, self.logs_dir, self.period_s = dash, sock_path, logs_dir, period_s
        self.procs = {}
        self.restarts = 0
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, daemon=True, name="rca-agent-supervisor")
        self._thread.start()

    def _spawn(self, nid):
        pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        cmd = [sys.executable, "-m", "ray_community_amd._private.dashboard_agent", "--sock", self.sock_path,
               "--node-id", nid, "--period", str(self.period_s), "--parent-pid", str(os.getpid())]
        out = subprocess.DEVNULL
        if self.logs_dir and os.path.isdir(self.logs_dir):
            out = open(os.path.join(self.logs_dir, f"dashboard_agent_{nid[:8]}.log"), "ab")
        try:
            return subprocess.Popen(cmd, env=env, stdout=out, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                    start_new_session=True)
        finally:
            if out is not subprocess.DEVNULL:
                out.close()

    def sync(self):
        alive = {n["NodeID"] for n in self.dash._call("nodes") if n.get("Alive")}
        with self._lock:
            if self._stop.is_set():
                return
            for nid in list(self.procs):
                if nid not in alive:
                    self._terminate(self.procs.pop(nid))
                    self._forget(nid)
            for nid in alive:
                p = self.procs.get(nid)
                if p is not None and p.poll() is not None:
                    self.restarts += 1
                    p = None
                if p is None:
                    self.procs[nid] = self._spawn(nid)

    def _loop(self):
        while not self._stop.is_set():
            try:
                self.sync()
            except Exception:  # noqa - head shutting down: the next period (or stop) decides
                pass
            self._stop.wait(max(self.period_s, 0.5))

    def _forget(self, nid):
        from .dashboard_agent import AGENT_NAMESPACE, agent_key

        try:
            self.dash._call("kv_del", agent_key(nid), AGENT_NAMESPACE)
        except Exception:  # noqa
            pass

    @staticmethod
    def _terminate(p):
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait(5)

    def stop(self):
        self._stop.set()
        with self._lock:
            procs, self.procs = list(self.procs.values()), {}
        for p in procs:
            self._terminate(p)

    def reports(self):
        from .dashboard_agent import AGENT_NAMESPACE

        out = {}
        for key in self.dash._call("kv_keys", "node:", AGENT_NAMESPACE) or []:
            k = key.decode() if isinstance(key, bytes) else key
            raw = self.dash._call("kv_get", k, AGENT_NAMESPACE)
            if raw:
                try:
                    out[k[len("node:"):]] = json.loads(raw)
                except ValueError:
                    pass
        return out

    def prometheus_lines(self):
        """Per-node agent metrics (reference reporter_agent METRICS_GAUGES ``ray_component_*``):
        labelled by NodeId, and by Component (worker id prefix) and pid for worker processes."""
        reports = self.reports()
        now = time.time()
        gauges = {"ray_node_agent_up": ("1 while the node's dashboard agent reports (age < 5 periods)", []),
                  "ray_node_agent_report_age_seconds": ("seconds since the node agent's last report", []),
                  "ray_node_num_workers": ("alive worker processes on the node", []),
                  "ray_component_cpu_percentage": ("CPU percent of a worker process", []),
                  "ray_component_rss_mb": ("resident set size of a worker process, MB", []),
                  "ray_component_uss_mb": ("unique set size of a worker process, MB", []),
                  "ray_component_num_threads": ("threads of a worker process", [])}
        for nid, rep in sorted(reports.items()):
            lab = f'NodeId="{nid}"'
            age = now - float(rep.get("timestamp") or 0)
            gauges["ray_node_agent_up"][1].append((lab, 1 if age < 5 * max(self.period_s, 1.0) else 0))
            gauges["ray_node_agent_report_age_seconds"][1].append((lab, round(age, 3)))
            gauges["ray_node_num_workers"][1].append((lab, rep.get("num_workers", 0)))
            for w in rep.get("workers", []):
                wl = f'{lab},Component="worker-{(w.get("worker_id") or "")[:8]}",pid="{w.get("pid")}"'
                gauges["ray_component_cpu_percentage"][1].append((wl, w.get("cpu_percent")))
                gauges["ray_component_rss_mb"][1].append((wl, (w.get("rss") or 0) / 1e6))
                if w.get("uss") is not None:
                    gauges["ray_component_uss_mb"][1].append((wl, w["uss"] / 1e6))
                gauges["ray_component_num_threads"][1].append((wl, w.get("num_threads")))
        lines = []
        for name, (help_, samples) in gauges.items():
            samples = [(l, v) for l, v in samples if v is not None]
            if not samples:
                continue
            lines += [f"# HELP {name} {help_}", f"# TYPE {name} gauge"]
            lines += [f"{name}{{{l}}} {v}" for l, v in samples]
        return lines


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
