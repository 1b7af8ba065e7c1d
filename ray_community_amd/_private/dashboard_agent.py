"""Per-node dashboard agent: reporter + log agent of one node (reference:
``python/ray/dashboard/agent.py`` DashboardAgent, ``modules/reporter/reporter_agent.py``
ReporterAgent._collect_stats / _generate_reseted_stats_records and ``modules/log/log_agent.py``
LogAgentV1Grpc.ListLogs / StreamLog).

One process per node, started and stopped by the dashboard's supervisor (``dashboard.py``
``_AgentSupervisor``), run as ``python -m ray_community_amd._private.dashboard_agent``. It never
imports torch or opens the GPU. Every ``--period`` seconds it:

  * reads node CPU / memory / disk (psutil) and the node's AMD GPUs from sysfs (no ``amd-smi``
    fork, no HIP context; ``node_telemetry.read_gpus``);
  * reads the processes of the workers the head placed on THIS node (``list_workers`` filtered by
    ``node_id``): CPU %, RSS / USS, threads, open files -- the reference's per-component stats;
  * publishes the report as JSON to the head KV (namespace ``dashboard_agent``, key
    ``node:<node_id>``), where the dashboard reads it for ``/nodes`` and ``/metrics``.

It also serves its node's worker logs over HTTP (``GET /logs``, ``GET /logs/<file>?lines=N``), so
the dashboard's log route is answered by the agent of the node that holds the file, as in the
reference, instead of the head reading every node's files. The agent exits when its head
connection drops or its parent (the dashboard's process) is gone.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional
from urllib.parse import parse_qs, urlparse

AGENT_NAMESPACE = "dashboard_agent"


def agent_key(node_id: str) -> str:
    return f"node:{node_id}"


class _ProcStats:
    """psutil.Process handles kept across periods: ``cpu_percent`` is the delta since the previous
    call on the SAME handle, so a fresh handle each period would always read 0."""

    def __init__(self):
        self._procs: Dict[int, object] = {}

    def read(self, workers: List[Dict]) -> List[Dict]:
        try:
            import psutil
        except ImportError:
            return []
        out, seen = [], set()
        for w in workers:
            pid = w.get("pid")
            if not pid or pid <= 0:
                continue
            seen.add(pid)
            p = self._procs.get(pid)
            try:
                if p is None:
                    p = self._procs[pid] = psutil.Process(pid)
                    p.cpu_percent(None)  # prime the delta
                with p.oneshot():
                    mem = p.memory_info()
                    rec = {"pid": pid, "worker_id": w.get("worker_id"), "is_actor": w.get("is_actor"),
                           "state": w.get("state"), "cpu_percent": p.cpu_percent(None),
                           "rss": mem.rss, "vms": mem.vms, "num_threads": p.num_threads(),
                           "create_time": p.create_time(), "cmdline": " ".join(p.cmdline()[:4])}
                try:
                    rec["uss"] = p.memory_full_info().uss
                except Exception:  # noqa - /proc/<pid>/smaps not readable here
                    rec["uss"] = None
                try:
                    rec["num_fds"] = p.num_fds()
                except Exception:  # noqa
                    rec["num_fds"] = None
                out.append(rec)
            except Exception:  # noqa - exited between list_workers and now
                self._procs.pop(pid, None)
        for pid in [pid for pid in self._procs if pid not in seen]:
            self._procs.pop(pid, None)
        return out


class DashboardAgent:
    def __init__(self, sock_path: str, node_id: str, period_s: float = 1.0, parent_pid: Optional[int] = None,
                 host: str = "127.0.0.1"):
        from .core_worker import SocketClient

        self.node_id = node_id
        self.period_s = period_s
        self.parent_pid = parent_pid
        self._stop = threading.Event()
        self.client = SocketClient(sock_path, "client", os.urandom(16), on_message=self._on_message)
        hello = self.client.hello or {}
        self.session_dir = hello.get("session_dir") or ""
        self.logs_dir = os.path.join(self.session_dir, "logs")
        self._procs = _ProcStats()
        self._reports = 0
        agent = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _send(self, code, body, ctype="application/json"):
                data = body.encode() if isinstance(body, str) else body
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            def do_GET(self):
                u = urlparse(self.path)
                parts = [p for p in u.path.split("/") if p]
                q = parse_qs(u.query)
                try:
                    if parts == ["logs"]:
                        return self._send(200, json.dumps(agent.list_logs()))
                    if len(parts) == 2 and parts[0] == "logs":
                        lines = int((q.get("lines") or ["-1"])[0])
                        text = agent.read_log(parts[1], lines)
                        if text is None:
                            return self._send(404, json.dumps({"error": f"{parts[1]} is not a log of node "
                                                                        f"{agent.node_id}"}))
                        return self._send(200, text, "text/plain; charset=utf-8")
                    if parts == ["stats"]:
                        return self._send(200, json.dumps(agent.last_report, default=str))
                    return self._send(404, json.dumps({"error": "not found"}))
                except Exception as e:  # noqa
                    return self._send(500, json.dumps({"error": f"{type(e).__name__}: {e}"}))

        self.server = ThreadingHTTPServer((host, 0), Handler)
        self.host, self.port = host, self.server.server_address[1]
        self.last_report: Dict = {}

    # ------------------------------------------------------------------ head link
    def _on_message(self, msg):
        from . import protocol as P

        if msg and msg[0] == P.EXIT:
            self._stop.set()

    def _parent_alive(self) -> bool:
        if self.parent_pid is None:
            return True
        try:
            os.kill(self.parent_pid, 0)
            return True
        except ProcessLookupError:
            return False
        except PermissionError:
            return True

    # ------------------------------------------------------------------ logs
    def list_logs(self) -> List[str]:
        names = (self.client.call("list_logs", self.node_id, None) or {}).get(self.node_id, [])
        return [n for n in names if os.path.exists(os.path.join(self.logs_dir, n))]

    def read_log(self, name: str, lines: int = -1) -> Optional[str]:
        name = os.path.basename(name)
        if name not in self.list_logs():
            return None
        path = os.path.join(self.logs_dir, name)
        with open(path, "rb") as f:
            if lines is None or lines < 0:
                data = f.read()
            else:  # tail: read backwards in blocks until enough newlines are held
                f.seek(0, os.SEEK_END)
                pos = f.tell()
                data = b""
                while pos > 0 and data.count(b"\n") <= lines:
                    step = min(65536, pos)
                    pos -= step
                    f.seek(pos)
                    data = f.read(step) + data
                data = b"\n".join(data.splitlines()[-lines:] if lines else [])
        return data.decode("utf-8", "replace")

    # ------------------------------------------------------------------ reporter
    def collect(self) -> Dict:
        from .node_telemetry import read_gpus, read_node

        workers = [w for w in (self.client.call("list_workers") or [])
                   if w.get("node_id") == self.node_id and w.get("is_alive")]
        try:
            gpus = read_gpus(allow_amd_smi=False)
        except Exception:  # noqa - sysfs hidden: no GPU section
            gpus = []
        procs = self._procs.read(workers)
        rep = {"node_id": self.node_id, "hostname": socket.gethostname(), "agent_pid": os.getpid(),
               "agent_http": f"http://{self.host}:{self.port}", "timestamp": time.time(),
               "node": read_node(), "gpus": gpus, "workers": procs, "num_workers": len(workers),
               "reports": self._reports + 1}
        rep["workers_cpu_percent"] = sum(p["cpu_percent"] or 0.0 for p in procs)
        rep["workers_rss"] = sum(p["rss"] or 0 for p in procs)
        return rep

    def report_once(self):
        rep = self.collect()
        self.client.call("kv_put", agent_key(self.node_id), json.dumps(rep, default=str).encode(), True,
                         AGENT_NAMESPACE)
        self._reports += 1
        self.last_report = rep
        return rep

    def run(self):
        threading.Thread(target=self.server.serve_forever, daemon=True, name="rca-agent-http").start()
        try:
            while not self._stop.is_set() and self._parent_alive():
                try:
                    self.report_once()
                except Exception as e:  # noqa - head gone or busy: retry next period / exit below
                    if self.client._closed:
                        break
                    print(f"dashboard agent {self.node_id[:8]}: report failed: {e}", file=sys.stderr)
                self._stop.wait(self.period_s)
        finally:
            try:
                self.client.call("kv_del", agent_key(self.node_id), AGENT_NAMESPACE)
            except Exception:  # noqa
                pass
            self.server.shutdown()
            self.client.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description="per-node dashboard agent")
    ap.add_argument("--sock", required=True)
    ap.add_argument("--node-id", required=True)
    ap.add_argument("--period", type=float, default=1.0)
    ap.add_argument("--parent-pid", type=int, default=None)
    a = ap.parse_args(argv)
    agent = DashboardAgent(a.sock, a.node_id, a.period, a.parent_pid)
    import signal

    signal.signal(signal.SIGTERM, lambda *_: agent._stop.set())  # leave through run()'s cleanup
    agent.run()


if __name__ == "__main__":
    main()
