"""Command-line interface (reference: ``python/ray/scripts/scripts.py`` — the ``ray`` CLI, and
``python/ray/util/state/state_cli.py`` / ``dashboard/modules/job/cli.py`` for ``list``,
``summary`` and ``job``).

    python -m ray_community_amd start --head [--num-cpus N] [--num-gpus N] [--block]
    python -m ray_community_amd status | stop [--force] | timeline [--output F] | memory
    python -m ray_community_amd list actors|tasks|objects|nodes|workers|placement-groups|jobs
    python -m ray_community_amd summary tasks|actors|objects
    python -m ray_community_amd job submit [--submission-id ID] [--no-wait] -- <entrypoint ...>
    python -m ray_community_amd job status|logs|stop|delete <id> | job list
    python -m ray_community_amd microbenchmark | healthcheck
    python -m ray_community_amd serve start|deploy CONFIG|run CONFIG_OR_IMPORT_PATH|status|config|build|shutdown

Single-node design: ``start --head`` runs the session's head (scheduler, object store, worker
pool) in a detached process that owns it until ``stop``; every other command and every
``init(address="auto")`` driver connects to it over its unix socket, located through
``<temp-dir>/latest_session.json``. ``stop`` signals exactly the head process it started (pid
recorded in that file) and the head shuts its worker processes down.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
from typing import List, Optional

DEFAULT_ROOT = "/tmp/rca"


def _root(args) -> str:
    return getattr(args, "temp_dir", None) or os.environ.get("RCA_TEMP_DIR") or DEFAULT_ROOT


def _session_file(root: str) -> str:
    return os.path.join(root, "latest_session.json")


def _read_session(root: str) -> Optional[dict]:
    try:
        with open(_session_file(root)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return None


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except OSError:
        return False


def _connect(args):
    import ray_community_amd as ray

    addr = getattr(args, "address", None) or "auto"
    if addr == "auto":
        os.environ.setdefault("RCA_TEMP_DIR", _root(args))
        sess = _read_session(_root(args))
        if not sess or not os.path.exists(sess.get("sock", "")):
            raise SystemExit(f"no running session under {_root(args)} (start one with `start --head`)")
    ray.init(address=addr, namespace="_rca_cli", log_to_driver=False)
    return ray


# ------------------------------------------------------------------------------------- start/stop
def _run_head(args) -> int:
    """Foreground head: init() a local session and serve until SIGTERM/SIGINT."""
    import threading

    import ray_community_amd as ray

    os.environ["RCA_TEMP_DIR"] = _root(args)
    res = json.loads(args.resources) if args.resources else None
    ray.init(num_cpus=args.num_cpus, num_gpus=args.num_gpus, resources=res, namespace="",
             include_dashboard=args.include_dashboard, dashboard_port=args.dashboard_port,
             object_store_memory=args.object_store_memory, _temp_dir=_root(args))
    from .._private.gc_tuning import tune_gc

    tune_gc()  # this process is a dedicated head: freeze the startup heap too
    asc = None
    if getattr(args, "autoscaling_config", None):
        import yaml

        from ..autoscaler import StandardAutoscaler

        with open(args.autoscaling_config) as f:
            asc = StandardAutoscaler(yaml.safe_load(f)).start()
    if getattr(args, "ray_client_server_port", None):
        from ..util.client.server import serve

        serve(f"{args.ray_client_server_host}:{args.ray_client_server_port}")
    stop = threading.Event()
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, lambda *_: stop.set())
    sess = _read_session(_root(args)) or {}
    print(json.dumps({"address": sess.get("sock"), "pid": os.getpid(), "session": sess.get("session")}), flush=True)
    while not stop.wait(0.5):
        pass
    if asc is not None:
        asc.stop()
    ray.shutdown()
    try:
        cur = _read_session(_root(args))
        if cur and cur.get("pid") == os.getpid():
            os.unlink(_session_file(_root(args)))
    except OSError:
        pass
    return 0


def cmd_start(args) -> int:
    if not args.head:
        print("only single-node sessions are supported: use `start --head`", file=sys.stderr)
        return 2
    root = _root(args)
    cur = _read_session(root)
    if cur and _alive(int(cur.get("pid", -1))) and os.path.exists(cur.get("sock", "")):
        print(f"a session is already running (pid {cur['pid']}, address {cur['sock']}); run `stop` first",
              file=sys.stderr)
        return 1
    if args.block:
        return _run_head(args)
    os.makedirs(root, exist_ok=True)
    log = open(os.path.join(root, "head.out"), "ab")
    cmd = [sys.executable, "-m", "ray_community_amd.scripts.scripts", "_run_head", "--temp-dir", root]
    for flag in ("num_cpus", "num_gpus", "resources", "dashboard_port", "object_store_memory",
                 "ray_client_server_port", "ray_client_server_host", "autoscaling_config"):
        v = getattr(args, flag)
        if v is not None:
            cmd += ["--" + flag.replace("_", "-"), str(v)]
    if args.include_dashboard:
        cmd.append("--include-dashboard")
    env = dict(os.environ, RCA_TEMP_DIR=root)
    proc = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                            start_new_session=True, env=env)
    deadline = time.time() + args.timeout
    while time.time() < deadline:
        sess = _read_session(root)
        if sess and sess.get("pid") == proc.pid and os.path.exists(sess.get("sock", "")):
            print(f"Started head (pid {proc.pid}).\n  address: {sess['sock']}\n"
                  f"  connect with: init(address=\"auto\")  (RCA_TEMP_DIR={root})")
            return 0
        if proc.poll() is not None:
            print(f"head exited with code {proc.returncode}; see {os.path.join(root, 'head.out')}", file=sys.stderr)
            return 1
        time.sleep(0.1)
    print("timed out waiting for the head to come up", file=sys.stderr)
    return 1


def cmd_stop(args) -> int:
    root = _root(args)
    sess = _read_session(root)
    if not sess or not _alive(int(sess.get("pid", -1))):
        print("no running session")
        try:
            os.unlink(_session_file(root))
        except OSError:
            pass
        return 0
    pid = int(sess["pid"])
    os.kill(pid, signal.SIGTERM)
    deadline = time.time() + args.grace_period
    while time.time() < deadline and _alive(pid):
        time.sleep(0.1)
    if _alive(pid):
        if not args.force:
            print(f"head (pid {pid}) still running after {args.grace_period}s; use --force", file=sys.stderr)
            return 1
        os.kill(pid, signal.SIGKILL)
    try:
        os.unlink(_session_file(root))
    except OSError:
        pass
    print(f"Stopped head (pid {pid}).")
    return 0


# ------------------------------------------------------------------------------------- inspection
def _fmt_res(d: dict) -> str:
    out = []
    for k in sorted(d):
        v = d[k]
        if k in ("memory", "object_store_memory"):
            out.append(f"{k}: {v / 2**30:.1f} GiB")
        elif not k.startswith("node:"):
            out.append(f"{k}: {v:g}")
    return ", ".join(out)


def cmd_status(args) -> int:
    ray = _connect(args)
    try:
        nodes = ray.nodes()
        total, avail = ray.cluster_resources(), ray.available_resources()
        print("======== Cluster status ========")
        print(f"Nodes: {sum(1 for n in nodes if n.get('Alive', True))} alive / {len(nodes)} total")
        for n in nodes:
            print(f"  {n.get('NodeID', '?')[:12]}  alive={n.get('Alive', True)}  {_fmt_res(n.get('Resources', {}))}")
        print("Usage:")
        for k in sorted(total):
            if k.startswith("node:"):
                continue
            used = total[k] - avail.get(k, 0.0)
            if k in ("memory", "object_store_memory"):
                print(f"  {used / 2**30:.2f}/{total[k] / 2**30:.2f} GiB {k}")
            else:
                print(f"  {used:g}/{total[k]:g} {k}")
        if args.json:
            print(json.dumps({"nodes": nodes, "total": total, "available": avail}, default=str))
    finally:
        ray.shutdown()
    return 0


def cmd_healthcheck(args) -> int:
    try:
        ray = _connect(args)
    except Exception as e:  # noqa: BLE001
        print(f"unhealthy: {e}", file=sys.stderr)
        return 1
    ok = bool(ray.nodes())
    ray.shutdown()
    print("healthy" if ok else "unhealthy")
    return 0 if ok else 1


def cmd_stack(args) -> int:
    """Python stacks of every worker of the session on this machine: each worker process has a
    faulthandler on SIGUSR1 (worker_main.py), which writes all thread stacks into its log; this
    signals them and prints the dumps (the reference shells out to py-spy, not installed here)."""
    import signal
    import time

    from ray_community_amd.util import state

    ray = _connect(args)
    try:
        workers = [w for w in state.list_workers() if w.get("pid")]
        sent = []
        for w in workers:
            try:
                os.kill(int(w["pid"]), signal.SIGUSR1)
                sent.append(w)
            except (ProcessLookupError, PermissionError):
                continue
        time.sleep(args.wait)
        for w in sent:
            lines = list(state.get_log(pid=int(w["pid"]), tail=args.lines))
            heads = [i for i, l in enumerate(lines) if l.startswith(("Thread 0x", "Current thread"))]
            start = heads[0] if heads else 0  # the dump's first thread header within the tail
            print(f"=== worker pid {w['pid']} ({str(w.get('worker_id', ''))[:12]}) ===")
            print("\n".join(lines[start:]))
        print(f"{len(sent)} worker(s) dumped")
    finally:
        ray.shutdown()
    return 0


def _usage_stats_path() -> str:
    return os.path.join(os.path.expanduser("~"), ".ray", "config.json")


def cmd_usage_stats(args) -> int:
    """``disable-usage-stats`` / ``enable-usage-stats``: the reference's persistent opt-out
    (``~/.ray/config.json``). Nothing is ever reported from this framework; the setting is kept
    so tooling that reads it sees the user's choice."""
    path = _usage_stats_path()
    os.makedirs(os.path.dirname(path), exist_ok=True)
    cfg = {}
    if os.path.exists(path):
        with open(path) as f:
            try:
                cfg = json.load(f)
            except ValueError:
                cfg = {}
    cfg["usage_stats"] = bool(args.enable)
    with open(path, "w") as f:
        json.dump(cfg, f)
    print(f"usage stats {'enabled' if args.enable else 'disabled'} ({path})")
    return 0


def cmd_global_gc(args) -> int:
    """Run ``gc.collect()`` in the driver and in one task per CPU slot of every node (the
    workers the tasks land on free what only cyclic garbage kept alive)."""
    import gc

    ray = _connect(args)
    try:
        gc.collect()

        @ray.remote(num_cpus=0)
        def _collect():
            import gc as _gc

            return _gc.collect()

        n = max(1, int(sum(nd.get("Resources", {}).get("CPU", 1) for nd in ray.nodes())))
        freed = sum(ray.get([_collect.remote() for _ in range(n)]))
        print(f"global gc: {freed} objects collected in workers")
    finally:
        ray.shutdown()
    return 0


_LISTS = {"actors": "list_actors", "tasks": "list_tasks", "objects": "list_objects", "nodes": "list_nodes",
          "workers": "list_workers", "placement-groups": "list_placement_groups"}


def _parse_filters(fs: List[str]):
    out = []
    for f in fs or []:
        for op in ("!=", "="):
            if op in f:
                k, v = f.split(op, 1)
                out.append((k.strip(), op, v.strip()))
                break
        else:
            raise SystemExit(f"bad filter {f!r} (use key=value or key!=value)")
    return out


def _print_rows(rows, fmt: str):
    if fmt == "json":
        print(json.dumps(rows, indent=2, default=str))
        return
    if not rows:
        print("(none)")
        return
    cols = [c for c in rows[0].keys() if not isinstance(rows[0][c], (dict, list))][:8]
    width = {c: max(len(c), *(len(str(r.get(c, ""))[:40]) for r in rows)) for c in cols}
    print("  ".join(c.upper().ljust(width[c]) for c in cols))
    for r in rows:
        print("  ".join(str(r.get(c, ""))[:40].ljust(width[c]) for c in cols))


def cmd_list(args) -> int:
    ray = _connect(args)
    try:
        if args.resource == "jobs":
            from ..job_submission import JobSubmissionClient

            rows = [dict(vars(j)) if not isinstance(j, dict) else j for j in JobSubmissionClient().list_jobs()]
            rows = [{k: (str(v) if hasattr(v, "value") else v) for k, v in r.items()} for r in rows]
        else:
            from ..util import state

            rows = getattr(state, _LISTS[args.resource])(filters=_parse_filters(args.filter), limit=args.limit,
                                                          detail=args.detail)
            rows = [r if isinstance(r, dict) else dict(vars(r)) for r in rows]
        _print_rows(rows, args.format)
    finally:
        ray.shutdown()
    return 0


def cmd_logs(args) -> int:
    """``logs`` (list files) / ``logs <file>`` / ``logs --actor-id|--task-id|--pid`` [--tail N] [--follow]."""
    ray = _connect(args)
    try:
        from ..util import state

        if not (args.filename or args.actor_id or args.task_id or args.pid):
            for node, files in state.list_logs(glob_filter=args.glob).items():
                print(f"node {node}:")
                for f in files:
                    print(f"  {f}")
            return 0
        for line in state.get_log(filename=args.filename, actor_id=args.actor_id, task_id=args.task_id,
                                  pid=args.pid, tail=args.tail, follow=args.follow):
            print(line, flush=True)
    finally:
        ray.shutdown()
    return 0


def cmd_debug(args) -> int:
    """List the session's remote breakpoints (util.pdb.set_trace) and attach to one: this
    terminal's lines go to the breakpoint's pdb, its output comes back."""
    import select
    import socket as _socket

    ray = _connect(args)
    try:
        from ..util.pdb import list_breakpoints

        bps = list_breakpoints()
    finally:
        ray.shutdown()
    if not bps:
        print("No active breakpoints.")
        return 0
    for i, b in enumerate(bps):
        print(f"{i}: pid {b['pid']} at {b['host']}:{b['port']}")
    idx = args.index if args.index is not None else (0 if len(bps) == 1 else int(input("Enter breakpoint index: ")))
    b = bps[idx]
    conn = _socket.create_connection((b["host"], b["port"]))
    try:
        while True:
            r, _, _ = select.select([conn, sys.stdin], [], [])
            if conn in r:
                data = conn.recv(65536)
                if not data:
                    return 0
                sys.stdout.write(data.decode("utf-8", "replace"))
                sys.stdout.flush()
            if sys.stdin in r:
                line = sys.stdin.readline()
                if not line:
                    return 0
                conn.sendall(line.encode())
    finally:
        conn.close()


def cmd_summary(args) -> int:
    ray = _connect(args)
    try:
        from ..util import state

        out = getattr(state, f"summarize_{args.resource}")()
        print(json.dumps(out, indent=2, default=str))
    finally:
        ray.shutdown()
    return 0


def cmd_memory(args) -> int:
    ray = _connect(args)
    try:
        from ..util import state

        stats = state.object_store_stats()
        print("======== Object store ========")
        print(json.dumps(stats, indent=2, default=str))
        objs = state.list_objects(limit=args.limit)
        print(f"======== Objects ({len(objs)}) ========")
        _print_rows([o if isinstance(o, dict) else dict(vars(o)) for o in objs], "table")
    finally:
        ray.shutdown()
    return 0


def cmd_timeline(args) -> int:
    ray = _connect(args)
    try:
        path = args.output or os.path.join(_root(args), f"timeline-{time.strftime('%Y-%m-%d_%H-%M-%S')}.json")
        ray.timeline(filename=path)
        print(f"Trace file written to {path} (open in chrome://tracing or Perfetto).")
    finally:
        ray.shutdown()
    return 0


def cmd_microbenchmark(args) -> int:
    from .._private import ray_perf

    results = ray_perf.run(window=args.window, rounds=args.rounds, pattern=args.filter)
    ray_perf.report(results, out=args.out)
    return 0


# ------------------------------------------------------------------------------------- jobs
def cmd_job(args) -> int:
    ray = _connect(args)
    try:
        from ..job_submission import JobSubmissionClient

        c = JobSubmissionClient()
        if args.job_cmd == "submit":
            ep = args.entrypoint
            if ep and ep[0] == "--":
                ep = ep[1:]
            if not ep:
                print("missing entrypoint", file=sys.stderr)
                return 2
            renv = json.loads(args.runtime_env_json) if args.runtime_env_json else None
            sid = c.submit_job(entrypoint=" ".join(ep), submission_id=args.submission_id, runtime_env=renv)
            print(f"Job '{sid}' submitted successfully")
            if args.no_wait:
                return 0
            st = c.wait_until_finish(sid, timeout_s=args.timeout)
            sys.stdout.write(c.get_job_logs(sid))
            print(f"Job '{sid}' {st}")
            return 0 if str(st) == "SUCCEEDED" else 1
        if args.job_cmd == "status":
            print(c.get_job_status(args.job_id))
        elif args.job_cmd == "logs":
            sys.stdout.write(c.get_job_logs(args.job_id))
        elif args.job_cmd == "stop":
            print("stopped" if c.stop_job(args.job_id) else "not running")
        elif args.job_cmd == "delete":
            print("deleted" if c.delete_job(args.job_id) else "not found")
        elif args.job_cmd == "list":
            for j in c.list_jobs():
                d = j if isinstance(j, dict) else vars(j)
                print(json.dumps({k: str(v) for k, v in d.items()}))
    finally:
        ray.shutdown()
    return 0


# ------------------------------------------------------------------------------------- parser
def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="ray", description="ray_community_amd command-line interface")
    sub = p.add_subparsers(dest="cmd", required=True)

    def head_opts(sp):
        sp.add_argument("--num-cpus", type=int, default=None)
        sp.add_argument("--num-gpus", type=int, default=None)
        sp.add_argument("--resources", default=None, help='JSON, e.g. \'{"special": 2}\'')
        sp.add_argument("--object-store-memory", type=int, default=None)
        sp.add_argument("--include-dashboard", action="store_true")
        sp.add_argument("--dashboard-port", type=int, default=None)
        sp.add_argument("--temp-dir", default=None)
        sp.add_argument("--ray-client-server-port", type=int, default=None,
                        help="serve ray:// drivers on this TCP port (reference default 10001)")
        sp.add_argument("--ray-client-server-host", default="127.0.0.1")
        sp.add_argument("--autoscaling-config", default=None,
                        help="YAML with available_node_types/min_workers/max_workers/idle_timeout_minutes: run the "
                             "autoscaler over virtual nodes in the head process")

    sp = sub.add_parser("start", help="start a head session")
    sp.add_argument("--head", action="store_true")
    sp.add_argument("--block", action="store_true", help="run in the foreground")
    sp.add_argument("--timeout", type=float, default=60.0)
    head_opts(sp)
    sp.set_defaults(fn=cmd_start)

    sp = sub.add_parser("_run_head")
    head_opts(sp)
    sp.set_defaults(fn=_run_head)

    sp = sub.add_parser("stop", help="stop the running session")
    sp.add_argument("--force", action="store_true")
    sp.add_argument("--grace-period", type=float, default=10.0)
    sp.add_argument("--temp-dir", default=None)
    sp.set_defaults(fn=cmd_stop)

    def conn_opts(sp):
        sp.add_argument("--address", default=None)
        sp.add_argument("--temp-dir", default=None)

    sp = sub.add_parser("status", help="nodes and resource usage")
    sp.add_argument("--json", action="store_true")
    conn_opts(sp)
    sp.set_defaults(fn=cmd_status)

    sp = sub.add_parser("healthcheck")
    conn_opts(sp)
    sp.set_defaults(fn=cmd_healthcheck)

    sp = sub.add_parser("stack", help="dump the Python stacks of the session's workers")
    sp.add_argument("--lines", type=int, default=200)
    sp.add_argument("--wait", type=float, default=0.5)
    conn_opts(sp)
    sp.set_defaults(fn=cmd_stack)

    for name, on in (("disable-usage-stats", False), ("enable-usage-stats", True)):
        sp = sub.add_parser(name, help=f"{'enable' if on else 'disable'} usage stats collection (a persisted flag)")
        sp.set_defaults(fn=cmd_usage_stats, enable=on)

    sp = sub.add_parser("global-gc", help="garbage-collect in the driver and the workers")
    conn_opts(sp)
    sp.set_defaults(fn=cmd_global_gc)

    sp = sub.add_parser("list", help="state API listing")
    sp.add_argument("resource", choices=sorted(list(_LISTS) + ["jobs"]))
    sp.add_argument("--filter", action="append", default=[])
    sp.add_argument("--limit", type=int, default=100)
    sp.add_argument("--detail", action="store_true")
    sp.add_argument("--format", choices=["table", "json"], default="table")
    conn_opts(sp)
    sp.set_defaults(fn=cmd_list)

    sp = sub.add_parser("logs", help="list worker log files or print one (by file, actor, task or pid)")
    sp.add_argument("filename", nargs="?")
    sp.add_argument("--actor-id")
    sp.add_argument("--task-id")
    sp.add_argument("--pid", type=int)
    sp.add_argument("--glob")
    sp.add_argument("--tail", type=int, default=-1)
    sp.add_argument("--follow", action="store_true")
    conn_opts(sp)
    sp.set_defaults(fn=cmd_logs)

    sp = sub.add_parser("debug", help="attach to a remote breakpoint (ray_community_amd.util.pdb)")
    sp.add_argument("--index", type=int)
    conn_opts(sp)
    sp.set_defaults(fn=cmd_debug)

    sp = sub.add_parser("summary", help="state API summaries")
    sp.add_argument("resource", choices=["tasks", "actors", "objects"])
    conn_opts(sp)
    sp.set_defaults(fn=cmd_summary)

    sp = sub.add_parser("memory", help="object store usage and objects")
    sp.add_argument("--limit", type=int, default=100)
    conn_opts(sp)
    sp.set_defaults(fn=cmd_memory)

    sp = sub.add_parser("timeline", help="dump a chrome trace of task events")
    sp.add_argument("--output", default=None)
    conn_opts(sp)
    sp.set_defaults(fn=cmd_timeline)

    sp = sub.add_parser("microbenchmark", help="core task/actor/object microbenchmarks")
    sp.add_argument("--window", type=float, default=1.0)
    sp.add_argument("--rounds", type=int, default=2)
    sp.add_argument("--filter", default="")
    sp.add_argument("--out", default=None)
    sp.set_defaults(fn=cmd_microbenchmark)

    sp = sub.add_parser("job", help="job submission")
    jsub = sp.add_subparsers(dest="job_cmd", required=True)
    js = jsub.add_parser("submit")
    js.add_argument("--submission-id", default=None)
    js.add_argument("--runtime-env-json", default=None)
    js.add_argument("--no-wait", action="store_true")
    js.add_argument("--timeout", type=float, default=3600.0)
    js.add_argument("entrypoint", nargs=argparse.REMAINDER)
    conn_opts(js)
    for name in ("status", "logs", "stop", "delete"):
        jx = jsub.add_parser(name)
        jx.add_argument("job_id")
        conn_opts(jx)
    jl = jsub.add_parser("list")
    conn_opts(jl)
    sp.set_defaults(fn=cmd_job)

    sp = sub.add_parser("serve", help="Serve: deploy / run / status / config / build / shutdown")
    ssub = sp.add_subparsers(dest="serve_cmd", required=True)
    ss = ssub.add_parser("start", help="start Serve (controller + proxies) on the cluster")
    ss.add_argument("--http-host", default="127.0.0.1")
    ss.add_argument("--http-port", type=int, default=8000)
    ss.add_argument("--grpc-port", type=int, default=9000)
    ss.add_argument("--grpc-servicer-functions", action="append", default=[])
    conn_opts(ss)
    ss = ssub.add_parser("deploy", help="declaratively deploy a config file (apps not in it are deleted)")
    ss.add_argument("config_file_name")
    conn_opts(ss)
    ss = ssub.add_parser("run", help="deploy a config file or an import path and wait until it runs")
    ss.add_argument("config_or_import_path")
    ss.add_argument("arguments", nargs="*", help="key=value application builder args")
    ss.add_argument("--name", default=None)
    ss.add_argument("--route-prefix", default=None)
    ss.add_argument("--working-dir", default=None)
    ss.add_argument("--app-dir", default=None)
    ss.add_argument("--runtime-env-json", default=None)
    ss.add_argument("--non-blocking", action="store_true")
    conn_opts(ss)
    ss = ssub.add_parser("status", help="application and deployment status (YAML)")
    ss.add_argument("--name", default=None)
    conn_opts(ss)
    ss = ssub.add_parser("config", help="the configs the running applications were deployed from")
    ss.add_argument("--name", default=None)
    conn_opts(ss)
    ss = ssub.add_parser("build", help="write a deployable config for import paths")
    ss.add_argument("import_paths", nargs="+")
    ss.add_argument("--app-dir", default=None)
    ss.add_argument("--output-path", "-o", default=None)
    ss = ssub.add_parser("shutdown", help="delete every application and stop Serve")
    ss.add_argument("--yes", "-y", action="store_true")
    conn_opts(ss)
    sp.set_defaults(fn=cmd_serve)
    return p


# ------------------------------------------------------------------------------------- serve
def _serve_config_from_target(args):
    """A ServeDeploySchema from ``serve run``'s target: a config file, or an import path plus
    --name / --route-prefix / --working-dir / --app-dir / --runtime-env-json / key=value args."""
    from ..serve.schema import parse_config

    target = args.config_or_import_path
    if os.path.exists(target) and target.endswith((".yaml", ".yml", ".json")):
        return parse_config(target)
    env = json.loads(args.runtime_env_json) if getattr(args, "runtime_env_json", None) else {}
    wd = getattr(args, "working_dir", None) or getattr(args, "app_dir", None)
    if wd:
        env["working_dir"] = os.path.abspath(wd)
    app_args = dict(a.split("=", 1) for a in (getattr(args, "arguments", None) or []))
    app = {"name": args.name or "default", "import_path": target, "runtime_env": env, "args": app_args}
    if args.route_prefix is not None:
        app["route_prefix"] = args.route_prefix
    return parse_config({"applications": [app]})


def _yaml(obj) -> str:
    import yaml

    return yaml.safe_dump(json.loads(json.dumps(obj, default=str)), sort_keys=False)


def cmd_serve(args) -> int:
    """``serve start|deploy|run|status|config|build|shutdown`` (reference: ``serve/scripts.py``)."""
    sc = args.serve_cmd
    if sc == "build":
        from ..serve._private.config_deploy import build_config

        text = _yaml(build_config(args.import_paths, args.app_dir))
        if args.output_path:
            with open(args.output_path, "w") as f:
                f.write(text)
        else:
            print(text, end="")
        return 0
    ray = _connect(args)
    from .. import serve
    from ..serve import api as sapi
    from ..serve._private.controller import CONTROLLER_NAME, NAMESPACE

    def controller():
        try:
            return ray.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
        except ValueError:
            return None

    if sc == "start":
        grpc = None
        if args.grpc_servicer_functions:
            grpc = {"port": args.grpc_port, "grpc_servicer_functions": list(args.grpc_servicer_functions)}
        serve.start(http_options={"host": args.http_host, "port": args.http_port}, grpc_options=grpc)
        print(f"Serve started (HTTP {args.http_host}:{args.http_port}).")
        return 0
    if sc in ("deploy", "run"):
        from pydantic import ValidationError

        from ..serve._private.config_deploy import deploy_config
        from ..serve.schema import parse_config

        try:
            cfg = parse_config(args.config_file_name) if sc == "deploy" else _serve_config_from_target(args)
        except (ValidationError, ValueError, OSError) as e:
            print(f"invalid Serve config: {e}", file=sys.stderr)
            return 1
        st = deploy_config(cfg, wait_running=(sc == "run"))
        if sc == "deploy":
            print(f"Sent deploy request for {len(cfg.applications)} application(s): {', '.join(st)}.")
            return 0
        bad = {k: v for k, v in st.items() if v != "RUNNING"}
        if bad:
            print(f"deploy failed: {bad}", file=sys.stderr)
            return 1
        print(f"Deployed {', '.join(st)}: RUNNING.", flush=True)
        if args.non_blocking:
            return 0
        stop = {"v": False}
        for sig in (signal.SIGTERM, signal.SIGINT):
            signal.signal(sig, lambda *_: stop.update(v=True))
        while not stop["v"]:
            time.sleep(0.5)
        serve.shutdown()
        return 0
    if sc == "status":
        c = controller()
        if c is None:
            print(_yaml({"proxies": {}, "applications": {}, "target_capacity": None}), end="")
            return 0
        d = ray.get(c.get_serve_instance_details.remote())
        apps = {n: {"status": a["status"], "message": a["message"], "last_deployed_time_s": a["last_deployed_time_s"],
                    "deployments": {dn: {"status": dd["status"], "replica_states": {"RUNNING": len(dd["replicas"])},
                                         "target_num_replicas": dd["target_num_replicas"], "message": dd["message"]}
                                    for dn, dd in a["deployments"].items()}}
                for n, a in d["applications"].items() if not args.name or n == args.name}
        print(_yaml({"proxies": {k: v.get("status") for k, v in d["proxies"].items()}, "applications": apps,
                     "target_capacity": d.get("target_capacity")}), end="")
        return 0
    if sc == "config":
        c = controller()
        cfgs = ray.get(c.get_app_configs.remote()) if c is not None else {}
        sel = [v for n, v in cfgs.items() if v is not None and (not args.name or n == args.name)]
        print("\n---\n\n".join(_yaml(v) for v in sel) if sel else "No config has been deployed.", end="\n")
        return 0
    if sc == "shutdown":
        if not args.yes:
            ans = input("This will shut down Serve on the cluster. Continue? [y/N] ")
            if ans.strip().lower() not in ("y", "yes"):
                return 1
        if controller() is not None:
            serve.shutdown()
        sapi._STATE["controller"] = None
        print("Sent shutdown request; applications will be deleted asynchronously.")
        return 0
    raise SystemExit(f"unknown serve command {sc}")


def main(argv: Optional[List[str]] = None) -> int:
    args = build_parser().parse_args(argv)
    return int(args.fn(args) or 0)


if __name__ == "__main__":
    sys.exit(main())
