"""Public core API implementation (reference: ``python/ray/_private/worker.py``)."""
from __future__ import annotations

import atexit
import glob
import json
import logging
import os
import threading
import time
from typing import Any, List, Optional, Sequence

from .. import exceptions as exc
from . import core_worker as cw
from .core_worker import CoreWorker, DirectClient, ObjectRef, SocketClient

log = logging.getLogger("ray_community_amd")

SCRIPT_MODE = 0
WORKER_MODE = 1
LOCAL_MODE = 2

_state = {"head": None, "core": None, "mode": None, "namespace": "", "runtime_env": None, "init_lock": threading.RLock()}


def _attach_worker_core(core):
    _state["core"] = core
    _state["mode"] = WORKER_MODE
    _state["namespace"] = core.namespace


def is_initialized() -> bool:
    return _state["core"] is not None


def _core() -> CoreWorker:
    c = _state["core"]
    if c is None:
        import threading

        if _state.get("explicit_shutdown") and threading.current_thread() is not threading.main_thread():
            # a background thread of the session that was shut down (a data pump, a router
            # poller, ...): failing here beats auto-initialising a fresh session behind the user
            from ..exceptions import RaySystemError

            raise RaySystemError("the session was shut down; call init() to start a new one")
        init()
        c = _state["core"]
    return c


def _detect_gpus() -> int:
    v = os.environ.get("HIP_VISIBLE_DEVICES")
    if v is None:
        v = os.environ.get("CUDA_VISIBLE_DEVICES")
    if v is not None:
        return len([x for x in v.split(",") if x.strip() != ""])
    n = 0
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            with open(p) as f:
                txt = f.read()
            for line in txt.splitlines():
                if line.startswith("simd_count"):
                    if int(line.split()[1]) > 0:
                        n += 1
                    break
        except OSError:
            pass
    return n


def _detect_cpus() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def init(address: Optional[str] = None, *, num_cpus: Optional[int] = None, num_gpus: Optional[int] = None,
         resources: Optional[dict] = None, labels: Optional[dict] = None, object_store_memory: Optional[int] = None,
         local_mode: bool = False, ignore_reinit_error: bool = False, include_dashboard=None, dashboard_host=None,
         dashboard_port=None, job_config=None, configure_logging=True, logging_level=logging.INFO,
         logging_format=None, log_to_driver=True, namespace: Optional[str] = None, runtime_env=None,
         _system_config: Optional[dict] = None, _temp_dir: Optional[str] = None, **kwargs):
    """Start (or connect to) a session. Returns a context dict-like with ``address_info``."""
    _state["explicit_shutdown"] = False
    with _state["init_lock"]:
        if _state["core"] is not None:
            if ignore_reinit_error:
                return RayContext(_state)
            if address is not None and address == _state.get("address") and _state.get("head") is not None:
                # ``ray.init(address=cluster.address)`` after an in-process ``cluster_utils.Cluster``
                # started this very session: connecting to it is what the caller asked for
                return RayContext(_state)
            raise RuntimeError("Maybe you called init() twice by accident? Use ignore_reinit_error=True.")
        if job_config is not None:
            if namespace is None and job_config.ray_namespace is not None:
                namespace = job_config.ray_namespace
            if runtime_env is None and job_config.runtime_env:
                runtime_env = job_config.runtime_env
        _state["job_config"] = job_config
        if address is None:
            address = os.environ.get("RAY_ADDRESS") or os.environ.get("RCA_ADDRESS")
        if address in ("local", None):
            address = None
        ns = namespace if namespace is not None else ("" if address else "anon_" + os.urandom(4).hex())
        if address is not None and address.startswith("ray://"):
            from ..util.client import connect as _client_connect

            core, addr = _client_connect(address, ns, log_to_driver)
            _state.update(head=None, core=core, mode=SCRIPT_MODE, namespace=ns, address=addr, client_mode=True)
        elif address is not None:
            sock = _resolve_address(address)
            ident = os.urandom(20)
            client = SocketClient(sock, "client", ident, on_message=_driver_push_handler(log_to_driver),
                                  register_extra={"log_to_driver": bool(log_to_driver)})
            hello = client.hello
            from .object_store import ObjectStore

            store = ObjectStore(hello["store"])
            core = CoreWorker("client", client, store, hello["node_id"], hello["job_id"], ns,
                              session_dir=hello["session_dir"])
            _state.update(head=None, core=core, mode=SCRIPT_MODE, namespace=ns, address=sock)
        else:
            from .head import Head

            res = dict(resources or {})
            res["CPU"] = float(num_cpus if num_cpus is not None else _detect_cpus())
            ng = num_gpus if num_gpus is not None else _detect_gpus()
            if ng:
                res["GPU"] = float(ng)
                res.setdefault("accelerator_type:MI355X", 1.0)
            res.setdefault("memory", float(_mem_bytes() * 0.7))
            root = _temp_dir or os.environ.get("RCA_TEMP_DIR") or "/tmp/rca"
            session = os.path.join(root, f"session_{time.strftime('%Y%m%d-%H%M%S')}_{os.getpid()}_{os.urandom(2).hex()}")
            sysconf = dict(_system_config or {})
            head = Head(session, res, object_store_memory=object_store_memory, namespace=ns, system_config=sysconf,
                        labels=labels)
            res["object_store_memory"] = float(head.store_capacity)
            if log_to_driver:
                from .log_monitor import print_batches

                head.log_monitor.add_sink(print_batches)
            client = DirectClient(head)
            core = CoreWorker("driver", client, head.store, head.head_node_id, head.job_id, ns,
                              session_dir=session)
            head.driver_free_gpu_cb = core.free_gpu_objects
            head.driver_gpu_cmd_cb = core.gpu_command
            _state.update(head=head, core=core, mode=SCRIPT_MODE, namespace=ns, address=head.sock_path)
            if include_dashboard:
                from .dashboard import Dashboard

                _state["dashboard"] = Dashboard(head, dashboard_host or "127.0.0.1",
                                                8265 if dashboard_port is None else int(dashboard_port))
            try:
                os.makedirs(root, exist_ok=True)
                # temp file + rename: a concurrent ``address="auto"`` reader sees the old record or
                # the new one, never a truncated file
                tmp = os.path.join(root, f".latest_session.{os.getpid()}.tmp")
                with open(tmp, "w") as f:
                    json.dump({"sock": head.sock_path, "pid": os.getpid(), "session": session}, f)
                os.replace(tmp, os.path.join(root, "latest_session.json"))
            except OSError:
                pass
        from ..runtime_env import validate as _validate_env

        _state["runtime_env"] = _validate_env(runtime_env)
        if kwargs.get("_tracing_startup_hook"):
            from ..util import tracing

            tracing.setup_tracing(kwargs["_tracing_startup_hook"])
        cw.set_global_core(core)
        return RayContext(_state)


def _driver_push_handler(log_to_driver):
    """Head -> driver pushes on a socket driver: forwarded worker log lines."""
    from . import protocol as P

    def on_message(msg):
        if msg[0] == P.LOG_BATCH and log_to_driver:
            from .log_monitor import print_batches

            print_batches(msg[1])

    return on_message


def _mem_bytes():
    try:
        import psutil

        return psutil.virtual_memory().total
    except Exception:
        return 16 << 30


def _resolve_address(address: str) -> str:
    if address == "auto":
        root = os.environ.get("RCA_TEMP_DIR", "/tmp/rca")
        path = os.path.join(root, "latest_session.json")
        with open(path) as f:
            return json.load(f)["sock"]
    if address.startswith("unix://"):
        return address[len("unix://"):]
    if os.path.exists(address):
        return address
    raise ConnectionError(f"cannot resolve address {address!r}")


class RayContext(dict):
    def __init__(self, st):
        super().__init__(address=st.get("address"), node_id=st["core"].node_id if st["core"] else None,
                         namespace=st.get("namespace"))
        dash = st.get("dashboard")
        self.dashboard_url = dash.url if dash is not None else None
        if dash is not None:
            self["dashboard_url"] = self.dashboard_url
        self.address_info = dict(self)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        shutdown()

    def disconnect(self):
        shutdown()


def shutdown(_exiting_interpreter: bool = False):
    _state["explicit_shutdown"] = True
    with _state["init_lock"]:
        core = _state["core"]
        head = _state["head"]
        if core is None:
            return
        if _state["mode"] == WORKER_MODE:
            return
        from ..util import tracing

        tracing.enable_tracing(False)
        tracing.drain()
        for srv in _state.pop("client_servers", []) or []:
            try:
                srv.stop()
            except Exception:
                pass
        _state.pop("client_mode", None)
        dash = _state.pop("dashboard", None)
        if dash is not None:
            try:
                dash.stop()
            except Exception:
                pass
        core.shutdown()
        cw.set_global_core(None)
        _state.update(core=None, head=None, mode=None)
        if head is not None:
            head.shutdown()
        else:
            try:
                core.client.close()
            except Exception:
                pass
        _run_shutdown_hooks()


_shutdown_hooks = []


def _register_shutdown_hook(fn):
    _shutdown_hooks.append(fn)


def _run_shutdown_hooks():
    for fn in list(_shutdown_hooks):
        try:
            fn()
        except Exception:
            pass


atexit.register(lambda: shutdown(True))


# ---------------------------------------------------------------------------------- objects
def put(value, *, _owner=None) -> ObjectRef:
    return _core().put(value)


_CDR = []


def _compiled_dag_ref_type():
    if not _CDR:
        from ..dag.compiled_dag_node import CompiledDAGRef

        _CDR.append(CompiledDAGRef)
    return _CDR[0]


def get(object_refs, *, timeout: Optional[float] = None):
    core = _core()
    from .core_worker import ObjectRefGenerator

    if isinstance(object_refs, ObjectRefGenerator):
        object_refs = list(object_refs)
    cdr = _compiled_dag_ref_type()
    if isinstance(object_refs, cdr):  # compiled-DAG result (reference: ray.get dispatches these too)
        return object_refs.get(timeout=timeout)
    if isinstance(object_refs, (list, tuple)):
        refs = list(object_refs)
        if not refs:
            return []
        if all(isinstance(r, cdr) for r in refs):
            return [r.get(timeout=timeout) for r in refs]
        for r in refs:
            if not isinstance(r, ObjectRef):
                raise ValueError(f"'object_refs' must either be an ObjectRef or a list of ObjectRefs; got {type(r)}")
        return core.get(refs, timeout=timeout)
    if not isinstance(object_refs, ObjectRef):
        raise ValueError(f"'object_refs' must either be an ObjectRef or a list of ObjectRefs; got {type(object_refs)}")
    return core.get(object_refs, timeout=timeout)


def wait(object_refs, *, num_returns: int = 1, timeout: Optional[float] = None, fetch_local: bool = True):
    return _core().wait(object_refs, num_returns=num_returns, timeout=timeout, fetch_local=fetch_local)


def cancel(object_ref, *, force: bool = False, recursive: bool = True):
    from .core_worker import ObjectRefGenerator

    if isinstance(object_ref, ObjectRefGenerator):
        object_ref = object_ref._main
    if not isinstance(object_ref, ObjectRef):
        raise TypeError("cancel() only supports ObjectRefs")
    return _core().cancel(object_ref._id, force, recursive)


def free(object_refs, local_only=False):
    if isinstance(object_refs, ObjectRef):
        object_refs = [object_refs]
    core = _core()
    for r in object_refs:
        if r._id in core.owned.objs:
            core.owned.publish(r._id)
    core.forget_puts([r._id for r in object_refs])
    core.client.call("free", [r._id for r in object_refs])


# ---------------------------------------------------------------------------------- cluster
def nodes():
    return _core().client.call("nodes")


def cluster_resources():
    return _core().client.call("cluster_resources")


def available_resources():
    return _core().client.call("available_resources")


def get_gpu_ids():
    core = _core()
    return list(core.gpu_ids)


def timeline(filename=None):
    from ..util import tracing

    tracing._flush_to_head()
    from ..util.state import _flush_own_task_records

    _flush_own_task_records()
    evs = _core().client.call("timeline")
    if filename:
        with open(filename, "w") as f:
            json.dump(evs, f)
        return None
    return evs


def kill(actor, *, no_restart: bool = True):
    from ..actor import ActorHandle

    if not isinstance(actor, ActorHandle):
        raise ValueError(f"kill() only supported for actors. Got: {type(actor)}.")
    _core().client.call("kill_actor", actor._actor_id, no_restart)


def get_actor(name: str, namespace: Optional[str] = None):
    from ..actor import ActorHandle

    if not name:
        raise ValueError("Please supply a non-empty value to get_actor")
    core = _core()
    ns = namespace if namespace is not None else core.namespace
    info = core.client.call("get_actor", name, ns)
    if info is None:
        raise ValueError(f"Failed to look up actor with name '{name}'. This could because 1. You are trying to look "
                         f"up a named actor you didn't create. 2. The named actor died. 3. You did not use a "
                         f"namespace matching the namespace of the actor.")
    return ActorHandle._from_meta(info["actor_id"], info["meta"])


def _actor_handle_by_id(aid: bytes):
    from ..actor import ActorHandle

    info = _core().client.call("actor_handle", aid)
    if info is None:
        raise ValueError(f"actor {aid.hex()} is not alive")
    return ActorHandle._from_meta(info["actor_id"], info["meta"])


def get_runtime_context():
    from ..runtime_context import RuntimeContext

    return RuntimeContext(_core())


def _head():
    return _state["head"]


def get_dashboard_url() -> Optional[str]:
    """``host:port`` of this session's dashboard (None when it runs without one);
    ``RAY_OVERRIDE_DASHBOARD_URL`` wins, as in the reference."""
    override = os.environ.get("RAY_OVERRIDE_DASHBOARD_URL")
    if override:
        return override.split("://", 1)[-1]
    dash = _state.get("dashboard")
    url = getattr(dash, "url", None)
    return url.split("://", 1)[-1] if url else None


def get_resource_ids():
    """Deprecated alias of ``get_runtime_context().get_resource_ids()``."""
    return get_runtime_context().get_resource_ids()
