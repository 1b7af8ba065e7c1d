"""Durable workflows (reference: ``python/ray/workflow/api.py``, ``workflow_executor.py``,
``workflow_storage.py``).

``workflow.run(dag, *args, workflow_id=...)`` executes a DAG of ``@remote`` functions built with
``.bind()`` and checkpoints every task's output to the workflow storage directory as it
completes. After a failure (or a crash of the whole session) ``workflow.resume(workflow_id)``
reloads the stored DAG and re-runs only the tasks without a checkpoint. A task may return
``workflow.continuation(dag)`` to extend the workflow dynamically (recursion, loops); the
continuation's tasks are checkpointed under the parent task's id.

The workflow driver itself runs as a zero-CPU task of the session (``run_async`` returns its
ObjectRef); independent ready tasks are submitted together each wave.
"""
from __future__ import annotations

import enum
import json
import os
import shutil
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

import cloudpickle

from ..dag.dag_node import DAGNode, FunctionNode, InputAttributeNode, InputNode, _map_nested

_STORAGE = {"root": None}
_CTX = threading.local()
WORKFLOW_OPTIONS = "workflow.io/options"


class WorkflowStatus(str, enum.Enum):
    NONE = "NONE"
    RUNNING = "RUNNING"
    CANCELED = "CANCELED"
    SUCCESSFUL = "SUCCESSFUL"
    FAILED = "FAILED"
    RESUMABLE = "RESUMABLE"
    PENDING = "PENDING"


class WorkflowError(Exception):
    pass


class WorkflowExecutionError(WorkflowError):
    def __init__(self, workflow_id: str, cause: Optional[BaseException] = None):
        self.workflow_id = workflow_id
        self.cause = cause
        super().__init__(f"Workflow[id={workflow_id}] failed during execution: {cause!r}")

    def __reduce__(self):
        return (WorkflowExecutionError, (self.workflow_id, self.cause))


class WorkflowCancellationError(WorkflowError):
    def __init__(self, workflow_id: str):
        self.workflow_id = workflow_id
        super().__init__(f"Workflow[id={workflow_id}] is cancelled during execution.")

    def __reduce__(self):
        return (WorkflowCancellationError, (self.workflow_id,))


class WorkflowNotFoundError(WorkflowError):
    def __init__(self, workflow_id: str):
        self.workflow_id = workflow_id
        super().__init__(f"Workflow[id={workflow_id}] was referenced but doesn't exist.")

    def __reduce__(self):
        return (WorkflowNotFoundError, (self.workflow_id,))


# ------------------------------------------------------------------------------------ storage
def init(storage: Optional[str] = None, max_running_workflows: Optional[int] = None,
         max_pending_workflows: Optional[int] = None):
    from .._private import worker as w

    root = storage or os.environ.get("RCA_WORKFLOW_STORAGE") or "/tmp/rca/workflow_data"
    if root.startswith("file://"):
        root = root[len("file://"):]
    os.makedirs(root, exist_ok=True)
    _STORAGE["root"] = root
    if not w.is_initialized():
        w.init()


def _root() -> str:
    if _STORAGE["root"] is None:
        init()
    return _STORAGE["root"]


def _wdir(workflow_id: str, root: Optional[str] = None) -> str:
    return os.path.join(root or _root(), workflow_id)


def _write_json(path, obj):
    tmp = path + f".tmp{os.getpid()}_{threading.get_ident()}"
    with open(tmp, "w") as f:
        json.dump(obj, f)
    os.replace(tmp, path)


def _read_json(path, default=None):
    try:
        with open(path) as f:
            return json.load(f)
    except (FileNotFoundError, json.JSONDecodeError):
        return default


def _write_pickle(path, obj):
    tmp = path + f".tmp{os.getpid()}_{threading.get_ident()}"
    with open(tmp, "wb") as f:
        cloudpickle.dump(obj, f)
    os.replace(tmp, path)


def _set_status(wdir, status: WorkflowStatus, **extra):
    meta = _read_json(os.path.join(wdir, "meta.json"), {})
    meta.update(extra)
    meta["status"] = status.value
    meta["updated_at"] = time.time()
    _write_json(os.path.join(wdir, "meta.json"), meta)


# ------------------------------------------------------------------------------------ DAG -> spec
class _Step:
    __slots__ = ("task_id", "fn", "args", "kwargs", "options", "wf_options", "deps")


def _build_spec(root: DAGNode, prefix: str = "") -> Dict:
    nodes = root._topo()
    ids: Dict[int, int] = {}
    steps: List[Dict] = []
    used: Dict[str, int] = {}
    for n in nodes:
        if isinstance(n, (InputNode, InputAttributeNode)):
            continue
        if not isinstance(n, FunctionNode):
            raise TypeError(f"workflows support function nodes only (got {type(n).__name__})")
        opts = {**n._body._options, **n.get_options()}
        wf = dict(((opts.pop("_metadata", None) or {}).get(WORKFLOW_OPTIONS)) or {})
        base = wf.get("task_id") or n._body._name
        k = used.get(base, 0)
        used[base] = k + 1
        tid = prefix + (base if k == 0 else f"{base}_{k}")

        def enc(x):
            if isinstance(x, InputNode):
                return ("__wf_input__", None, None)
            if isinstance(x, InputAttributeNode):
                return ("__wf_input__", x.key, x._accessor)
            return ("__wf_step__", ids[id(x)])

        steps.append({"task_id": tid, "fn": n._body._function, "name": n._body._name,
                      "args": _map_nested(list(n.get_args()), enc), "kwargs": _map_nested(n.get_kwargs(), enc),
                      "options": opts, "wf": wf})
        ids[id(n)] = len(steps) - 1
    return {"steps": steps, "output": ids[id(root)]}


def _decode(x, values, inp):
    if isinstance(x, tuple) and len(x) == 3 and x[0] == "__wf_input__":
        args, kwargs = inp
        if x[1] is None:
            return args[0] if len(args) == 1 and not kwargs else (args, kwargs)
        if isinstance(x[1], int):
            return args[x[1]]
        return kwargs[x[1]] if x[1] in kwargs else getattr(args[0], x[1])
    if isinstance(x, tuple) and len(x) == 2 and x[0] == "__wf_step__":
        return values[x[1]]
    if isinstance(x, list):
        return [_decode(v, values, inp) for v in x]
    if isinstance(x, tuple):
        return tuple(_decode(v, values, inp) for v in x)
    if isinstance(x, dict):
        return {k: _decode(v, values, inp) for k, v in x.items()}
    return x


def _deps(x, out: set):
    if isinstance(x, tuple) and len(x) == 2 and x[0] == "__wf_step__":
        out.add(x[1])
    elif isinstance(x, (list, tuple)):
        for v in x:
            _deps(v, out)
    elif isinstance(x, dict):
        for v in x.values():
            _deps(v, out)
    return out


class _Continuation:
    def __init__(self, spec):
        self.spec = spec


def _run_task(fn, args, kwargs, task_id):
    """Body of one workflow task (runs in a worker)."""
    _CTX.in_workflow = True
    _CTX.task_id = task_id
    try:
        out = fn(*args, **kwargs)
    finally:
        _CTX.in_workflow = False
    if isinstance(out, DAGNode):
        return _Continuation(_build_spec(out, prefix=task_id + "."))
    return out


def in_workflow_execution() -> bool:
    return bool(getattr(_CTX, "in_workflow", False))


def continuation(dag_node: DAGNode):
    if not isinstance(dag_node, DAGNode):
        raise TypeError("Input should be a DAG.")
    if in_workflow_execution():
        return dag_node
    from .._private.worker import get

    return get(dag_node.execute())


# ------------------------------------------------------------------------------------ engine
def _execute_spec(spec: Dict, inp, wdir: str, workflow_id: str):
    from .._private.worker import get
    from ..remote_function import RemoteFunction

    steps = spec["steps"]
    values: Dict[int, Any] = {}
    deps = [_deps(s["args"], set()) | _deps(s["kwargs"], set()) for s in steps]
    done = set()
    runner = RemoteFunction(_run_task)
    while len(done) < len(steps):
        if os.path.exists(os.path.join(wdir, "cancel_requested")):
            _set_status(wdir, WorkflowStatus.CANCELED)
            raise WorkflowCancellationError(workflow_id)
        wave = [i for i in range(len(steps)) if i not in done and deps[i] <= done]
        submitted = []
        for i in wave:
            s = steps[i]
            tdir = os.path.join(wdir, "tasks", s["task_id"])
            out_path = os.path.join(tdir, "output.pkl")
            if os.path.exists(out_path):
                with open(out_path, "rb") as f:
                    values[i] = cloudpickle.load(f)
                done.add(i)
                continue
            args = _decode(s["args"], values, inp)
            kwargs = _decode(s["kwargs"], values, inp)
            opts = dict(s["options"])
            opts.setdefault("max_retries", s["wf"].get("max_retries", 3))
            ref = runner._remote((s["fn"], args, kwargs, s["task_id"]), {}, opts)
            submitted.append((i, ref, tdir, out_path))
        for i, ref, tdir, out_path in submitted:
            s = steps[i]
            catch = s["wf"].get("catch_exceptions", False)
            try:
                val = get(ref)
                err = None
            except Exception as e:  # noqa
                if not catch:
                    raise
                val, err = None, e
            if isinstance(val, _Continuation):
                val = _execute_spec(val.spec, inp, wdir, workflow_id)
            if catch:
                val = (val, err)
            if s["wf"].get("checkpoint", True):
                os.makedirs(tdir, exist_ok=True)
                _write_pickle(out_path, val)
                _write_json(os.path.join(tdir, "meta.json"), {"task_id": s["task_id"], "name": s["name"],
                                                              "metadata": s["wf"].get("metadata") or {},
                                                              "end_time": time.time()})
            values[i] = val
            done.add(i)
    return values[spec["output"]]


def _workflow_main(workflow_id: str, root: str):
    """Runs as a zero-CPU task: executes (or resumes) a stored workflow."""
    _STORAGE["root"] = root
    wdir = _wdir(workflow_id, root)
    with open(os.path.join(wdir, "dag.pkl"), "rb") as f:
        spec, inp = cloudpickle.load(f)
    if os.path.exists(os.path.join(wdir, "cancel_requested")):
        raise WorkflowCancellationError(workflow_id)
    _set_status(wdir, WorkflowStatus.RUNNING, start_time=time.time())
    try:
        out = _execute_spec(spec, inp, wdir, workflow_id)
    except WorkflowCancellationError:
        raise
    except Exception as e:  # noqa
        if os.path.exists(os.path.join(wdir, "cancel_requested")):
            _set_status(wdir, WorkflowStatus.CANCELED)
            raise WorkflowCancellationError(workflow_id) from e
        _set_status(wdir, WorkflowStatus.FAILED, error=repr(e))
        raise WorkflowExecutionError(workflow_id, e) from e
    _write_pickle(os.path.join(wdir, "output.pkl"), out)
    _set_status(wdir, WorkflowStatus.SUCCESSFUL, end_time=time.time())
    return out


def _launch(workflow_id: str):
    from ..remote_function import RemoteFunction

    return RemoteFunction(_workflow_main, {"num_cpus": 0, "max_retries": 0}).remote(workflow_id, _root())


def run_async(dag: DAGNode, *args, workflow_id: Optional[str] = None, metadata: Optional[Dict] = None, **kwargs):
    if not isinstance(dag, DAGNode):
        raise TypeError("Input should be a DAG.")
    workflow_id = workflow_id or f"workflow_{int(time.time() * 1000)}_{os.urandom(3).hex()}"
    wdir = _wdir(workflow_id)
    meta = _read_json(os.path.join(wdir, "meta.json"))
    if meta is not None:
        if meta["status"] == WorkflowStatus.SUCCESSFUL.value:
            from .._private.worker import put

            return put(get_output(workflow_id))
        if meta["status"] == WorkflowStatus.RUNNING.value:
            raise RuntimeError(f"Workflow[id={workflow_id}] is already running.")
        return resume_async(workflow_id)
    os.makedirs(os.path.join(wdir, "tasks"), exist_ok=True)
    spec = _build_spec(dag)
    _write_pickle(os.path.join(wdir, "dag.pkl"), (spec, (args, kwargs)))
    _write_json(os.path.join(wdir, "meta.json"), {"workflow_id": workflow_id, "status": WorkflowStatus.PENDING.value,
                                                  "metadata": dict(metadata or {}), "created_at": time.time()})
    return _launch(workflow_id)


def run(dag: DAGNode, *args, workflow_id: Optional[str] = None, metadata: Optional[Dict] = None, **kwargs) -> Any:
    from .._private.worker import get

    return get(run_async(dag, *args, workflow_id=workflow_id, metadata=metadata, **kwargs))


def resume_async(workflow_id: str):
    wdir = _wdir(workflow_id)
    if not os.path.exists(os.path.join(wdir, "dag.pkl")):
        raise WorkflowNotFoundError(workflow_id)
    meta = _read_json(os.path.join(wdir, "meta.json"), {})
    if meta.get("status") == WorkflowStatus.CANCELED.value:
        raise WorkflowCancellationError(workflow_id)
    return _launch(workflow_id)


def resume(workflow_id: str) -> Any:
    from .._private.worker import get

    return get(resume_async(workflow_id))


def resume_all(include_failed: bool = False) -> List[Tuple[str, Any]]:
    out = []
    for wid, st in list_all():
        if st == WorkflowStatus.RESUMABLE or (include_failed and st == WorkflowStatus.FAILED):
            out.append((wid, resume_async(wid)))
    return out


def get_status(workflow_id: str) -> WorkflowStatus:
    meta = _read_json(os.path.join(_wdir(workflow_id), "meta.json"))
    if meta is None:
        raise WorkflowNotFoundError(workflow_id)
    return WorkflowStatus(meta["status"])


def get_output(workflow_id: str, *, task_id: Optional[str] = None, timeout: Optional[float] = None) -> Any:
    wdir = _wdir(workflow_id)
    if task_id is not None:
        p = os.path.join(wdir, "tasks", task_id, "output.pkl")
        if not os.path.exists(p):
            raise ValueError(f"task {task_id} of workflow {workflow_id} has no checkpointed output")
        with open(p, "rb") as f:
            return cloudpickle.load(f)
    deadline = None if timeout is None else time.time() + timeout
    while True:
        st = get_status(workflow_id)
        if st == WorkflowStatus.SUCCESSFUL:
            with open(os.path.join(wdir, "output.pkl"), "rb") as f:
                return cloudpickle.load(f)
        if st in (WorkflowStatus.FAILED, WorkflowStatus.CANCELED):
            raise WorkflowExecutionError(workflow_id) if st == WorkflowStatus.FAILED else \
                WorkflowCancellationError(workflow_id)
        if deadline is not None and time.time() > deadline:
            raise TimeoutError(f"workflow {workflow_id} not finished")
        time.sleep(0.05)


def get_output_async(workflow_id: str, *, task_id: Optional[str] = None):
    from .._private.worker import put

    return put(get_output(workflow_id, task_id=task_id))


def get_metadata(workflow_id: str, task_id: Optional[str] = None) -> Dict[str, Any]:
    wdir = _wdir(workflow_id)
    if task_id is None:
        meta = _read_json(os.path.join(wdir, "meta.json"))
        if meta is None:
            raise WorkflowNotFoundError(workflow_id)
        return {"status": meta["status"], "user_metadata": meta.get("metadata", {}),
                "stats": {k: meta[k] for k in ("start_time", "end_time", "created_at") if k in meta}}
    meta = _read_json(os.path.join(wdir, "tasks", task_id, "meta.json"))
    if meta is None:
        raise ValueError(f"No such task {task_id} in workflow {workflow_id}")
    return {"task_id": task_id, "task_name": meta["name"], "user_metadata": meta.get("metadata", {}),
            "stats": {"end_time": meta.get("end_time")}}


def list_all(status_filter=None) -> List[Tuple[str, WorkflowStatus]]:
    root = _root()
    if isinstance(status_filter, (str, WorkflowStatus)):
        status_filter = {WorkflowStatus(status_filter)}
    elif status_filter is not None:
        status_filter = {WorkflowStatus(s) for s in status_filter}
    out = []
    for wid in sorted(os.listdir(root)):
        meta = _read_json(os.path.join(root, wid, "meta.json"))
        if meta is None:
            continue
        st = WorkflowStatus(meta["status"])
        if status_filter is None or st in status_filter:
            out.append((wid, st))
    return out


def cancel(workflow_id: str) -> None:
    wdir = _wdir(workflow_id)
    if not os.path.exists(os.path.join(wdir, "meta.json")):
        raise WorkflowNotFoundError(workflow_id)
    with open(os.path.join(wdir, "cancel_requested"), "w") as f:
        f.write(str(time.time()))
    _set_status(wdir, WorkflowStatus.CANCELED)


def delete(workflow_id: str) -> None:
    wdir = _wdir(workflow_id)
    if not os.path.exists(wdir):
        raise WorkflowNotFoundError(workflow_id)
    if get_status(workflow_id) == WorkflowStatus.RUNNING:
        raise WorkflowError(f"cannot delete running workflow {workflow_id}; cancel it first")
    shutil.rmtree(wdir, ignore_errors=True)


class options:
    """Decorator / ``.options(**workflow.options(...))`` source for per-task workflow options."""

    _VALID = {"task_id", "metadata", "catch_exceptions", "checkpoint", "max_retries"}

    def __init__(self, **workflow_options):
        bad = set(workflow_options) - self._VALID
        if bad:
            raise ValueError(f"Invalid option keywords {bad} for workflow tasks. Valid ones are {self._VALID}.")
        md = workflow_options.get("metadata")
        if md is not None:
            if not isinstance(md, dict):
                raise ValueError("metadata must be a dict.")
            json.dumps(md)
        self.options = {"_metadata": {WORKFLOW_OPTIONS: workflow_options}}

    def keys(self):
        return ("_metadata",)

    def __getitem__(self, key):
        return self.options[key]

    def __call__(self, f):
        from ..remote_function import RemoteFunction

        if not isinstance(f, RemoteFunction):
            raise ValueError("Only apply 'workflow.options' to remote functions.")
        f._options.update(self.options)
        return f


# ------------------------------------------------------------------------------ timers and events
def _sleep_until(end_time: float):
    time.sleep(max(0.0, end_time - time.time()))
    return end_time


def sleep(duration: float) -> DAGNode:
    """A workflow task that finishes ``duration`` seconds after this DAG was BUILT (reference
    ``workflow/api.py::sleep``): the wake-up time is stored with the DAG, so a resumed workflow
    only waits for what is left."""
    from ..remote_function import RemoteFunction

    return RemoteFunction(_sleep_until, {"num_cpus": 0}).bind(time.time() + float(duration))


class EventListener:
    """Subclass and implement ``poll_for_event`` (async, returns the event); ``event_checkpointed``
    is called once the event is part of the workflow's durable state (reference
    ``workflow/event_listener.py``)."""

    def __init__(self):
        pass

    async def poll_for_event(self, *args, **kwargs):
        raise NotImplementedError

    async def event_checkpointed(self, event) -> None:
        pass


class TimerListener(EventListener):
    async def poll_for_event(self, timestamp):
        import asyncio

        await asyncio.sleep(max(0.0, timestamp - time.time()))
        return timestamp


def _wait_event(listener_type, args, kwargs):
    import asyncio

    listener = listener_type()

    async def go():
        ev = await listener.poll_for_event(*args, **kwargs)
        await listener.event_checkpointed(ev)
        return ev

    return asyncio.run(go())


def wait_for_event(event_listener_type, *args, **kwargs) -> DAGNode:
    """A workflow task whose output is the first event ``event_listener_type().poll_for_event(*args)``
    returns; once checkpointed, a resumed workflow does not wait for it again."""
    from ..remote_function import RemoteFunction

    if not (isinstance(event_listener_type, type) and issubclass(event_listener_type, EventListener)):
        raise TypeError("wait_for_event needs an EventListener subclass")
    return RemoteFunction(_wait_event, {"num_cpus": 0}).bind(event_listener_type, args, kwargs)


__all__ = ["init", "run", "run_async", "resume", "resume_async", "resume_all", "cancel", "list_all", "delete",
           "get_output", "get_output_async", "get_status", "get_metadata", "continuation", "options",
           "WorkflowStatus", "WorkflowError", "WorkflowExecutionError", "WorkflowCancellationError",
           "WorkflowNotFoundError", "sleep", "wait_for_event", "EventListener", "TimerListener"]


def client_mode_wrap(func):
    """Identity here: a ``ray://`` client drives the same API as a local driver (the calls are
    relayed), so there is nothing to wrap into a remote task (reference
    _private/client_mode_hook.py)."""
    return func
