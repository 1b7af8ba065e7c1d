"""Worker process main loop (reference: ``python/ray/_private/workers/default_worker.py`` and the
task-execution path of ``_raylet.pyx:execute_task``).

A worker connects to the head, then executes tasks pushed to it. Normal tasks and default
actors run on the main thread in arrival order; threaded actors (``max_concurrency > 1``) use a
thread pool; async actors run coroutines on a dedicated asyncio loop.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import contextlib
import ctypes
import inspect
import json
import os
import queue
import sys
import threading
import time
import traceback


def _setup_paths():
    try:
        for p in reversed(json.loads(os.environ.get("RCA_SYS_PATH", "[]"))):
            if p not in sys.path:
                sys.path.insert(0, p)
    except Exception:
        pass
    wd = os.environ.get("RCA_WORKING_DIR")
    if wd:
        try:
            os.chdir(wd)
            sys.path.insert(0, wd)
        except OSError:
            pass
    for p in json.loads(os.environ.get("RCA_PY_MODULES", "[]") or "[]"):
        d = p if os.path.isdir(p) else os.path.dirname(p)
        if d not in sys.path:
            sys.path.insert(0, d)


_setup_paths()


def _setup_runtime_env():
    """pip/conda requirement check + worker_process_setup_hook; the error (if any) fails every task."""
    spec = os.environ.get("RCA_RUNTIME_ENV")
    if not spec:
        return None
    try:
        from ..runtime_env import apply_setup_hook, check_requirements

        env = json.loads(spec)
        check_requirements(env)
        apply_setup_hook(env)
        return None
    except Exception as e:  # noqa
        return e


_ENV_ERROR = _setup_runtime_env()

from .. import exceptions as exc  # noqa: E402
from . import protocol as P  # noqa: E402
from . import serialization as ser  # noqa: E402
from .core_worker import (CoreWorker, DynamicObjectRefGenerator, ObjectRef, SocketClient, _ErrorValue,  # noqa: E402
                          set_global_core)
from .ids import new_id  # noqa: E402
from .log_monitor import LOG_LABEL_MARK  # noqa: E402
from ..util import tracing  # noqa: E402
from .object_store import ObjectStore  # noqa: E402


class _ActorExit(BaseException):
    pass


class Worker:
    def __init__(self):
        self._log_label = None  # last task / actor label announced to the log monitor
        self._calls_by_fn = {}  # function id -> executions (max_calls)
        self.group_pools = {}   # concurrency group -> thread pool (threaded actors)
        self.group_limits = {}  # concurrency group -> limit (async actors)
        self.group_sems = {}
        env = os.environ
        self.wid = bytes.fromhex(env["RCA_WORKER_ID"])
        self.inbox: "queue.SimpleQueue" = queue.SimpleQueue()  # C-level put/get: the actor-call hand-off
        self.functions = {}
        self.actor = None
        self._value_keepalive = {}
        self.actor_spec = None
        self.pool = None
        self.aloop = None
        self.asem = None
        self.running = {}  # tid -> thread ident
        self.exiting = False
        from .direct_transport import DirectServer

        # direct-call endpoint: callers of an actor hosted here push their calls to this socket
        self.direct = DirectServer(self, env.get("RCA_SESSION_DIR", ""), self.wid)
        self.client = SocketClient(env["RCA_HEAD_SOCK"], "worker", self.wid, on_message=self._on_message,
                                   register_extra={"direct_addr": self.direct.path})
        self.store = ObjectStore(env["RCA_STORE"])
        self.core = CoreWorker("worker", self.client, self.store, env["RCA_NODE_ID"], bytes.fromhex(env["RCA_JOB_ID"]),
                               env.get("RCA_NAMESPACE", ""), worker_id=self.wid, session_dir=env.get("RCA_SESSION_DIR", ""))
        gids = env.get("RCA_GPU_IDS", "")
        self.core.gpu_ids = tuple(int(x) for x in gids.split(",") if x != "")
        set_global_core(self.core)
        from .. import _private as _p  # noqa

        from . import worker as api_worker

        api_worker._attach_worker_core(self.core)

    # ------------------------------------------------------------------ messaging
    def _on_message(self, msg):
        t = msg[0]
        if t == P.EXECUTE:
            self._dispatch_spec(msg[1])
        elif t == P.EXIT:
            self.exiting = True
            self.inbox.put(None)
        elif t == P.CANCEL:
            self._cancel(msg[1], msg[2])
        elif t == P.FREE_GPU:
            self.core.free_gpu_objects(msg[1])
        elif t == P.GPU_CMD:
            threading.Thread(target=self.core.gpu_command, args=(msg[1], msg[2]), daemon=True).start()

    def _dispatch_spec(self, spec):
        """Route a task (from the head, or a direct actor call) to its executor."""
        gp = self.group_pools.get(spec.get("concurrency_group")) if spec["kind"] == "actor_task" else None
        if self.aloop is not None and spec["kind"] == "actor_task":
            self.aloop.call_soon_threadsafe(self.direct._spawn, self._run_async(spec))
        elif gp is not None:  # the method's concurrency group: its own thread pool
            gp.submit(self._execute, spec)
        elif self.pool is not None and spec["kind"] == "actor_task":
            self.pool.submit(self._execute, spec)
        else:
            self.inbox.put(spec)

    def _finish(self, spec, results, info, t_start):
        """Report a finished task: to the head, or -- for a direct actor call -- to the caller."""
        if info.get("actor_exit"):
            self.actor_exited = True
        conn = spec.get("_reply")
        tid = spec["tid"]
        if conn is None:
            self.client.send((P.TASK_DONE, tid, results, info))
            return
        # results the head has to manage (shm / GPU / nested refs) are registered before replying
        head_managed = any(r[0] != "inline" or r[3] or r[5] for r in results)
        failed = bool(info.get("error"))
        if head_managed:
            lineage = None
            if spec["kind"] == "task" and spec.get("max_retries", 0) != 0 and not failed:
                lineage = _lineage_spec(spec)  # leased task: lost outputs stay recomputable
            self.client.call("put_owned", [(rid, r[0:3], r[3], r[5], r[4]) for rid, r in
                                           zip(spec["return_ids"], results)], spec["owner_key"], lineage)
        if info.get("spans"):  # tracing on: spans reach the head before the caller sees the result
            self.client.call("add_spans", info["spans"])
        leased = spec["kind"] == "task"
        # a leased task's (start, end, outcome) rides on the reply: its CALLER reports it to the
        # head (and flushes before its own state-API / timeline queries); actor calls are batched
        # by this worker
        rec = (t_start, time.time(), failed, info.get("error_type")) if leased else None
        try:
            conn.send((P.DDONE, tid, [(r[0], r[1], r[2], r[4]) for r in results], head_managed,
                       failed and bool(info.get("retryable")), rec))
        except OSError:
            pass
        if not leased:
            self.direct.record(spec, t_start, time.time(), info)
        if info.get("actor_exit"):
            self.direct.flush()
            self.client.call_async("actor_exit")

    def _cancel(self, tid, force):
        if force:
            os._exit(1)
        ident = self.running.get(tid)
        if ident is None:
            return
        fut = getattr(self, "_async_tasks", {}).get(tid)
        if fut is not None:
            self.aloop.call_soon_threadsafe(fut.cancel)
            return
        ctypes.pythonapi.PyThreadState_SetAsyncExc(ctypes.c_ulong(ident), ctypes.py_object(exc.TaskCancelledError))

    def loop(self):
        while True:
            spec = self.inbox.get()
            if spec is None:
                break
            self._execute(spec)
        self._exit()

    def _exit(self):
        try:
            self.direct.flush()
            self.client.flush_refs()
        except Exception:
            pass
        self.direct.close()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)

    # ------------------------------------------------------------------ execution
    def _resolve_args(self, spec):
        vals = []
        for a in spec["args"]:
            if a[0] == "v":
                v, _ = ser.deserialize(a[1])
            else:  # ("d", oid, desc)
                v = self.core._materialize(a[1], a[2])
                if isinstance(v, _ErrorValue):
                    raise _DepError(v.err)
            vals.append(v)
        kw = spec.get("kw_names") or []
        if kw:
            pos, kv = vals[: len(vals) - len(kw)], vals[len(vals) - len(kw):]
            return pos, dict(zip(kw, kv))
        return vals, {}

    def _get_function(self, spec):
        fid = spec.get("fid")
        if spec.get("fblob") is not None:
            self.functions[fid] = ser.loads_function(spec["fblob"])
        fn = self.functions.get(fid)
        if fn is None and fid is not None:
            blob = self.client.call("get_function", fid)  # a task pushed by its caller directly
            if blob is not None:
                fn = self.functions[fid] = ser.loads_function(blob)
        if fn is None:
            raise exc.RaySystemError(f"function {spec.get('name')} not available on this worker")
        return fn

    def _set_ctx(self, spec):
        c = self.core.ctx
        c.task_id = spec["tid"]
        c.task_name = spec.get("name")
        c.put_index = 0
        if spec.get("gpu_ids") is not None and spec["kind"] != "actor_task":
            self.core.gpu_ids = tuple(spec.get("gpu_ids") or ())
        # an actor's methods hold the actor's resources (get_runtime_context().get_assigned_resources())
        rs = spec if spec["kind"] != "actor_task" else (getattr(self, "actor_spec", None) or spec)
        self.core.assigned_resources = rs.get("resources") or {}
        # placement group membership: an actor's calls run in the group its creation was placed in
        st = (self.actor_spec if spec["kind"] == "actor_task" and getattr(self, "actor_spec", None) else spec).get(
            "strategy")
        if st and st.get("kind") == "pg":
            c.pg_id = st["pg_id"]
            c.capture_pg = dict(st, bundle_index=-1) if st.get("capture") else None
        else:
            c.pg_id = c.capture_pg = None
        c.runtime_env = spec.get("runtime_env") if spec["kind"] != "actor_task" else \
            (getattr(self, "actor_spec", None) or {}).get("runtime_env")

    def _execute(self, spec):
        tid = spec["tid"]
        kind = spec["kind"]
        if kind != "actor_task":
            label = spec.get("class_name") if kind == "actor_creation" else spec.get("name")
            if label and label != self._log_label:
                # tells the head's log monitor what this worker's next lines belong to
                self._log_label = label
                try:
                    os.write(1, f"{LOG_LABEL_MARK}{label}\n".encode())
                except OSError:
                    pass
        t_start = time.time()
        self._set_ctx(spec)
        self.running[tid] = threading.get_ident()
        info = {}
        results = None
        trace = spec.get("trace")
        with (tracing.start_span(_span_name(spec), _span_attrs(spec), parent=trace, kind="server") if trace
              else contextlib.nullcontext()) as span:
            results, info = self._execute_body(spec, tid, kind, info)
            if span is not None and info.get("error"):
                span["status"] = "error"
        spans = tracing.drain()
        if spans:
            info["spans"] = spans
        mcalls = spec.get("max_calls") or 0
        retire = False
        if kind == "task" and mcalls > 0:
            # ``max_calls``: this worker retires after running the function that many times
            # (reference semantics, e.g. to hand leaked GPU memory back). The head learns it with
            # the completion, so it never hands the retiring worker another task.
            n = self._calls_by_fn[spec["fid"]] = self._calls_by_fn.get(spec["fid"], 0) + 1
            retire = n >= mcalls
            if retire:
                info["retire"] = True
        self._finish(spec, results, info, t_start)
        self._keepalive = None
        self._value_keepalive.pop(tid, None)
        if retire:
            self._retire_when_unowned()

    def _owns_live_objects(self) -> bool:
        """Objects whose value lives only in this process: device tensors in its GPU object store
        (the head maps readers to them over HIP IPC) and results of calls it made that it still has
        to forward (pending owned entries)."""
        from . import gpu_store

        st = gpu_store._STORE
        if st is not None and st.entries:
            return True
        owned = getattr(self.core, "owned", None)
        if owned is None:
            return False
        with owned.cond:
            return any(e.desc is None for e in owned.objs.values())

    def _retire_when_unowned(self):
        """``max_calls`` retirement. The head no longer hands this worker work; the process exits
        once nothing it owns is alive -- a CUDA tensor returned by the task stays in this process's
        GPU store until every reader has dropped it (exiting earlier would turn it into an
        OwnerDiedError for the caller)."""
        if not self._owns_live_objects():
            self.inbox.put(None)
            return

        def drain():
            while not self.exiting:
                time.sleep(0.05)
                if not self._owns_live_objects():
                    self.inbox.put(None)
                    return

        threading.Thread(target=drain, name="rca-retire-drain", daemon=True).start()

    def _execute_body(self, spec, tid, kind, info):
        results = None
        try:
            try:
                if _ENV_ERROR is not None:
                    raise _ENV_ERROR
                args, kwargs = self._resolve_args(spec)
                if kind == "actor_creation":
                    cls = self._get_function(spec)
                    self._setup_actor(spec, cls)
                    self.actor = cls(*args, **kwargs) if not spec.get("is_cross_lang") else None
                    value = None
                elif kind == "actor_task":
                    method = spec["method"]
                    if getattr(self, "actor_exited", False):
                        # calls queued behind exit_actor() / __ray_terminate__ never run
                        raise _DepError(exc.ActorDiedError(self.core.actor_id, "The actor exited (exit_actor() "
                                                                               "or __ray_terminate__)."))
                    if method == "__ray_terminate__":
                        raise _ActorExit()
                    if method == "__ray_ready__":
                        value = True
                    elif method == "__ray_call__":
                        fn, args = args[0], args[1:]
                        value = fn(self.actor, *args, **kwargs)
                    else:
                        value = getattr(self.actor, method)(*args, **kwargs)
                else:
                    fn = self._get_function(spec)
                    value = fn(*args, **kwargs)
                # refs nested in the value (ray.put inside the task) must outlive the TASK_DONE send
                self._value_keepalive[tid] = value
                results = self._pack_returns(spec, value)
            except _ActorExit:
                info["actor_exit"] = True
                results = self._pack_returns(spec, None) if spec["return_ids"] else []
        except _DepError as d:
            results, info = self._error_results(spec, d.err, dep=True)
        except exc.TaskCancelledError as e:
            results, info = self._error_results(spec, exc.TaskCancelledError(tid.hex()))
            info["retryable"] = False
        except BaseException as e:  # noqa
            if _is_exit_actor(e):
                info["actor_exit"] = True
                results = self._pack_returns(spec, None) if spec["return_ids"] else []
            else:
                results, info = self._error_results(spec, e)
        finally:
            self.running.pop(tid, None)
        return results, info

    def _error_results(self, spec, e, dep=False):
        if dep or isinstance(e, exc.RayTaskError):
            err = e
        else:
            actor_repr = None
            if self.actor is not None:
                try:
                    actor_repr = repr(self.actor)
                except Exception:
                    actor_repr = None
            err = exc.RayTaskError.from_exception(e, spec.get("name") or "task", actor_repr=actor_repr,
                                                  actor_id=self.core.actor_id)
        b = ser.serialize(err, error=True)
        data = b.to_bytes()
        res = [("inline", data, len(data), [], ser.FLAG_ERROR, False) for _ in spec["return_ids"]]
        info = {"error": True, "error_type": type(e).__name__,
                "error_msg": "".join(traceback.format_exception_only(type(e), e)).strip()}
        re_ = spec.get("retry_exceptions")
        if re_ and not dep:
            if re_ is True:
                info["retryable"] = True
            elif isinstance(re_, (list, tuple)):
                info["retryable"] = any(isinstance(e, t) for t in re_)
        return res, info

    def _pack_one(self, oid, value):
        s = ser.serialize(value)
        is_gpu = bool(s.gpu_tensors)
        desc = self.core._store_serialized(oid, s)
        gpu = self.core.gpu_info(oid) if is_gpu else False
        return (desc[0], desc[1], desc[2], s.contained, s.flags | (ser.FLAG_GPU if is_gpu else 0), gpu)

    def _pack_returns(self, spec, value):
        rids = spec["return_ids"]
        gen = spec.get("generator")
        if gen == "streaming":
            n = spec.get("_streamed", 0)  # items already streamed by an async generator
            it = value
            bp = int(spec.get("gen_backpressure") or 0)
            consumed = 0
            if inspect.isgenerator(it) or hasattr(it, "__next__") or hasattr(it, "__iter__"):
                for item in it:
                    oid = new_id()
                    r = self._pack_one(oid, item)
                    self.client.send((P.GEN_ITEM, spec["tid"], n, r + (oid,)))
                    n += 1
                    if bp and n - consumed >= bp:
                        # backpressure: do not run ahead of the consumer by more than bp items
                        consumed = self.client.call("gen_wait_consumed", spec["tid"], n - bp + 1)
                        if consumed < 0:  # the stream is gone: stop producing
                            _close_gen(it)
                            if consumed == -2:
                                raise exc.TaskCancelledError(spec["tid"].hex())
                            break
            return [self._pack_one(rids[0], n)] if rids else []
        if gen == "dynamic":
            refs = []
            for item in value:
                oid = new_id()
                r = self._pack_one(oid, item)
                # register the item object with the head, owned by the caller through the container
                self.client.call("put", oid, r[0:3], r[3], r[5], r[4])
                refs.append(ObjectRef(oid))
            container = DynamicObjectRefGenerator(refs)
            out = [self._pack_one(rids[0], container)]
            # keep the item refs alive until TASK_DONE (which pins them) has been sent
            self._keepalive = container
            return out
        n = len(rids)
        if n == 0:
            return []
        if n == 1:
            return [self._pack_one(rids[0], value)]
        if not isinstance(value, (tuple, list)) or len(value) != n:
            raise ValueError(f"Task returned {type(value).__name__} but num_returns={n}; "
                             f"return a tuple/list of length {n}.")
        return [self._pack_one(r, v) for r, v in zip(rids, value)]

    # ------------------------------------------------------------------ actors
    def _setup_actor(self, spec, cls):
        self.actor_spec = spec
        self.core.actor_id = spec["actor_id"]
        self.core.gpu_ids = tuple(spec.get("gpu_ids") or ())
        mc = spec.get("max_concurrency")
        is_async = any(inspect.iscoroutinefunction(getattr(cls, n, None)) or inspect.isasyncgenfunction(
            getattr(cls, n, None)) for n in dir(cls) if not n.startswith("__"))
        if is_async:
            self.aloop = asyncio.new_event_loop()
            self._async_tasks = {}
            t = threading.Thread(target=self.aloop.run_forever, name="rca-actor-asyncio", daemon=True)
            t.start()
            self.asem = None
            self._amc = mc or 1000
        elif mc and mc > 1:
            self.pool = concurrent.futures.ThreadPoolExecutor(max_workers=mc, thread_name_prefix="rca-actor")
        groups = spec.get("concurrency_groups") or {}
        if is_async:  # async actors: a semaphore per group bounds its concurrent coroutines
            self.group_limits = dict(groups)
            self.group_sems = {}
        else:
            self.group_pools = {g: concurrent.futures.ThreadPoolExecutor(max_workers=n, thread_name_prefix=f"rca-{g}")
                                for g, n in groups.items()}

    async def _run_async(self, spec):
        if self.asem is None:
            self.asem = asyncio.Semaphore(self._amc)
        sem = self.asem
        g = spec.get("concurrency_group")
        if g is not None and g in self.group_limits:
            sem = self.group_sems.get(g)
            if sem is None:
                sem = self.group_sems[g] = asyncio.Semaphore(self.group_limits[g])
        async with sem:
            tid = spec["tid"]
            self._set_ctx(spec)
            t_start = time.time()
            info = {}
            try:
                if getattr(self, "actor_exited", False):
                    raise _DepError(exc.ActorDiedError(self.core.actor_id, "The actor exited (exit_actor() "
                                                                           "or __ray_terminate__)."))
                args, kwargs = self._resolve_args(spec)
                method = spec["method"]
                if method == "__ray_terminate__":
                    raise _ActorExit()
                if method == "__ray_ready__":
                    fn = lambda: True  # noqa: E731
                else:
                    fn = getattr(self.actor, method) if method != "__ray_call__" else None
                if fn is None:
                    f0, args = args[0], args[1:]
                    value = f0(self.actor, *args, **kwargs)
                else:
                    value = fn(*args, **kwargs)
                if inspect.isawaitable(value):
                    task = asyncio.ensure_future(value)
                    self._async_tasks[tid] = task
                    self.running[tid] = 0
                    try:
                        value = await task
                    finally:
                        self._async_tasks.pop(tid, None)
                        self.running.pop(tid, None)
                elif inspect.isasyncgen(value):
                    if spec.get("generator") == "streaming":
                        # stream each item to the caller as the coroutine produces it
                        loop = asyncio.get_running_loop()
                        n = 0
                        bp = int(spec.get("gen_backpressure") or 0)
                        consumed = 0
                        async for x in value:
                            oid = new_id()
                            r = await loop.run_in_executor(None, self._pack_one, oid, x)
                            self.client.send((P.GEN_ITEM, spec["tid"], n, r + (oid,)))
                            n += 1
                            if bp and n - consumed >= bp:
                                consumed = await loop.run_in_executor(None, self.client.call, "gen_wait_consumed",
                                                                      spec["tid"], n - bp + 1)
                                if consumed < 0:  # the stream is gone: stop producing
                                    await value.aclose()
                                    if consumed == -2:
                                        raise exc.TaskCancelledError(spec["tid"].hex())
                                    break
                        value = iter(())
                        spec = dict(spec, _streamed=n)
                    else:
                        items = []
                        async for x in value:
                            items.append(x)
                        value = iter(items)
                if _small_value(value):
                    # small results serialise in microseconds: no thread-pool round trip
                    results = self._pack_returns(spec, value)
                else:
                    loop = asyncio.get_running_loop()
                    results = await loop.run_in_executor(None, self._pack_returns, spec, value)
            except _ActorExit:
                info["actor_exit"] = True
                results = []
                for rid in spec["return_ids"]:
                    results.append(self._pack_one(rid, None))
            except asyncio.CancelledError:
                results, info = self._error_results(spec, exc.TaskCancelledError(tid.hex()))
            except _DepError as d:
                results, info = self._error_results(spec, d.err, dep=True)
            except BaseException as e:  # noqa
                if _is_exit_actor(e):
                    info["actor_exit"] = True
                    results = [self._pack_one(rid, None) for rid in spec["return_ids"]]
                else:
                    results, info = self._error_results(spec, e)
            if spec.get("trace"):
                tr = spec["trace"]
                tracing._record({"trace_id": tr[0], "span_id": tracing._new_id(8), "parent_id": tr[1],
                                 "name": _span_name(spec), "kind": "server", "start": t_start, "end": time.time(),
                                 "pid": os.getpid(), "thread": 0, "attributes": _span_attrs(spec),
                                 "status": "error" if info.get("error") else "ok"})
            spans = tracing.drain()
            if spans:
                info["spans"] = spans
            self._finish(spec, results, info, t_start)


_SCALARS = (type(None), bool, int, float, complex)


def _close_gen(it):
    """Run a generator's ``finally`` blocks now that nobody will consume its items."""
    close = getattr(it, "close", None)
    if close is not None:
        try:
            close()
        except Exception:
            pass


def _small_value(v, depth: int = 0) -> bool:
    """True for results cheap enough to pickle on the event loop (no large buffers, no object refs
    to register): scalars, short str/bytes, small arrays and shallow small containers."""
    if isinstance(v, _SCALARS):
        return True
    if isinstance(v, (str, bytes, bytearray)):
        return len(v) <= 65536
    nb = getattr(v, "nbytes", None)
    if nb is not None and type(v).__module__ == "numpy":
        return nb <= 65536 and v.dtype != object
    if depth < 2 and isinstance(v, (tuple, list)) and len(v) <= 64:
        return all(_small_value(x, depth + 1) for x in v)
    if depth < 2 and isinstance(v, dict) and len(v) <= 64:
        return all(isinstance(k, (str, int)) and _small_value(x, depth + 1) for k, x in v.items())
    return False


class _DepError(Exception):
    def __init__(self, err):
        super().__init__(str(err))
        self.err = err


def _lineage_spec(spec):
    """The submission form of a leased task's spec (arguments back to refs), for the head's
    lineage table."""
    out = {k: v for k, v in spec.items() if k not in ("_reply", "gpu_ids", "node_id", "fblob")}
    out["args"] = [("r", a[1]) if a[0] == "d" else a for a in spec["args"]]
    return out


def _span_name(spec):
    kind = spec["kind"]
    if kind == "actor_task":
        return f"actor_method::{spec.get('name')}"
    if kind == "actor_creation":
        return f"actor_creation::{spec.get('class_name') or spec.get('name')}"
    return f"task::{spec.get('name')}"


def _span_attrs(spec):
    return {"task_id": spec["tid"].hex(), "kind": spec["kind"], "pid": os.getpid()}


def _is_exit_actor(e):
    return type(e).__name__ == "AsyncioActorExit" or type(e).__name__ == "_ActorExitSignal"


def main():
    import faulthandler
    import signal

    faulthandler.register(signal.SIGUSR1, all_threads=True)  # stack dump of a stuck worker: kill -USR1 <pid>
    from .gc_tuning import tune_gc

    tune_gc()
    w = Worker()
    try:
        w.loop()
    except KeyboardInterrupt:
        pass
    finally:
        w._exit()


if __name__ == "__main__":
    main()
