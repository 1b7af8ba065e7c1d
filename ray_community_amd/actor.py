"""Actors (reference: ``python/ray/actor.py``)."""
from __future__ import annotations

import inspect
import threading
from typing import Any, Dict, List, Optional

from . import exceptions as exc
from ._private import serialization as ser
from ._private.core_worker import ObjectRef, ObjectRefGenerator
from ._private.ids import new_id, return_ids
from .remote_function import _merge_runtime_env, build_resources, build_strategy

_ACTOR_OPTIONS = {"num_cpus", "num_gpus", "memory", "resources", "accelerator_type", "max_restarts",
                  "max_task_retries", "max_concurrency", "name", "namespace", "lifetime", "scheduling_strategy",
                  "runtime_env", "get_if_exists", "placement_group", "placement_group_bundle_index",
                  "placement_group_capture_child_tasks", "concurrency_groups", "max_pending_calls", "_metadata",
                  "object_store_memory", "label_selector", "enable_task_events", "_labels"}


def method(*args, **kwargs):
    """Annotate an actor method: ``@ray.method(num_returns=2, concurrency_group="io")``."""
    valid = {"num_returns", "concurrency_group", "max_task_retries", "retry_exceptions", "_generator_backpressure_num_objects",
             "enable_task_events", "tensor_transport"}

    def deco(f):
        bad = set(kwargs) - valid
        if bad:
            raise ValueError(f"Unexpected keyword arguments {bad} for @method")
        f.__rca_method_options__ = dict(kwargs)
        return f

    if len(args) == 1 and callable(args[0]) and not kwargs:
        return deco(args[0])
    return deco


def exit_actor():
    """Terminate the current actor gracefully (reference ``ray.actor.exit_actor``)."""
    from ._private.worker import _core

    core = _core()
    if core.actor_id is None:
        raise TypeError("exit_actor API is called on a non-actor worker.")
    raise exc.AsyncioActorExit()


def _class_meta(cls, opts):
    methods = {}
    for name, m in inspect.getmembers(cls, predicate=lambda x: inspect.isfunction(x) or inspect.ismethod(x)):
        if name.startswith("__") and name not in ("__call__",):
            continue
        mo = dict(getattr(m, "__rca_method_options__", {}))
        if inspect.isgeneratorfunction(m) or inspect.isasyncgenfunction(m):
            mo.setdefault("num_returns", "streaming")
        mo["is_async"] = inspect.iscoroutinefunction(m) or inspect.isasyncgenfunction(m)
        methods[name] = mo
    return {"class_name": cls.__name__, "methods": methods, "max_task_retries": opts.get("max_task_retries", 0),
            "module": cls.__module__, "max_pending_calls": int(opts.get("max_pending_calls", -1) or -1)}


class ActorClassInheritanceException(TypeError):
    """Raised on ``class B(A)`` where ``A`` is a ``@remote`` actor class: subclass the plain class
    and decorate the subclass instead."""


class ActorClass:
    def __init__(self, cls, options: Optional[dict] = None, *extra):
        if extra or isinstance(cls, str):  # class B(A) with A an ActorClass: type(A)(name, bases, ns)
            raise ActorClassInheritanceException(
                f"Cannot inherit from the actor class {getattr(options[0], '__name__', '?') if options else '?'}: "
                "inherit from the undecorated class and apply @remote to the subclass")
        self._cls = cls
        self._options = dict(options or {})
        bad = set(self._options) - _ACTOR_OPTIONS
        if bad:
            raise ValueError(f"Invalid option keyword(s) {sorted(bad)} for actors.")
        self._blob = None
        self._fid = None
        self.__name__ = cls.__name__
        self.__qualname__ = getattr(cls, "__qualname__", cls.__name__)
        self.__module__ = cls.__module__
        self.__doc__ = cls.__doc__

    def __call__(self, *args, **kwargs):
        raise TypeError(f"Actors cannot be instantiated directly. Instead of '{self.__name__}()', use "
                        f"'{self.__name__}.remote()'.")

    def _ensure_exported(self, core):
        if self._blob is None:
            self._blob = ser.dumps_function(self._cls)
            self._fid = core.function_id(self._blob)
        return self._fid

    def options(self, **options):
        bad = set(options) - _ACTOR_OPTIONS
        if bad:
            raise ValueError(f"Invalid option keyword(s) {sorted(bad)} for actors.")
        parent = self

        class _Opt:
            def remote(_self, *args, **kwargs):
                return parent._remote(args, kwargs, {**parent._options, **options})

            def bind(_self, *args, **kwargs):
                from .dag.dag_node import ClassNode

                return ClassNode(parent, args, kwargs, {**parent._options, **options})

        return _Opt()

    def remote(self, *args, **kwargs):
        return self._remote(args, kwargs, self._options)

    def bind(self, *args, **kwargs):
        from .dag.dag_node import ClassNode

        return ClassNode(self, args, kwargs, self._options)

    def _remote(self, args, kwargs, opts):
        from ._private.worker import _core, get_actor

        core = _core()
        name = opts.get("name")
        ns = opts.get("namespace")
        if ns is None:
            ns = core.namespace
        if name is not None and not isinstance(name, str):
            raise TypeError(f"name must be None or a string, got {type(name)}")
        if name == "":
            raise ValueError("Actor name cannot be an empty string.")
        if ns is not None and not isinstance(ns, str):
            raise TypeError(f"namespace must be None or a string, got {type(ns)}")
        if opts.get("get_if_exists") and not name:
            raise ValueError("The actor name must be specified to use `get_if_exists`.")
        if opts.get("get_if_exists") and name:
            try:
                return get_actor(name, namespace=ns)
            except ValueError:
                pass
        lifetime = opts.get("lifetime")
        if lifetime is None:
            from ._private.worker import _state as _wstate

            jc = _wstate.get("job_config")
            if jc is not None and getattr(jc, "default_actor_lifetime", None) == "detached":
                lifetime = "detached"
        if lifetime not in (None, "detached", "non_detached"):
            raise ValueError("actor `lifetime` argument must be one of 'detached', 'non_detached' and 'None'.")
        fid = self._ensure_exported(core)
        meta = _class_meta(self._cls, opts)
        is_async = any(m["is_async"] for m in meta["methods"].values())
        mc = opts.get("max_concurrency")
        if mc is None:
            mc = 1000 if is_async else 1
        if mc < 1:
            raise ValueError("max_concurrency must be >= 1")
        enc, kw_names, contained, deps = core.encode_args(args, kwargs)
        aid = new_id()
        res = build_resources(opts, 0)
        spec = {
            "tid": new_id(), "kind": "actor_creation", "fid": fid, "name": f"{self._cls.__name__}.__init__",
            "class_name": self._cls.__name__, "actor_id": aid, "args": enc, "kw_names": kw_names, "return_ids": [],
            "resources": res, "strategy": build_strategy(opts), "max_restarts": opts.get("max_restarts", 0),
            "max_task_retries": opts.get("max_task_retries", 0), "max_concurrency": mc,
            "concurrency_groups": opts.get("concurrency_groups"), "namespace": ns,
            "lifetime": lifetime, "runtime_env": _merge_runtime_env(opts), "contained": contained,
            "class_meta": meta, "max_retries": 0,
        }
        spec["actor_name"] = name
        if opts.get("label_selector"):
            from .util.scheduling_strategies import normalize_label_selector

            spec["label_selector"] = normalize_label_selector(opts["label_selector"])
        if fid not in core.registered_functions:
            spec["fblob"] = self._blob
            core.registered_functions.add(fid)
        spec["parent"] = core.ctx.task_id
        spec["caller_node"] = core.node_id
        from .util import tracing

        trace = tracing.submission_context()
        if trace is not None:
            spec["trace"] = trace
        if name:
            core.client.call("submit", spec)
        else:
            core.client.submit(spec)
        return ActorHandle(aid, meta, _owner=True)


class ActorMethod:
    def __init__(self, handle, name, opts):
        self._handle = handle
        self._name = name
        self._opts = opts

    def __call__(self, *args, **kwargs):
        raise TypeError(f"Actor methods cannot be called directly. Instead of running 'object.{self._name}()', "
                        f"try 'object.{self._name}.remote()'.")

    def remote(self, *args, **kwargs):
        return self._handle._submit(self._name, args, kwargs, self._opts)

    def options(self, **options):
        m = ActorMethod(self._handle, self._name, {**self._opts, **options})
        return m

    def bind(self, *args, **kwargs):
        from .dag.dag_node import ClassMethodNode

        return ClassMethodNode(self._handle, self._name, args, kwargs, self._opts)


# ``max_pending_calls`` bookkeeping, independent of the transport a call takes (direct actor
# channel, head-routed generator methods, ray:// clients, calls parked across a restart): a
# per-actor count of this process's submitted, unfinished calls, incremented at submit and
# decremented by a completion callback on the call's first return object -- whether or not the
# caller still holds its refs, and with no RPC on the submit path (reference: the submitter's
# per-actor pending-task count in ``ActorTaskSubmitter``).
_INFLIGHT: Dict[bytes, int] = {}
_PENDING_LOCK = threading.Lock()


def _pending_calls(core, actor_id) -> int:
    with _PENDING_LOCK:
        return _INFLIGHT.get(actor_id, 0)


def _track_call(core, actor_id, rid):
    with _PENDING_LOCK:
        _INFLIGHT[actor_id] = _INFLIGHT.get(actor_id, 0) + 1
    done = [False]

    def finished(*_a):
        with _PENDING_LOCK:
            if done[0]:
                return
            done[0] = True
            n = _INFLIGHT.get(actor_id, 0) - 1
            if n > 0:
                _INFLIGHT[actor_id] = n
            else:
                _INFLIGHT.pop(actor_id, None)

    owned = getattr(core, "owned", None)
    if owned is not None and owned.get_entry(rid) is not None:
        owned.on_ready(rid, finished)  # the entry outlives dropped refs while it has callbacks
        return
    try:  # head-managed result: one async wait, off the submit path
        core.client.call_async("wait", [rid], 1, None, False, True).add_done_callback(finished)
    except Exception:  # noqa  (no head connection: nothing will ever complete it)
        finished()


class ActorHandle:
    def __init__(self, actor_id: bytes, meta: dict, _owner=False, _register=True):
        self._actor_id = actor_id
        self._meta = meta
        self._ray_actor_id = actor_id
        from ._private.core_worker import _core

        self._core = _core
        if _register and _core is not None:
            _core.ref_add(b"A" + actor_id)

    @classmethod
    def _from_meta(cls, actor_id, meta):
        return cls(actor_id, meta)

    def __del__(self):
        c = self._core
        if c is not None:
            try:
                c.ref_remove(b"A" + self._actor_id)
            except Exception:
                pass

    def __getattr__(self, name):
        if name.startswith("__") and name.endswith("__") and name not in ("__ray_terminate__", "__ray_call__",
                                                                          "__ray_ready__"):
            raise AttributeError(name)
        meta = self.__dict__.get("_meta") or {}
        methods = meta.get("methods", {})
        if name not in methods and name not in ("__ray_terminate__", "__ray_call__", "__ray_ready__"):
            raise AttributeError(f"'ActorHandle' object has no attribute '{name}' "
                                 f"(actor class {meta.get('class_name')})")
        return ActorMethod(self, name, {})

    def _submit(self, name, args, kwargs, opts):
        from ._private.worker import _core

        core = _core()
        mo = dict(self._meta.get("methods", {}).get(name, {}))
        mo.update(opts)
        num_returns = mo.get("num_returns", 1)
        generator = None
        if num_returns == "streaming":
            generator, nret = "streaming", 1
        elif num_returns == "dynamic":
            generator, nret = "dynamic", 1
        else:
            nret = int(num_returns)
        limit = self._meta.get("max_pending_calls", -1)
        if limit is not None and limit > 0:
            if _pending_calls(core, self._actor_id) >= limit:
                from .exceptions import PendingCallsLimitExceeded

                raise PendingCallsLimitExceeded(
                    f"The task {self._meta.get('class_name', 'Actor')}.{name} could not be submitted because more "
                    f"than {limit} tasks are queued on the actor. This limit can be adjusted with the "
                    "`max_pending_calls` actor option.")
        enc, kw_names, contained, deps = core.encode_args(args, kwargs)
        tid = new_id()
        rids = return_ids(tid, nret)
        spec = {
            "tid": tid, "kind": "actor_task", "actor_id": self._actor_id, "method": name,
            "name": mo.get("name") or f"{self._meta.get('class_name', 'Actor')}.{name}", "args": enc,
            "kw_names": kw_names, "return_ids": rids, "contained": contained, "generator": generator,
            "max_task_retries": mo.get("max_task_retries", self._meta.get("max_task_retries", 0)),
            "concurrency_group": mo.get("concurrency_group"),
        }
        bp = int(mo.get("_generator_backpressure_num_objects") or 0)
        if generator == "streaming" and bp > 0:
            spec["gen_backpressure"] = bp
        refs = [ObjectRef(r, _register=False) for r in rids]
        with core._ref_lock:
            for r in rids:
                core._refs[r] = core._refs.get(r, 0) + 1
        core.submit_actor_task(spec, deps)
        if limit is not None and limit > 0 and rids:
            _track_call(core, self._actor_id, rids[0])
        if generator == "streaming":
            return ObjectRefGenerator(tid, refs[0])
        if nret == 0:
            return None
        return refs[0] if nret == 1 else refs

    def __reduce__(self):
        from ._private import serialization as s

        ctx = s.current_context()
        if ctx is not None:
            ctx.contained.append(b"A" + self._actor_id)
        return (ActorHandle._from_meta, (self._actor_id, self._meta))

    def __repr__(self):
        return f"Actor({self._meta.get('class_name')}, {self._actor_id.hex()})"

    def __hash__(self):
        return hash(self._actor_id)

    def __eq__(self, other):
        return isinstance(other, ActorHandle) and other._actor_id == self._actor_id

    @property
    def _actor_id_hex(self):
        return self._actor_id.hex()


def _modify_class(cls):
    return cls
