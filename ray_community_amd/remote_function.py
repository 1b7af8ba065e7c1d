"""``@remote`` functions (reference: ``python/ray/remote_function.py``)."""
from __future__ import annotations

import functools
import inspect
from typing import Any, Dict, Optional

from ._private import core_worker as _cw
from ._private import serialization as ser
from ._private.core_worker import ObjectRef, ObjectRefGenerator
from ._private.ids import new_id, return_ids

_WORKER = None  # ._private.worker, bound on first use (it imports this module): no per-call import


def _worker_mod():
    global _WORKER
    if _WORKER is None:
        from ._private import worker

        _WORKER = worker
    return _WORKER

_TASK_OPTIONS = {"num_cpus", "num_gpus", "memory", "resources", "accelerator_type", "num_returns", "max_retries",
                 "retry_exceptions", "scheduling_strategy", "runtime_env", "name", "max_calls", "placement_group",
                 "placement_group_bundle_index", "placement_group_capture_child_tasks", "_metadata",
                 "object_store_memory", "label_selector", "enable_task_events", "_generator_backpressure_num_objects"}


def build_resources(opts: dict, default_cpus: float) -> Dict[str, float]:
    res = dict(opts.get("resources") or {})
    for k in ("CPU", "GPU"):
        if k in res:
            raise ValueError(f"Use the '{k.lower()}' argument instead of resources={{'{k}': ...}}")
    cpus = opts.get("num_cpus")
    res["CPU"] = float(default_cpus if cpus is None else cpus)
    if opts.get("num_gpus"):
        res["GPU"] = float(opts["num_gpus"])
    if opts.get("memory"):
        res["memory"] = float(opts["memory"])
    if opts.get("accelerator_type"):
        res[f"accelerator_type:{opts['accelerator_type']}"] = 0.001
    for k, v in list(res.items()):
        if v is None or v < 0:
            raise ValueError(f"resource {k} must be non-negative")
    return {k: float(v) for k, v in res.items() if v}


def _default_strategy():
    core = _cw._core
    return getattr(core.ctx, "capture_pg", None) if core is not None else None


def build_strategy(opts: dict):
    s = opts.get("scheduling_strategy")
    pg = opts.get("placement_group")
    if (s is None or s == "DEFAULT") and (pg is None or pg == "default"):
        return _default_strategy()  # the hot path: no per-call imports
    from .util.placement_group import PlacementGroup
    from .util.scheduling_strategies import (NodeAffinitySchedulingStrategy, NodeLabelSchedulingStrategy,
                                             PlacementGroupSchedulingStrategy)

    if pg is not None and pg != "default" and s is None:
        s = PlacementGroupSchedulingStrategy(pg, opts.get("placement_group_bundle_index", -1),
                                             opts.get("placement_group_capture_child_tasks"))
    if s is None or s == "DEFAULT":
        from ._private.core_worker import _core

        core = _core
        cur = getattr(core.ctx, "capture_pg", None) if core is not None else None
        if cur is not None:
            return cur
        return None
    if s == "SPREAD":
        return {"kind": "spread"}
    if isinstance(s, NodeAffinitySchedulingStrategy):
        return {"kind": "node_affinity", "node_id": s.node_id, "soft": s.soft}
    if isinstance(s, PlacementGroupSchedulingStrategy):
        if s.placement_group is None:
            return None
        idx = s.placement_group_bundle_index
        return {"kind": "pg", "pg_id": s.placement_group.id.binary(), "bundle_index": -1 if idx is None else idx,
                "capture": bool(s.placement_group_capture_child_tasks)}
    if isinstance(s, NodeLabelSchedulingStrategy):
        from .util.scheduling_strategies import normalize_label_selector

        # hard constraints are enforced; soft preferences are not ranked (placement as DEFAULT)
        return {"kind": "labels", "hard": normalize_label_selector(s.hard)}
    if isinstance(s, PlacementGroup):
        return {"kind": "pg", "pg_id": s.id.binary(), "bundle_index": -1}
    raise ValueError(f"unsupported scheduling_strategy {s!r}")


def _merge_runtime_env(opts):
    job_env = _worker_mod()._state.get("runtime_env") or {}
    if not job_env and not opts.get("runtime_env"):
        return None
    from .runtime_env import validate

    env = validate(opts.get("runtime_env"))
    if not job_env and not env:
        return None
    out = dict(job_env)
    if env:
        for k, v in dict(env).items():
            if k == "env_vars":
                ev = dict(out.get("env_vars") or {})
                ev.update(v or {})
                out["env_vars"] = ev
            else:
                out[k] = v
    return out


class RemoteFunction:
    def __init__(self, function, options: Optional[dict] = None):
        if inspect.iscoroutinefunction(function):
            raise ValueError("'async def' should not be used for remote tasks. You can wrap the async function "
                             "with `asyncio.run(f())`.")
        self._function = function
        self._options = dict(options or {})
        bad = set(self._options) - _TASK_OPTIONS
        if bad:
            raise ValueError(f"Invalid option keyword(s) {sorted(bad)} for remote functions.")
        self._blob = None
        self._fid = None
        self._name = getattr(function, "__name__", "task")
        self._is_gen = inspect.isgeneratorfunction(function)
        self._res = None  # build_resources(self._options): the default options never change
        functools.update_wrapper(self, function)

    def __call__(self, *args, **kwargs):
        raise TypeError(f"Remote functions cannot be called directly. Instead of running '{self._name}()', "
                        f"try '{self._name}.remote()'.")

    def _ensure_exported(self, core):
        if self._blob is None:
            self._blob = ser.dumps_function(self._function)
            self._fid = core.function_id(self._blob)
        return self._fid

    def options(self, **options):
        bad = set(options) - _TASK_OPTIONS
        if bad:
            raise ValueError(f"Invalid option keyword(s) {sorted(bad)} for remote functions.")
        parent = self

        class _Opt:
            def remote(_self, *args, **kwargs):
                return parent._remote(args, kwargs, {**parent._options, **options})

            def bind(_self, *args, **kwargs):
                from .dag.dag_node import FunctionNode

                return FunctionNode(parent, args, kwargs, {**parent._options, **options})

        return _Opt()

    def remote(self, *args, **kwargs):
        return self._remote(args, kwargs, self._options)

    def _resources(self, opts):
        if opts is not self._options:
            return build_resources(opts, 1)
        if self._res is None:
            self._res = build_resources(opts, 1)
        return dict(self._res)  # the spec may be mutated downstream

    def bind(self, *args, **kwargs):
        from .dag.dag_node import FunctionNode

        return FunctionNode(self, args, kwargs, self._options)

    def _remote(self, args, kwargs, opts):
        core = _worker_mod()._core()
        fid = self._ensure_exported(core)
        num_returns = opts.get("num_returns", 1)
        generator = None
        if num_returns == "streaming":
            generator, nret = "streaming", 1
        elif num_returns == "dynamic":
            generator, nret = "dynamic", 1
        else:
            nret = int(num_returns)
        if self._is_gen and num_returns == 1 and "num_returns" not in opts:
            generator, nret = "streaming", 1
        enc, kw_names, contained, deps = core.encode_args(args, kwargs)
        tid = new_id()
        rids = return_ids(tid, nret)
        spec = {
            "tid": tid, "kind": "task", "fid": fid, "name": opts.get("name") or self._name, "args": enc,
            "kw_names": kw_names, "return_ids": rids, "resources": self._resources(opts),
            "strategy": build_strategy(opts), "max_retries": opts.get("max_retries", 3),
            "max_calls": int(opts.get("max_calls") or 0),
            "retry_exceptions": opts.get("retry_exceptions", False), "runtime_env": _merge_runtime_env(opts),
            "contained": contained, "generator": generator,
        }
        bp = int(opts.get("_generator_backpressure_num_objects") or 0)
        if generator == "streaming" and bp > 0:
            spec["gen_backpressure"] = bp  # producer pauses with this many items unconsumed
        if opts.get("label_selector"):
            from .util.scheduling_strategies import normalize_label_selector

            spec["label_selector"] = normalize_label_selector(opts["label_selector"])
        if fid not in core.registered_functions:
            spec["fblob"] = self._blob
            core.registered_functions.add(fid)
        refs = [ObjectRef(r, _register=False) for r in rids]
        with core._ref_lock:
            for r in rids:
                core._refs[r] = core._refs.get(r, 0) + 1
        core.submit_spec(spec, deps)
        del deps
        if generator == "streaming":
            return ObjectRefGenerator(tid, refs[0])
        if nret == 0:
            return None
        return refs[0] if nret == 1 else refs
