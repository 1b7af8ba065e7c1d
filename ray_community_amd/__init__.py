"""ray_community_amd — an MI355X-native distributed compute framework with the capabilities of
Ray (tasks, actors, objects, placement groups, collectives, Train, Tune, Data, Serve, RLlib).

Core runtime: C++ shared-memory object store + C++ resource scheduler (``_native``), Python
control plane. Compute path: PyTorch-ROCm + hand-written gfx950 HIP kernels (``ops``) + RCCL
over xGMI (``parallel``, ``util.collective``).
"""
from __future__ import annotations

__version__ = "0.1.0"

import functools
import inspect

from ._private import import_paths as _import_paths

_import_paths.install()  # the reference's secondary module paths (``ray.tune.result_grid``, ...)

from . import exceptions
from ._private.core_worker import DynamicObjectRefGenerator, ObjectRef, ObjectRefGenerator
from ._private.ids import (ActorClassID, ActorID, FunctionID, JobID, NodeID, ObjectID, PlacementGroupID, TaskID,
                           UniqueID, WorkerID)
from ._private.worker import (LOCAL_MODE, SCRIPT_MODE, WORKER_MODE, available_resources, cancel, cluster_resources,
                              free, get, get_actor, get_gpu_ids, get_runtime_context, init, is_initialized, kill,
                              nodes, put, shutdown, timeline, wait)
from .actor import ActorClass, ActorHandle, exit_actor, method
from .remote_function import RemoteFunction


def remote(*args, **kwargs):
    """``@remote`` / ``@remote(num_cpus=..., num_gpus=..., ...)`` for functions and classes."""

    def make(obj, opts):
        if inspect.isclass(obj):
            return ActorClass(obj, opts)
        if callable(obj):
            return RemoteFunction(obj, opts)
        raise TypeError("The @remote decorator must be applied to either a function or a class.")

    if len(args) == 1 and not kwargs and callable(args[0]):
        return make(args[0], {})
    if args:
        raise TypeError("The @remote decorator must be applied either with no arguments and no parentheses, for "
                        "example '@remote', or it must be applied using some of the arguments in the list "
                        "['num_cpus', 'num_gpus', ...], for example '@remote(num_returns=2, resources={\"CustomResource\": 1})'.")
    return lambda obj: make(obj, kwargs)


class Language:
    """Task/actor languages (reference: ``ray.Language``). Only PYTHON workers exist here."""
    PYTHON = 0
    JAVA = 1
    CPP = 2


def _cross_language(kind):
    def unsupported(*a, **k):
        raise NotImplementedError(f"{kind}: cross-language (Java/C++) workers are not part of ray_community_amd; "
                                  "only Python tasks and actors are supported")
    return unsupported


java_function = _cross_language("java_function")
java_actor_class = _cross_language("java_actor_class")
cpp_function = _cross_language("cpp_function")


def show_in_dashboard(message: str, key: str = "", dtype: str = "text"):
    """Attach a message to the current actor/task, shown in its state-API record (``list_actors``
    ``repr``/dashboard): reference ``ray.show_in_dashboard``."""
    from ._private.worker import _core

    core = _core()
    aid = getattr(core, "actor_id", None)
    if aid is None:
        return
    try:
        core.client.call("actor_annotate", aid, key or "message", str(message))
    except Exception:  # noqa
        pass


def client(address: str = None):
    """``ray.client("host:port").namespace(..).connect()`` builder for Ray Client sessions."""
    return ClientBuilder(address)


class ClientBuilder:
    def __init__(self, address=None):
        self._address = address
        self._kw = {}

    def namespace(self, ns):
        self._kw["namespace"] = ns
        return self

    def env(self, runtime_env):
        self._kw["runtime_env"] = runtime_env
        return self

    def connect(self):
        addr = self._address or ""
        if addr and not addr.startswith("ray://"):
            addr = "ray://" + addr
        return init(address=addr or None, **self._kw)


_LAZY = {"util", "train", "tune", "data", "serve", "rllib", "dag", "air", "experimental", "models", "ops", "parallel",
         "cluster_utils", "job_submission", "workflow", "runtime_env", "autoscaler", "utils", "job_config", "scripts",
         "internal", "widgets"}


class _SystemConfig:
    """``ray._config`` (reference: the raylet's ``Config`` object): read-only access to the
    session's ``_system_config`` values by attribute (``ray._config.object_spilling_threshold()``
    style calls return the value)."""

    def _values(self):
        try:
            from ._private.worker import _state

            head = _state.get("head")
            return dict(getattr(head, "config", {}) or {}) if head is not None else {}
        except Exception:
            return {}

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        vals = self._values()
        if name not in vals:
            raise AttributeError(f"system config has no entry {name!r}")
        v = vals[name]
        return lambda: v


_config = _SystemConfig()


def __getattr__(name):
    if name in _LAZY:
        import importlib

        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)


__all__ = [
    "__version__", "remote", "init", "shutdown", "is_initialized", "get", "put", "wait", "cancel", "kill", "free",
    "get_actor", "get_gpu_ids", "nodes", "cluster_resources", "available_resources", "timeline", "method",
    "get_runtime_context", "ObjectRef", "ObjectRefGenerator", "DynamicObjectRefGenerator", "ActorHandle",
    "ActorClass", "RemoteFunction", "exceptions", "exit_actor", "LOCAL_MODE", "SCRIPT_MODE", "WORKER_MODE",
    "ActorID", "TaskID", "NodeID", "JobID", "ObjectID", "WorkerID", "FunctionID", "PlacementGroupID", "UniqueID",
    "ActorClassID", "Language", "java_function", "java_actor_class", "cpp_function", "show_in_dashboard",
    "client", "ClientBuilder",
]
