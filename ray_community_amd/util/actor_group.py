"""``ray.util.actor_group.ActorGroup`` (deprecated in the reference, kept for API parity:
``python/ray/util/actor_group.py``): N identical actors driven as one -- ``group.method.remote()``
fans the call out and returns one ref per actor; ``start`` / ``shutdown(patience_s)`` /
``add_actors`` / ``remove_actors``; ``group[i]`` is an ``ActorWrapper(actor, metadata)`` whose
metadata (node, pid, GPU ids) each actor reports about itself once it is up."""
from __future__ import annotations

import os
import socket
import warnings
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple, Type


@dataclass
class ActorMetadata:
    node_id: str
    node_ip: str
    hostname: str
    gpu_ids: List[Any] = field(default_factory=list)
    pid: int = 0


@dataclass
class ActorWrapper:
    actor: Any
    metadata: ActorMetadata


@dataclass
class ActorConfig:
    num_cpus: float
    num_gpus: float
    resources: Optional[Dict[str, float]]
    init_args: Tuple
    init_kwargs: Dict


def _self_metadata() -> ActorMetadata:
    from .. import get_gpu_ids, get_runtime_context
    from . import get_node_ip_address

    ctx = get_runtime_context()
    return ActorMetadata(node_id=str(ctx.get_node_id()), node_ip=get_node_ip_address(), hostname=socket.gethostname(),
                         gpu_ids=list(get_gpu_ids()), pid=os.getpid())


class _GroupMethod:
    def __init__(self, group: "ActorGroup", name: str):
        self._group = group
        self._name = name

    def __call__(self, *args, **kwargs):
        raise TypeError(f"ActorGroup methods cannot be called directly: use '{self._name}.remote()'.")

    def remote(self, *args, **kwargs):
        return [getattr(w.actor, self._name).remote(*args, **kwargs) for w in self._group.actors]


class ActorGroup:
    def __init__(self, actor_cls: Type, num_actors: int = 1, num_cpus_per_actor: float = 1,
                 num_gpus_per_actor: float = 0, resources_per_actor: Optional[Dict[str, float]] = None,
                 init_args: Optional[Tuple] = None, init_kwargs: Optional[Dict] = None):
        warnings.warn("ActorGroup is deprecated: use ray.util.multiprocessing for stateless work or "
                      "Dataset.map_batches with an actor pool for stateful batch processing.", DeprecationWarning,
                      stacklevel=2)
        if num_actors <= 0:
            raise ValueError(f"The provided `num_actors` must be greater than 0. Received num_actors={num_actors}.")
        if num_cpus_per_actor < 0 or num_gpus_per_actor < 0:
            raise ValueError("The number of CPUs and GPUs per actor must not be negative.")
        from .. import remote

        self.num_actors = num_actors
        self.actor_config = ActorConfig(num_cpus_per_actor, num_gpus_per_actor, resources_per_actor,
                                        tuple(init_args or ()), dict(init_kwargs or {}))
        # each actor reports its own placement: the user's class plus one metadata method
        body = type(actor_cls.__name__, (actor_cls,), {"_rca_group_metadata": lambda self: _self_metadata()})
        opts = {"num_cpus": num_cpus_per_actor, "num_gpus": num_gpus_per_actor}
        if resources_per_actor:
            opts["resources"] = resources_per_actor
        self._remote_cls = remote(**opts)(body)
        self.actors: List[ActorWrapper] = []
        self.start()

    def __getattr__(self, name):
        if name.startswith("_") or name in ("actors", "num_actors", "actor_config"):
            raise AttributeError(name)
        if not self.actors:
            raise RuntimeError("This ActorGroup has been shutdown. Please start it again.")
        return _GroupMethod(self, name)

    def __len__(self):
        return len(self.actors)

    def __getitem__(self, i):
        return self.actors[i]

    @property
    def actor_metadata(self) -> List[ActorMetadata]:
        return [w.metadata for w in self.actors]

    def start(self):
        if self.actors:
            raise RuntimeError("The actors have already been started. Call `shutdown` first to restart them.")
        self.add_actors(self.num_actors)

    def add_actors(self, num_actors: int):
        from .. import get

        cfg = self.actor_config
        handles = [self._remote_cls.remote(*cfg.init_args, **cfg.init_kwargs) for _ in range(num_actors)]
        metas = get([h._rca_group_metadata.remote() for h in handles])
        self.actors.extend(ActorWrapper(h, m) for h, m in zip(handles, metas))

    def remove_actors(self, actor_indexes: List[int]):
        drop = set(actor_indexes)
        self.actors = [w for i, w in enumerate(self.actors) if i not in drop]

    def shutdown(self, patience_s: float = 5):
        """Graceful ``__ray_terminate__`` for up to ``patience_s`` seconds, then force kill."""
        from .. import kill, wait

        if patience_s > 0:
            refs = [w.actor.__ray_terminate__.remote() for w in self.actors]
            _, pending = wait(refs, num_returns=len(refs), timeout=patience_s)
            if pending:
                for w in self.actors:
                    kill(w.actor)
        else:
            for w in self.actors:
                kill(w.actor)
        self.actors = []


__all__ = ["ActorGroup", "ActorWrapper", "ActorMetadata", "ActorConfig"]
