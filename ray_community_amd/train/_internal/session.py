"""Per-worker training session (reference: ``python/ray/train/_internal/session.py``).

A session exists in every Train worker. Under ``TorchTrainer`` it is installed by the worker
actor and ``report`` streams results back to the driver; under an external launcher
(``torchrun``) a session is synthesised from the launcher's environment variables.
"""
from __future__ import annotations

import os
import queue
import threading
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional


@dataclass
class TrainContext:
    world_rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    node_rank: int = 0
    experiment_name: str = ""
    trial_name: str = ""
    trial_id: str = ""
    trial_dir: str = ""
    storage_path: str = ""
    metadata: Dict[str, Any] = field(default_factory=dict)

    def get_trial_resources(self):
        """The trial's resource request (its PlacementGroupFactory) under Tune, else the worker's
        assigned resources."""
        r = (self.metadata or {}).get("_trial_resources")
        if r is not None:
            return r
        from ..._private.worker import get_runtime_context

        try:
            return get_runtime_context().get_assigned_resources()
        except Exception:
            return {}

    def get_world_rank(self):
        return self.world_rank

    def get_world_size(self):
        return self.world_size

    def get_local_rank(self):
        return self.local_rank

    def get_local_world_size(self):
        return self.local_world_size

    def get_node_rank(self):
        return self.node_rank

    def get_experiment_name(self):
        return self.experiment_name

    def get_trial_name(self):
        return self.trial_name

    def get_trial_id(self):
        return self.trial_id

    def get_trial_dir(self):
        return self.trial_dir

    def get_storage(self):
        return self.storage_path

    def get_metadata(self):
        return self.metadata


class _Session:
    def __init__(self, context: TrainContext, checkpoint=None, dataset_shards=None, synchronous: bool = False):
        self.context = context
        self.checkpoint = checkpoint
        self.dataset_shards = dataset_shards or {}
        self.results: "queue.Queue" = queue.Queue()
        self.history: List[Dict[str, Any]] = []
        self.iteration = 0
        self.synchronous = synchronous
        self._continue = threading.Event()
        self._continue.set()
        self.stop_requested = False

    def report(self, metrics: Dict[str, Any], checkpoint=None):
        self.iteration += 1
        rec = dict(metrics)
        rec.setdefault("training_iteration", self.iteration)
        self.history.append(rec)
        if checkpoint is not None and self.context.trial_dir:
            # persist synchronously (the caller may delete its temp dir right after report)
            import shutil

            from .._checkpoint import Checkpoint

            start = int(self.context.metadata.get("_ckpt_start", 0))
            dst = os.path.join(self.context.trial_dir, f"checkpoint_{start + self.iteration - 1:06d}")
            if os.path.abspath(checkpoint.path) != os.path.abspath(dst):
                shutil.copytree(checkpoint.path, dst, dirs_exist_ok=True)
            checkpoint = Checkpoint.from_directory(dst)
        if checkpoint is not None:
            self.checkpoint = checkpoint
        self.results.put((rec, checkpoint))


_SESSION: Optional[_Session] = None


def init_session(context: TrainContext, **kw) -> _Session:
    global _SESSION
    _SESSION = _Session(context, **kw)
    return _SESSION


def shutdown_session():
    global _SESSION
    _SESSION = None


def get_session() -> _Session:
    global _SESSION
    if _SESSION is None:
        # external launcher (torchrun) or plain script: derive the context from the environment
        env = os.environ
        ctx = TrainContext(world_rank=int(env.get("RANK", 0)), world_size=int(env.get("WORLD_SIZE", 1)),
                           local_rank=int(env.get("LOCAL_RANK", 0)),
                           local_world_size=int(env.get("LOCAL_WORLD_SIZE", env.get("WORLD_SIZE", 1))),
                           node_rank=int(env.get("GROUP_RANK", 0)))
        _SESSION = _Session(ctx)
    return _SESSION
