"""Runtime context (reference: ``python/ray/runtime_context.py``)."""
from __future__ import annotations

import os


class RuntimeContext:
    def __init__(self, core):
        self._core = core

    def get_job_id(self) -> str:
        return self._core.job_id.hex()

    @property
    def job_id(self):
        return self._core.job_id

    def get_node_id(self) -> str:
        return self._core.node_id

    @property
    def node_id(self):
        return self._core.node_id

    def get_worker_id(self) -> str:
        return self._core.worker_id.hex()

    def get_task_id(self):
        t = self._core.ctx.task_id
        return t.hex() if t else None

    @property
    def task_id(self):
        return self._core.ctx.task_id

    def get_task_name(self):
        return self._core.ctx.task_name

    def get_actor_id(self):
        a = self._core.actor_id
        return a.hex() if a else None

    @property
    def actor_id(self):
        return self._core.actor_id

    def get_actor_name(self):
        return None

    @property
    def namespace(self):
        return self._core.namespace

    def get_namespace(self):
        return self._core.namespace

    @property
    def was_current_actor_reconstructed(self):
        if self._core.actor_id is None:
            return False
        info = self._core.client.call("actor_info", self._core.actor_id)
        return bool(info and info.get("num_restarts", 0) > 0)

    def get_assigned_resources(self):
        return dict(self._core.assigned_resources or {})

    def get_accelerator_ids(self):
        return {"GPU": [str(g) for g in self._core.gpu_ids]}

    def get_runtime_env_string(self):
        return "{}"

    @property
    def gcs_address(self):
        return self._core.session_dir

    def get_placement_group_id(self):
        return None

    @property
    def current_placement_group_id(self):
        return None

    def get(self):
        return {"job_id": self.job_id, "node_id": self.node_id, "namespace": self.namespace,
                "task_id": self.task_id, "actor_id": self.actor_id}

    @property
    def pid(self):
        return os.getpid()
