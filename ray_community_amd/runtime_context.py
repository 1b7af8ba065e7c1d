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
        """The current actor's name (None outside an actor or for an anonymous one)."""
        if self._core.actor_id is None:
            return None
        info = self._core.client.call("actor_info", self._core.actor_id)
        return (info or {}).get("name") or None

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
        import json

        return json.dumps(self.runtime_env or {}, default=str)

    @property
    def runtime_env(self):
        """The runtime environment of the running task / actor (the job's in the driver)."""
        env = getattr(self._core.ctx, "runtime_env", None)
        if env is None and self._core.mode != "worker":
            from ._private import worker as w

            env = w._state.get("runtime_env")
        return dict(env or {})

    @property
    def current_actor(self):
        """Handle of the actor this code runs in (reference: ``get_runtime_context().current_actor``)."""
        from ._private import worker as w

        aid = self._core.actor_id
        if aid is None:
            raise RuntimeError("This method is only available in an actor.")
        return w._actor_handle_by_id(aid)

    def get_resource_ids(self):
        return {"GPU": [(int(g) if str(g).isdigit() else g, 1.0) for g in self._core.gpu_ids]}

    def should_capture_child_tasks_in_placement_group(self) -> bool:
        return getattr(self._core.ctx, "capture_pg", None) is not None

    @property
    def gcs_address(self):
        return self._core.session_dir

    def get_placement_group_id(self):
        pg = getattr(self._core.ctx, "pg_id", None)
        return pg.hex() if pg is not None else None

    @property
    def current_placement_group_id(self):
        from ._private.ids import PlacementGroupID

        pg = getattr(self._core.ctx, "pg_id", None)
        return PlacementGroupID(pg) if pg is not None else None

    def get(self):
        return {"job_id": self.job_id, "node_id": self.node_id, "namespace": self.namespace,
                "task_id": self.task_id, "actor_id": self.actor_id}

    @property
    def pid(self):
        return os.getpid()


def get_runtime_context() -> RuntimeContext:
    """The runtime context of the calling driver / task / actor (reference module-level API)."""
    from ._private.worker import get_runtime_context as _g

    return _g()
