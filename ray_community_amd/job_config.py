"""Per-job configuration passed to ``init(job_config=...)`` (reference: ``python/ray/job_config.py``).

Carries the job-level runtime_env (applied to every task/actor of the job unless overridden), the
namespace, job metadata (visible in the state API / job table), and the default actor lifetime
("non_detached" or "detached").
"""
from __future__ import annotations

import json
from typing import Any, Dict, List, Optional


class JobConfig:
    def __init__(self, jvm_options: Optional[List[str]] = None, code_search_path: Optional[List[str]] = None,
                 runtime_env: Optional[Dict[str, Any]] = None, metadata: Optional[Dict[str, str]] = None,
                 ray_namespace: Optional[str] = None, default_actor_lifetime: str = "non_detached",
                 _client_job: bool = False, _py_driver_sys_path: Optional[List[str]] = None):
        self.jvm_options = list(jvm_options or [])  # accepted for API parity; no JVM workers here
        self.code_search_path = list(code_search_path or [])
        self.metadata: Dict[str, str] = dict(metadata or {})
        self.ray_namespace = ray_namespace
        self.runtime_env: Dict[str, Any] = {}
        self.set_runtime_env(runtime_env)
        self.default_actor_lifetime = "non_detached"
        self.set_default_actor_lifetime(default_actor_lifetime)
        self._client_job = _client_job
        self._py_driver_sys_path = list(_py_driver_sys_path or [])

    def set_metadata(self, key: str, value: str) -> None:
        self.metadata[key] = value

    def set_runtime_env(self, runtime_env: Optional[Dict[str, Any]], validate: bool = False) -> None:
        self.runtime_env = dict(runtime_env) if runtime_env is not None else {}
        if validate and self.runtime_env:
            from .runtime_env import validate as _validate

            self.runtime_env = dict(_validate(self.runtime_env) or {})

    def set_ray_namespace(self, ray_namespace: str) -> None:
        if not isinstance(ray_namespace, str):
            raise TypeError("ray_namespace must be a string")
        self.ray_namespace = ray_namespace

    def set_default_actor_lifetime(self, default_actor_lifetime: str) -> None:
        if default_actor_lifetime not in ("detached", "non_detached"):
            raise ValueError("default_actor_lifetime must be 'detached' or 'non_detached'")
        self.default_actor_lifetime = default_actor_lifetime

    def _serialize(self) -> str:
        return json.dumps({"runtime_env": self.runtime_env, "metadata": self.metadata,
                           "ray_namespace": self.ray_namespace, "default_actor_lifetime": self.default_actor_lifetime,
                           "code_search_path": self.code_search_path, "jvm_options": self.jvm_options})

    @classmethod
    def from_json(cls, job_config_json) -> "JobConfig":
        d = json.loads(job_config_json) if isinstance(job_config_json, str) else dict(job_config_json)
        return cls(runtime_env=d.get("runtime_env"), metadata=d.get("metadata"),
                   ray_namespace=d.get("ray_namespace"),
                   default_actor_lifetime=d.get("default_actor_lifetime", "non_detached"),
                   code_search_path=d.get("code_search_path"), jvm_options=d.get("jvm_options"))

    def __repr__(self):
        return f"JobConfig({self._serialize()})"
