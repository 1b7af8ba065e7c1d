"""Declarative Serve config (reference: ``python/ray/serve/schema.py`` -- ``ServeDeploySchema`` :724,
``ServeApplicationSchema`` :511, ``DeploymentSchema`` :271).

A config file describes every application of a Serve instance: where its code lives
(``import_path`` to a bound ``Application`` or to a builder function taking ``args``), the
``runtime_env`` its replicas run in, and per-deployment overrides of the options written in the
code. ``serve deploy`` / ``PUT /api/serve/applications/`` apply one declaratively: applications
not in the config are deleted, changed ones are updated in place (``num_replicas`` /
``user_config`` changes do not restart replicas), new ones are started.

Models are pydantic (v2) so a config validates with clear errors before anything is deployed;
``ServeDeploySchema.model_validate(yaml.safe_load(f))`` is the parse path for files and for the
REST body alike.
"""
from __future__ import annotations

from enum import Enum
from typing import Any, Dict, List, Optional, Union

from pydantic import BaseModel, ConfigDict, Field, field_validator, model_validator


class ProxyLocation(str, Enum):
    Disabled = "Disabled"
    HeadOnly = "HeadOnly"
    EveryNode = "EveryNode"


class _Model(BaseModel):
    model_config = ConfigDict(extra="forbid", populate_by_name=True)

    def to_dict(self, exclude_unset: bool = True) -> Dict[str, Any]:
        return self.model_dump(mode="json", exclude_unset=exclude_unset)


class LoggingConfig(_Model):
    encoding: str = "TEXT"
    log_level: Union[int, str] = "INFO"
    logs_dir: Optional[str] = None
    enable_access_log: bool = True

    @field_validator("encoding")
    @classmethod
    def valid_encoding_format(cls, v):
        if v not in ("TEXT", "JSON"):
            raise ValueError(f"Got '{v}' for encoding. Encoding must be one of ('TEXT', 'JSON').")
        return v

    @field_validator("log_level")
    @classmethod
    def valid_log_level(cls, v):
        import logging

        if isinstance(v, int):
            if v not in (logging.DEBUG, logging.INFO, logging.WARNING, logging.ERROR, logging.CRITICAL, logging.NOTSET):
                raise ValueError(f"Got '{v}' for log_level: not a logging level")
            return logging.getLevelName(v)
        if v not in ("DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL", "NOTSET"):
            raise ValueError(f'Got "{v}" for log_level. log_level must be one of DEBUG, INFO, WARNING, ERROR, '
                             f"CRITICAL, NOTSET.")
        return v


class RayActorOptionsSchema(_Model):
    runtime_env: Dict[str, Any] = Field(default_factory=dict)
    num_cpus: Optional[float] = None
    num_gpus: Optional[float] = None
    memory: Optional[float] = None
    object_store_memory: Optional[float] = None
    resources: Dict[str, float] = Field(default_factory=dict)
    accelerator_type: Optional[str] = None

    @field_validator("num_cpus", "num_gpus", "memory", "object_store_memory")
    @classmethod
    def _non_negative(cls, v):
        if v is not None and v < 0:
            raise ValueError("must be >= 0")
        return v


class DeploymentSchema(_Model):
    """Overrides for one deployment of an application (only the fields that are set apply)."""

    name: str
    num_replicas: Optional[Union[int, str]] = None
    route_prefix: Optional[str] = None
    max_ongoing_requests: Optional[int] = None
    max_concurrent_queries: Optional[int] = None
    max_queued_requests: Optional[int] = None
    user_config: Optional[Dict[str, Any]] = None
    autoscaling_config: Optional[Dict[str, Any]] = None
    graceful_shutdown_wait_loop_s: Optional[float] = None
    graceful_shutdown_timeout_s: Optional[float] = None
    health_check_period_s: Optional[float] = None
    health_check_timeout_s: Optional[float] = None
    ray_actor_options: Optional[RayActorOptionsSchema] = None
    placement_group_bundles: Optional[List[Dict[str, float]]] = None
    placement_group_strategy: Optional[str] = None
    max_replicas_per_node: Optional[int] = None
    logging_config: Optional[LoggingConfig] = None

    @field_validator("num_replicas")
    @classmethod
    def _replicas(cls, v):
        if isinstance(v, str) and v != "auto":
            raise ValueError('num_replicas must be a positive integer or "auto"')
        if isinstance(v, int) and v < 0:
            raise ValueError("num_replicas must be >= 0")
        return v

    @model_validator(mode="after")
    def _replicas_vs_autoscaling(self):
        if self.autoscaling_config is not None and self.num_replicas not in (None, "auto"):
            raise ValueError("Manually setting num_replicas is not allowed when autoscaling_config is provided.")
        return self


class ServeApplicationSchema(_Model):
    name: str = "default"
    route_prefix: Optional[str] = "/"
    import_path: str
    runtime_env: Dict[str, Any] = Field(default_factory=dict)
    host: str = "0.0.0.0"
    port: int = 8000
    deployments: List[DeploymentSchema] = Field(default_factory=list)
    args: Dict[str, Any] = Field(default_factory=dict)
    logging_config: Optional[LoggingConfig] = None

    @field_validator("import_path")
    @classmethod
    def _import_path(cls, v):
        if ":" in v:
            mod, attr = v.split(":", 1)
            if not mod or not attr or ":" in attr:
                raise ValueError(f'import_path "{v}" must be "module:attribute" or "module.attribute"')
        elif "." not in v:
            raise ValueError(f'import_path "{v}" must be "module:attribute" or "module.attribute"')
        return v

    @field_validator("route_prefix")
    @classmethod
    def _prefix(cls, v):
        if v is not None and (not v.startswith("/") or (len(v) > 1 and v.endswith("/"))):
            raise ValueError(f'route_prefix "{v}" must start with "/" and not end with "/"')
        return v

    @model_validator(mode="after")
    def _unique_deployments(self):
        names = [d.name for d in self.deployments]
        dup = {n for n in names if names.count(n) > 1}
        if dup:
            raise ValueError(f"duplicate deployment names in application {self.name!r}: {sorted(dup)}")
        return self


class HTTPOptionsSchema(_Model):
    host: str = "0.0.0.0"
    port: int = 8000
    root_path: str = ""
    request_timeout_s: Optional[float] = None
    keep_alive_timeout_s: int = 5


class gRPCOptionsSchema(_Model):  # noqa: N801 (reference name)
    port: int = 9000
    grpc_servicer_functions: List[str] = Field(default_factory=list)


class ServeDeploySchema(_Model):
    proxy_location: ProxyLocation = ProxyLocation.EveryNode
    http_options: HTTPOptionsSchema = Field(default_factory=HTTPOptionsSchema)
    grpc_options: gRPCOptionsSchema = Field(default_factory=gRPCOptionsSchema)
    logging_config: Optional[LoggingConfig] = None
    applications: List[ServeApplicationSchema] = Field(default_factory=list)
    target_capacity: Optional[float] = None

    @model_validator(mode="after")
    def _unique(self):
        names = [a.name for a in self.applications]
        dup = {n for n in names if names.count(n) > 1}
        if dup:
            raise ValueError(f"duplicate application names: {sorted(dup)}")
        prefixes = [a.route_prefix for a in self.applications if a.route_prefix is not None]
        dupp = {p for p in prefixes if prefixes.count(p) > 1}
        if dupp:
            raise ValueError(f"duplicate route prefixes: {sorted(dupp)}")
        return self


def parse_config(obj: Union[str, Dict[str, Any]]) -> ServeDeploySchema:
    """A ``ServeDeploySchema`` from a YAML/JSON file path, a YAML string or a dict. A file holding
    a single application (``import_path`` at the top level) is accepted as a one-app config."""
    import os

    import yaml

    if isinstance(obj, str):
        if os.path.exists(obj):
            with open(obj) as f:
                obj = yaml.safe_load(f)
        else:
            obj = yaml.safe_load(obj)
    obj = dict(obj or {})
    if "import_path" in obj and "applications" not in obj:
        obj = {"applications": [obj]}
    return ServeDeploySchema.model_validate(obj)


# ============================================================================ status / details models
# (reference schema.py: ServeStatus, ApplicationStatusOverview, DeploymentStatusOverview and the
# ServeInstanceDetails tree the dashboard's GET /api/serve/applications/ returns)
class EncodingType(str, Enum):
    TEXT = "TEXT"
    JSON = "JSON"


class _Details(BaseModel):
    model_config = ConfigDict(extra="allow", populate_by_name=True)

    def to_dict(self) -> Dict[str, Any]:
        return self.model_dump(mode="json")


class DeploymentStatusOverview(_Details):
    status: Optional[str] = None
    status_trigger: Optional[str] = None
    replica_states: Dict[str, int] = Field(default_factory=dict)
    message: str = ""


class ApplicationStatusOverview(_Details):
    status: Optional[str] = None
    message: str = ""
    last_deployed_time_s: Optional[float] = None
    deployments: Dict[str, DeploymentStatusOverview] = Field(default_factory=dict)


class ServeStatus(_Details):
    proxies: Dict[str, str] = Field(default_factory=dict)
    applications: Dict[str, ApplicationStatusOverview] = Field(default_factory=dict)
    target_capacity: Optional[float] = None


class ServeActorDetails(_Details):
    node_id: Optional[str] = None
    node_ip: Optional[str] = None
    actor_id: Optional[str] = None
    actor_name: Optional[str] = None
    worker_id: Optional[str] = None
    log_file_path: Optional[str] = None


class ReplicaDetails(ServeActorDetails):
    replica_id: str
    state: str
    pid: Optional[int] = None
    start_time_s: Optional[float] = None


class ProxyDetails(ServeActorDetails):
    status: str


class DeploymentDetails(_Details):
    name: str
    status: Optional[str] = None
    status_trigger: Optional[str] = None
    message: str = ""
    deployment_config: Dict[str, Any] = Field(default_factory=dict)
    target_num_replicas: Optional[int] = None
    replicas: List[ReplicaDetails] = Field(default_factory=list)


class ApplicationDetails(_Details):
    name: str
    route_prefix: Optional[str] = None
    docs_path: Optional[str] = None
    status: Optional[str] = None
    message: str = ""
    last_deployed_time_s: Optional[float] = None
    deployed_app_config: Optional[Dict[str, Any]] = None
    deployments: Dict[str, DeploymentDetails] = Field(default_factory=dict)


class ServeInstanceDetails(_Details):
    controller_info: Dict[str, Any] = Field(default_factory=dict)
    proxy_location: Optional[str] = None
    http_options: Optional[Dict[str, Any]] = None
    grpc_options: Optional[Dict[str, Any]] = None
    proxies: Dict[str, ProxyDetails] = Field(default_factory=dict)
    deploy_mode: str = "MULTI_APP"
    applications: Dict[str, ApplicationDetails] = Field(default_factory=dict)
    target_capacity: Optional[float] = None

    @staticmethod
    def get_empty_schema_dict() -> Dict[str, Any]:
        """The body of a Serve instance with nothing deployed."""
        return {"controller_info": {}, "proxies": {}, "applications": {}, "deploy_mode": "MULTI_APP",
                "target_capacity": None}

    def _get_status(self) -> ServeStatus:
        return ServeStatus(
            target_capacity=self.target_capacity,
            proxies={k: p.status for k, p in self.proxies.items()},
            applications={name: ApplicationStatusOverview(
                status=a.status, message=a.message, last_deployed_time_s=a.last_deployed_time_s,
                deployments={dn: DeploymentStatusOverview(
                    status=d.status, message=d.message,
                    replica_states=_count_states(d.replicas)) for dn, d in a.deployments.items()})
                for name, a in self.applications.items()})


def _count_states(replicas) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for r in replicas:
        out[r.state] = out.get(r.state, 0) + 1
    return out
