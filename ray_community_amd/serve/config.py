"""Serve configuration objects (reference: ``python/ray/serve/config.py``: ``HTTPOptions``,
``gRPCOptions``, ``AutoscalingConfig``, ``DeploymentMode`` / ``ProxyLocation``)."""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Callable, List, Optional, Union


class DeploymentMode(str, Enum):
    NoServer = "NoServer"
    HeadOnly = "HeadOnly"
    EveryNode = "EveryNode"


@dataclass
class AutoscalingConfig:
    """Replica autoscaling (reference ``AutoscalingConfig``): the controller scales between
    ``min_replicas`` and ``max_replicas`` to keep ``target_ongoing_requests`` per replica, after
    ``upscale_delay_s`` / ``downscale_delay_s`` of sustained pressure; the smoothing factors damp
    each decision."""
    min_replicas: int = 1
    initial_replicas: Optional[int] = None
    max_replicas: int = 1
    target_ongoing_requests: float = 2.0
    metrics_interval_s: float = 10.0
    look_back_period_s: float = 30.0
    smoothing_factor: float = 1.0
    upscale_smoothing_factor: Optional[float] = None
    downscale_smoothing_factor: Optional[float] = None
    upscaling_factor: Optional[float] = None
    downscaling_factor: Optional[float] = None
    downscale_delay_s: float = 600.0
    upscale_delay_s: float = 30.0
    target_num_ongoing_requests_per_replica: Optional[float] = None  # pre-2.10 name

    def __post_init__(self):
        if self.target_num_ongoing_requests_per_replica is not None:
            self.target_ongoing_requests = self.target_num_ongoing_requests_per_replica
        if self.min_replicas < 0 or self.max_replicas < max(1, self.min_replicas):
            raise ValueError("need 0 <= min_replicas <= max_replicas and max_replicas >= 1")
        if self.initial_replicas is not None and not (self.min_replicas <= self.initial_replicas <= self.max_replicas):
            raise ValueError("initial_replicas must lie in [min_replicas, max_replicas]")

    def get_upscaling_factor(self) -> float:
        return self.upscaling_factor or self.upscale_smoothing_factor or self.smoothing_factor

    def get_downscaling_factor(self) -> float:
        return self.downscaling_factor or self.downscale_smoothing_factor or self.smoothing_factor

    def dict(self):
        return {k: v for k, v in self.__dict__.items()}


class HTTPOptions:
    """HTTP proxy options for ``serve.start(http_options=HTTPOptions(...))``: ``host`` / ``port``
    bind the proxy, ``request_timeout_s`` bounds each HTTP request (408), ``keep_alive_timeout_s``
    is the server's keep-alive, ``root_path`` the ASGI root path (serving behind a path-prefixing
    reverse proxy) and ``root_url`` the externally visible URL. ``location`` is informational here:
    one proxy runs on the head node. ``middlewares`` / ``num_cpus`` are the reference's deprecated
    fields (accepted, with a warning)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 8000, root_path: str = "", location: str = "HeadOnly",
                 request_timeout_s: Optional[float] = None, keep_alive_timeout_s: int = 5, root_url: str = "",
                 middlewares: Optional[List[Any]] = None, num_cpus: int = 0, ssl_keyfile=None, ssl_certfile=None,
                 **kw):
        self.host, self.port, self.root_path = host, port, root_path
        self.location = location.value if isinstance(location, Enum) else location
        self.request_timeout_s = request_timeout_s
        self.keep_alive_timeout_s = keep_alive_timeout_s
        self.root_url = root_url
        self.middlewares = list(middlewares or [])
        self.num_cpus = num_cpus
        self.ssl_keyfile, self.ssl_certfile = ssl_keyfile, ssl_certfile
        self.warn_for_middlewares()
        self.warn_for_num_cpus()

    def location_backfill_no_server(self):
        if self.location in (None, "NoServer"):
            self.location = "NoServer"
        return self

    def warn_for_middlewares(self):
        if self.middlewares:
            import warnings

            warnings.warn("HTTPOptions.middlewares is deprecated: wrap the app with ASGI middleware in the "
                          "ingress deployment instead", DeprecationWarning, stacklevel=3)
        return self

    def warn_for_num_cpus(self):
        if self.num_cpus:
            import warnings

            warnings.warn("HTTPOptions.num_cpus is deprecated and ignored", DeprecationWarning, stacklevel=3)
        return self

    def __repr__(self):
        return f"HTTPOptions(host={self.host!r}, port={self.port}, root_path={self.root_path!r})"


@dataclass
class gRPCOptions:
    """``grpc_servicer_functions``: generated ``add_<Service>Servicer_to_server`` functions (or
    their import paths) whose methods the gRPC proxy serves."""
    port: int = 9000
    host: str = "127.0.0.1"
    grpc_servicer_functions: List[Union[str, Callable]] = field(default_factory=list)

    @property
    def grpc_servicer_func_callable(self) -> List[Callable]:
        import importlib

        out = []
        for f in self.grpc_servicer_functions:
            if isinstance(f, str):
                mod, _, name = f.rpartition(".")
                f = getattr(importlib.import_module(mod), name)
            out.append(f)
        return out

from .schema import ProxyLocation  # noqa: E402,F401  (reference exports it from serve.config too)
