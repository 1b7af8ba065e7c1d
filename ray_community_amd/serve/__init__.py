"""Ray Serve equivalent (reference: ``python/ray/serve``)."""
from .api import (Application, Deployment, delete, deployment, get_app_handle, get_deployment_handle,
                  get_replica_context, ingress, run, shutdown, start, status)
from .batching import batch
from .handle import DeploymentHandle, DeploymentResponse, DeploymentResponseGenerator
from .multiplex import get_multiplexed_model_id, multiplexed


class AutoscalingConfig:
    def __init__(self, min_replicas=1, max_replicas=1, target_ongoing_requests=2, initial_replicas=None,
                 upscale_delay_s=0.0, downscale_delay_s=5.0, **kw):
        self.min_replicas = min_replicas
        self.max_replicas = max_replicas
        self.target_ongoing_requests = target_ongoing_requests
        self.initial_replicas = initial_replicas
        self.upscale_delay_s = upscale_delay_s
        self.downscale_delay_s = downscale_delay_s


class HTTPOptions:
    """HTTP proxy options for ``serve.start(http_options=HTTPOptions(...))`` (reference
    ``serve/config.py``): ``host``/``port`` bind the proxy, ``request_timeout_s`` bounds each HTTP
    request (408), ``keep_alive_timeout_s`` is the server's keep-alive and ``root_path`` the ASGI
    root path (serving behind a path-prefixing reverse proxy). ``location`` is informational: one
    proxy runs on the head."""

    def __init__(self, host: str = "127.0.0.1", port: int = 8000, root_path: str = "", location: str = "HeadOnly",
                 request_timeout_s=None, keep_alive_timeout_s: int = 5, **kw):
        self.host, self.port, self.root_path, self.location = host, port, root_path, location
        self.request_timeout_s = request_timeout_s
        self.keep_alive_timeout_s = keep_alive_timeout_s


def _run(target, *, name: str = "default", route_prefix="/", _blocking: bool = True, **kw):
    """Internal alias of ``serve.run`` (the reference exports it for its own tooling)."""
    return run(target, name=name, route_prefix=route_prefix, blocking=False, **kw)


__all__ = ["deployment", "run", "delete", "shutdown", "start", "status", "ingress", "batch", "multiplexed",
           "get_multiplexed_model_id", "get_replica_context", "get_app_handle", "get_deployment_handle",
           "Deployment", "Application", "DeploymentHandle", "DeploymentResponse", "DeploymentResponseGenerator",
           "AutoscalingConfig", "HTTPOptions", "_run"]
