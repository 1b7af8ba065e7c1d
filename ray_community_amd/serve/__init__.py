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


__all__ = ["deployment", "run", "delete", "shutdown", "start", "status", "ingress", "batch", "multiplexed",
           "get_multiplexed_model_id", "get_replica_context", "get_app_handle", "get_deployment_handle",
           "Deployment", "Application", "DeploymentHandle", "DeploymentResponse", "DeploymentResponseGenerator",
           "AutoscalingConfig"]
