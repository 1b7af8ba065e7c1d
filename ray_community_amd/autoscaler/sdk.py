"""``request_resources`` (reference: ``python/ray/autoscaler/sdk/sdk.py``): command the
autoscaler to keep capacity for the given shapes regardless of current load; each call replaces
the previous request (``request_resources()`` clears it)."""
from __future__ import annotations

import json
from typing import Dict, List, Optional


def request_resources(num_cpus: Optional[int] = None, bundles: Optional[List[Dict[str, float]]] = None) -> None:
    from .._private.core_worker import global_core

    shapes: List[Dict[str, float]] = []
    if num_cpus:
        shapes += [{"CPU": 1.0}] * int(num_cpus)
    for b in bundles or []:
        shapes.append({k: float(v) for k, v in b.items() if v})
    global_core().client.call("kv_put", "__autoscaler_resource_request__", json.dumps(shapes).encode(), True,
                              "autoscaler")


# ---------------------------------------------------------------------------- cluster launcher
# The reference's cluster launcher provisions cloud VMs from a cluster YAML (AWS / GCP / Azure /
# k8s node providers). Nodes here are started with ``python -m ray start`` (or virtual nodes via
# ``cluster_utils`` / the autoscaler's local provider); the launcher entry points say so.
def _launcher(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"autoscaler.sdk.{name}: cloud cluster launching is not available; start nodes "
                                  "with `python -m ray_community_amd start --head` / `start --address=...`")
    f.__name__ = name
    return f


create_or_update_cluster = _launcher("create_or_update_cluster")
teardown_cluster = _launcher("teardown_cluster")
run_on_cluster = _launcher("run_on_cluster")
rsync = _launcher("rsync")
get_head_node_ip = _launcher("get_head_node_ip")
get_worker_node_ips = _launcher("get_worker_node_ips")
get_docker_host_mount_location = _launcher("get_docker_host_mount_location")


def fillout_defaults(config: Dict) -> Dict:
    """A cluster config with the defaults filled in (local provider, one head node type)."""
    out = dict(config or {})
    out.setdefault("cluster_name", "default")
    out.setdefault("max_workers", 2)
    out.setdefault("upscaling_speed", 1.0)
    out.setdefault("idle_timeout_minutes", 5)
    out.setdefault("provider", {"type": "local"})
    out.setdefault("available_node_types", {"head": {"resources": {}, "node_config": {}}})
    out.setdefault("head_node_type", next(iter(out["available_node_types"])))
    return out


def bootstrap_config(config: Dict, no_config_cache: bool = False) -> Dict:
    return fillout_defaults(config)


def configure_logging(log_style: Optional[str] = None, color_mode: Optional[str] = None,
                      verbosity: Optional[int] = None):
    import logging

    logging.getLogger("ray_community_amd.autoscaler").setLevel(
        logging.DEBUG if (verbosity or 0) > 1 else logging.INFO)


_callbacks = {}


def register_callback_handler(event_name: str, callback) -> None:
    """Register ``callback(event_data)`` for an autoscaler event name."""
    _callbacks.setdefault(event_name, []).append(callback)
