"""Backend interface (reference: ``python/ray/train/backend.py``)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class BackendConfig:
    @property
    def backend_cls(self):
        return Backend


class Backend:
    share_cuda_visible_devices: bool = False

    def on_start(self, worker_group, backend_config, scaling_config=None):
        infos = worker_group.execute(_node_info_fn)
        return _assign_ranks(infos)

    def on_shutdown(self, worker_group, backend_config):
        pass

    def on_training_start(self, worker_group, backend_config):
        pass


def _node_info_fn():
    import os

    import ray_community_amd as ray

    vis = os.environ.get("HIP_VISIBLE_DEVICES", "")
    return {"node_id": ray.get_runtime_context().get_node_id(), "pid": os.getpid(),
            "visible": [v for v in vis.split(",") if v != ""], "gpu_ids": ray.get_gpu_ids()}


def _assign_ranks(infos):
    node_order = []
    for inf in infos:
        if inf["node_id"] not in node_order:
            node_order.append(inf["node_id"])
    counters = {}
    for inf in infos:
        nid = inf["node_id"]
        inf["local_rank"] = counters.get(nid, 0)
        counters[nid] = inf["local_rank"] + 1
        inf["node_rank"] = node_order.index(nid)
    for inf in infos:
        inf["local_world_size"] = counters[inf["node_id"]]
    return infos
