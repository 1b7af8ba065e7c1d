"""Torch backend: process-group setup over RCCL (reference: ``python/ray/train/torch/config.py``).

GPU workers on one node are given the union of the group's GPUs in ``HIP_VISIBLE_DEVICES``
(ordered, each worker selecting its own by index) before HIP initialises, so RCCL sees every peer
and uses xGMI peer-to-peer paths between the ranks instead of staging through host memory.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from datetime import timedelta
from typing import Optional

from ..backend import Backend, BackendConfig, _assign_ranks, _node_info_fn


@dataclass
class TorchConfig(BackendConfig):
    backend: Optional[str] = None
    init_method: str = "tcp"
    timeout_s: int = 1800

    @property
    def backend_cls(self):
        return _TorchBackend


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rccl_pg_options(backend):
    """RCCL process-group options: collectives run on a HIGH-PRIORITY HIP stream, so the gradient
    all-reduce kernels issued during backward are dispatched ahead of the queued GEMM workgroups
    instead of waiting behind them (comm/compute overlap over xGMI). ``RCA_RCCL_HIGH_PRIORITY=0``
    restores the default stream priority."""
    if backend != "nccl" or os.environ.get("RCA_RCCL_HIGH_PRIORITY", "1") == "0":
        return None
    import torch.distributed as dist

    try:
        o = dist.ProcessGroupNCCL.Options()
        o.is_high_priority_stream = True
        return o
    except Exception:  # noqa  (no NCCL/RCCL in this torch build)
        return None


def _setup_torch_process_group(rank, world_size, local_rank, local_world_size, node_rank, device_index, visible,
                               backend, addr, port, timeout_s):
    env = {"MASTER_ADDR": addr, "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world_size),
           "LOCAL_RANK": str(local_rank), "LOCAL_WORLD_SIZE": str(local_world_size), "NODE_RANK": str(node_rank),
           "GROUP_RANK": str(node_rank)}
    os.environ.update(env)
    if device_index is not None:
        os.environ["RCA_TRAIN_DEVICE_INDEX"] = str(device_index)
        if visible:
            os.environ["HIP_VISIBLE_DEVICES"] = ",".join(visible)
    import torch
    import torch.distributed as dist

    kw = {}
    if device_index is not None and torch.cuda.is_available():
        torch.cuda.set_device(device_index)
        kw["device_id"] = torch.device("cuda", device_index)
    # a process group is formed even for world_size 1 so train loops can call collectives
    # (barrier / all_reduce of metrics) unconditionally
    if dist.is_initialized():
        dist.destroy_process_group()
    opts = rccl_pg_options(backend)
    if opts is not None:
        kw["pg_options"] = opts
    dist.init_process_group(backend=backend, init_method=f"tcp://{addr}:{port}", rank=rank,
                            world_size=world_size, timeout=timedelta(seconds=timeout_s), **kw)
    return True


class _TorchBackend(Backend):
    share_cuda_visible_devices = True

    def on_start(self, worker_group, backend_config: TorchConfig, scaling_config=None):
        from ..._private.worker import get

        infos = _assign_ranks(worker_group.execute(_node_info_fn))
        use_gpu = bool(scaling_config is not None and scaling_config.num_gpus_per_worker)
        backend = backend_config.backend or ("nccl" if use_gpu else "gloo")
        per_node = {}
        for inf in infos:
            per_node.setdefault(inf["node_id"], [])
            for v in inf["visible"]:
                if v not in per_node[inf["node_id"]]:
                    per_node[inf["node_id"]].append(v)
        for v in per_node.values():
            v.sort(key=lambda x: int(x) if x.isdigit() else x)
        port = worker_group.execute_single(0, _free_port)
        refs = []
        n = len(infos)
        for i, (w, inf) in enumerate(zip(worker_group.workers, infos)):
            dev = None
            vis = None
            if use_gpu and inf["visible"]:
                vis = per_node[inf["node_id"]]
                dev = vis.index(inf["visible"][0])
            elif use_gpu:
                dev = 0
            inf["device_index"] = dev
            refs.append(w.execute.remote(_setup_torch_process_group, i, n, inf["local_rank"], inf["local_world_size"],
                                         inf["node_rank"], dev, vis, backend, "127.0.0.1", port,
                                         backend_config.timeout_s))
        get(refs)
        return infos
