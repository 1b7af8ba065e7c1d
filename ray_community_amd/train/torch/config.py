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

    @property
    def train_func_context(self):
        """Context manager the training function runs under on each worker (reference
        ``TorchConfig.train_func_context``): it makes the worker's HIP device the current device."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            import torch

            if torch.cuda.is_available():
                from .train_loop_utils import get_device

                dev = get_device()
                if getattr(dev, "type", None) == "cuda":
                    with torch.cuda.device(dev):
                        yield
                    return
            yield

        return ctx


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


def plan_devices(infos, use_gpu: bool):
    """Per worker (device index, visible list): GPU workers on one node all get the node's union of
    the group's GPUs in ``HIP_VISIBLE_DEVICES`` (sorted) and select their own by its index in it,
    so RCCL sees every peer and uses xGMI peer paths. Pure function of the workers' reports."""
    per_node = {}
    for inf in infos:
        per_node.setdefault(inf["node_id"], [])
        for v in inf["visible"]:
            if v not in per_node[inf["node_id"]]:
                per_node[inf["node_id"]].append(v)
    for v in per_node.values():
        v.sort(key=lambda x: int(x) if x.isdigit() else x)
    plan = []
    for inf in infos:
        if use_gpu and inf["visible"]:
            vis = list(per_node[inf["node_id"]])
            plan.append((vis.index(inf["visible"][0]), vis))
        elif use_gpu:
            plan.append((0, None))
        else:
            plan.append((None, None))
    if use_gpu:  # one GPU per worker on a node: no two workers may select the same device
        seen = {}
        for inf, (dev, vis) in zip(infos, plan):
            if vis is None:
                continue
            key = (inf["node_id"], dev)
            if key in seen:
                raise RuntimeError(f"two workers on node {inf['node_id']} would both use GPU {vis[dev]} "
                                   f"(HIP_VISIBLE_DEVICES {inf['visible']} and {seen[key]})")
            seen[key] = inf["visible"]
    return plan


def _setup_torch_process_group(rank, world_size, local_rank, local_world_size, node_rank, device_index, visible,
                               backend, addr, port, timeout_s):
    """Join the group's process group. GPU workers must set ``HIP_VISIBLE_DEVICES`` before HIP
    initialises in this process: if something already initialised it with another device set,
    the env change would be silently ignored and the worker would pick the wrong GPU, so that
    case -- and any device-count / backend / world-size mismatch -- fails loudly here instead of
    degrading the run. Returns what was actually set up (backend, world size, RCCL version)."""
    import sys

    env = {"MASTER_ADDR": addr, "MASTER_PORT": str(port), "RANK": str(rank), "WORLD_SIZE": str(world_size),
           "LOCAL_RANK": str(local_rank), "LOCAL_WORLD_SIZE": str(local_world_size), "NODE_RANK": str(node_rank),
           "GROUP_RANK": str(node_rank)}
    os.environ.update(env)
    if device_index is not None:
        os.environ["RCA_TRAIN_DEVICE_INDEX"] = str(device_index)
        if visible:
            want = ",".join(visible)
            tmod = sys.modules.get("torch")
            if (tmod is not None and tmod.cuda.is_initialized()
                    and os.environ.get("HIP_VISIBLE_DEVICES", "") != want):
                raise RuntimeError(
                    f"rank {rank}: HIP was initialised in this worker before the process group was set up "
                    f"(HIP_VISIBLE_DEVICES={os.environ.get('HIP_VISIBLE_DEVICES')!r}); the group needs {want!r}. "
                    "Do not touch the GPU before TorchTrainer starts the training function.")
            os.environ["HIP_VISIBLE_DEVICES"] = want
    import torch
    import torch.distributed as dist

    kw = {}
    if device_index is not None and backend == "nccl":
        if not torch.cuda.is_available():
            raise RuntimeError(f"rank {rank}: a GPU worker sees no GPU (HIP_VISIBLE_DEVICES="
                               f"{os.environ.get('HIP_VISIBLE_DEVICES')!r})")
        n = torch.cuda.device_count()
        if visible and n != len(visible):
            raise RuntimeError(f"rank {rank}: torch sees {n} GPU(s) but HIP_VISIBLE_DEVICES lists {len(visible)} "
                               f"({visible})")
        if not 0 <= device_index < n:
            raise RuntimeError(f"rank {rank}: device index {device_index} outside the {n} visible GPU(s)")
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
    got_backend, got_world = dist.get_backend(), dist.get_world_size()
    if got_backend != backend or got_world != world_size:
        raise RuntimeError(f"rank {rank}: process group is {got_backend} x {got_world}, expected {backend} x "
                           f"{world_size}")
    return group_info(device_index)


def group_info(device_index=None):
    """Backend, world size, RCCL version and device of the current process group (bench JSON)."""
    import torch
    import torch.distributed as dist

    out = {"backend": dist.get_backend() if dist.is_initialized() else None,
           "world_size": dist.get_world_size() if dist.is_initialized() else 1, "device_index": device_index,
           "rccl_version": None, "hip_visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")}
    try:
        if torch.cuda.is_available():
            v = torch.cuda.nccl.version()
            out["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa
        pass
    return out


class _TorchBackend(Backend):
    share_cuda_visible_devices = True

    def on_start(self, worker_group, backend_config: TorchConfig, scaling_config=None):
        from ..._private.worker import get

        infos = _assign_ranks(worker_group.execute(_node_info_fn))
        use_gpu = bool(scaling_config is not None and scaling_config.num_gpus_per_worker)
        backend = backend_config.backend or ("nccl" if use_gpu else "gloo")
        plan = plan_devices(infos, use_gpu)
        port = worker_group.execute_single(0, _free_port)
        refs = []
        n = len(infos)
        for i, (w, inf, (dev, vis)) in enumerate(zip(worker_group.workers, infos, plan)):
            inf["device_index"] = dev
            refs.append(w.execute.remote(_setup_torch_process_group, i, n, inf["local_rank"], inf["local_world_size"],
                                         inf["node_rank"], dev, vis, backend, "127.0.0.1", port,
                                         backend_config.timeout_s))
        for inf, gi in zip(infos, get(refs)):
            inf["group"] = gi
        return infos
