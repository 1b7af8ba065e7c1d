"""Collective communication among actors/tasks (reference: ``python/ray/util/collective/collective.py``).

MI355X-native backends:
  * ``"nccl"`` / ``"rccl"`` -> a dedicated ``ProcessGroupNCCL`` (RCCL on ROCm) over xGMI for GPU tensors;
  * ``"gloo"`` -> ``ProcessGroupGloo`` for CPU tensors.
Each group is an independent c10d process group built on a PrefixStore over a FileStore in the
session directory (rendezvous needs no ports), so any number of groups with arbitrary
membership can coexist in one process alongside the default torch.distributed group.
``create_collective_group`` (declarative, from the driver) records membership in the head's KV;
members lazily join on their first collective call.
"""
from __future__ import annotations

import os
import threading
import time
from datetime import timedelta
from typing import Dict, List, Optional

from .types import Backend, ReduceOp

_GROUPS: Dict[str, "CollectiveGroup"] = {}
_LOCK = threading.Lock()
_KV_NS = "collective"


def _torch():
    import torch
    import torch.distributed as dist

    return torch, dist


def _reduce_op(op):
    _, dist = _torch()
    return {ReduceOp.SUM: dist.ReduceOp.SUM, ReduceOp.PRODUCT: dist.ReduceOp.PRODUCT, ReduceOp.MIN: dist.ReduceOp.MIN,
            ReduceOp.MAX: dist.ReduceOp.MAX, ReduceOp.AVG: getattr(dist.ReduceOp, "AVG", dist.ReduceOp.SUM)}[op]


def _session_dir():
    from ..._private.core_worker import _core

    if _core is not None and _core.session_dir:
        return _core.session_dir
    return os.environ.get("RCA_SESSION_DIR", "/tmp/rca")


class CollectiveGroup:
    def __init__(self, world_size: int, rank: int, backend: str, group_name: str, timeout_s: float = 1800.0):
        torch, dist = _torch()
        self.world_size = world_size
        self.rank = rank
        self.backend = Backend(backend)
        self.group_name = group_name
        base = os.path.join(_session_dir(), "collective")
        os.makedirs(base, exist_ok=True)
        path = os.path.join(base, f"{group_name}.store")
        self._store = dist.PrefixStore(group_name, dist.FileStore(path, world_size))
        to = timedelta(seconds=timeout_s)
        if self.backend == Backend.NCCL:
            if not torch.cuda.is_available():
                raise RuntimeError("the nccl/rccl collective backend needs a GPU in this process")
            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = to
            self.pg = dist.ProcessGroupNCCL(self._store, rank, world_size, opts)
        else:
            self.pg = dist.ProcessGroupGloo(self._store, rank, world_size, to)

    # ---------------------------------------------------------------- ops
    def allreduce(self, tensors, op=ReduceOp.SUM):
        _, dist = _torch()
        o = dist.AllreduceOptions()
        o.reduceOp = _reduce_op(op)
        self.pg.allreduce(tensors, o).wait()
        if op == ReduceOp.AVG and not hasattr(dist.ReduceOp, "AVG"):
            for t in tensors:
                t.div_(self.world_size)

    def barrier(self):
        _, dist = _torch()
        if self.backend == Backend.NCCL:
            torch, _ = _torch()
            t = torch.zeros(1, device="cuda")
            self.allreduce([t])
            torch.cuda.synchronize()
        else:
            self.pg.barrier(dist.BarrierOptions()).wait()

    def reduce(self, tensors, dst_rank=0, op=ReduceOp.SUM):
        _, dist = _torch()
        o = dist.ReduceOptions()
        o.reduceOp = _reduce_op(op)
        o.rootRank = dst_rank
        o.rootTensor = 0
        self.pg.reduce(tensors, o).wait()

    def broadcast(self, tensors, src_rank=0):
        _, dist = _torch()
        o = dist.BroadcastOptions()
        o.rootRank = src_rank
        o.rootTensor = 0
        self.pg.broadcast(tensors, o).wait()

    def allgather(self, tensor_lists, tensors):
        _, dist = _torch()
        from torch._C._distributed_c10d import AllgatherOptions

        self.pg.allgather(tensor_lists, tensors, AllgatherOptions()).wait()

    def reducescatter(self, tensors, tensor_lists, op=ReduceOp.SUM):
        torch, dist = _torch()
        if self.backend == Backend.GLOO:
            # gloo has no reduce_scatter: allreduce the stacked input, keep this rank's slice
            for out, inputs in zip(tensors, tensor_lists):
                flat = torch.stack(list(inputs))
                self.allreduce([flat], op)
                out.copy_(flat[self.rank])
            return
        o = dist.ReduceScatterOptions()
        o.reduceOp = _reduce_op(op)
        self.pg.reduce_scatter(tensors, tensor_lists, o).wait()

    def alltoall(self, output, input):
        _, dist = _torch()
        self.pg.alltoall_base(output, input, [], [], dist.AllToAllOptions()).wait()

    def send(self, tensors, dst_rank, tag=0):
        self.pg.send(tensors, dst_rank, tag).wait()

    def recv(self, tensors, src_rank, tag=0):
        self.pg.recv(tensors, src_rank, tag).wait()

    def destroy(self):
        try:
            if hasattr(self.pg, "shutdown"):
                self.pg.shutdown()
        except Exception:
            pass


def _kv():
    from ...experimental import internal_kv

    return internal_kv


def init_collective_group(world_size: int, rank: int, backend=Backend.NCCL, group_name: str = "default"):
    """Initialize this process as ``rank`` of ``group_name`` (called inside every member)."""
    if not (0 <= rank < world_size):
        raise ValueError(f"rank {rank} out of range for world_size {world_size}")
    with _LOCK:
        if group_name in _GROUPS:
            raise RuntimeError(f"Trying to initialize a group twice: {group_name}")
        _GROUPS[group_name] = CollectiveGroup(world_size, rank, backend, group_name)


def create_collective_group(actors, world_size: int, ranks: List[int], backend=Backend.NCCL,
                            group_name: str = "default"):
    """Declare a group from the driver; each actor joins lazily on its first collective call."""
    import pickle

    if len(actors) != world_size or len(ranks) != world_size:
        raise ValueError("actors/ranks must have world_size entries")
    if sorted(ranks) != list(range(world_size)):
        raise ValueError("ranks must be a permutation of range(world_size)")
    ids = [a._actor_id for a in actors]
    _kv()._internal_kv_put(f"info_{group_name}", pickle.dumps({"ids": ids, "world_size": world_size,
                                                                   "ranks": ranks, "backend": str(Backend(backend))}),
                           namespace=_KV_NS)


def _group(group_name: str) -> CollectiveGroup:
    g = _GROUPS.get(group_name)
    if g is not None:
        return g
    import pickle

    from ..._private.worker import _core

    info = _kv()._internal_kv_get(f"info_{group_name}", namespace=_KV_NS)
    if info is None:
        raise RuntimeError(f"The collective group '{group_name}' is not initialized in this process.")
    info = pickle.loads(info)
    me = _core().actor_id
    if me not in info["ids"]:
        raise RuntimeError(f"this actor is not a member of collective group '{group_name}'")
    rank = info["ranks"][info["ids"].index(me)]
    init_collective_group(info["world_size"], rank, info["backend"], group_name)
    return _GROUPS[group_name]


def is_group_initialized(group_name: str = "default") -> bool:
    return group_name in _GROUPS


def destroy_collective_group(group_name: str = "default"):
    with _LOCK:
        g = _GROUPS.pop(group_name, None)
    if g is not None:
        g.destroy()


def get_rank(group_name: str = "default") -> int:
    g = _GROUPS.get(group_name)
    return -1 if g is None else g.rank


def get_collective_group_size(group_name: str = "default") -> int:
    g = _GROUPS.get(group_name)
    return -1 if g is None else g.world_size


def allreduce(tensor, group_name: str = "default", op=ReduceOp.SUM):
    _group(group_name).allreduce([tensor], op)


# ---- multi-GPU-per-process variants (reference collective.py *_multigpu). A process here drives one
# GPU, but the list forms are kept: the local tensors are combined first, one collective runs on
# the combined tensor, and the result is copied back to every local tensor.
def nccl_available() -> bool:
    torch, dist = _torch()
    return bool(dist.is_nccl_available() and torch.cuda.is_available())


def gloo_available() -> bool:
    _, dist = _torch()
    return bool(dist.is_gloo_available())


def _local_sum(tensor_list, op=ReduceOp.SUM):
    acc = tensor_list[0].clone()
    for t in tensor_list[1:]:
        t = t.to(acc.device)
        if op in (ReduceOp.SUM, ReduceOp.AVG):
            acc += t
        elif op == ReduceOp.PRODUCT:
            acc *= t
        elif op == ReduceOp.MIN:
            acc = acc.minimum(t)
        elif op == ReduceOp.MAX:
            acc = acc.maximum(t)
    return acc


def allreduce_multigpu(tensor_list, group_name: str = "default", op=ReduceOp.SUM):
    tensor_list = list(tensor_list)
    acc = _local_sum(tensor_list, ReduceOp.SUM if op == ReduceOp.AVG else op)
    _group(group_name).allreduce([acc], op)
    if op == ReduceOp.AVG and len(tensor_list) > 1:
        acc /= len(tensor_list)
    for t in tensor_list:
        t.copy_(acc)


def reduce_multigpu(tensor_list, dst_rank: int = 0, dst_tensor: int = 0, group_name: str = "default",
                    op=ReduceOp.SUM):
    tensor_list = list(tensor_list)
    g = _group(group_name)
    acc = _local_sum(tensor_list, op)
    g.reduce([acc], dst_rank, op)
    if g.rank == dst_rank:
        tensor_list[dst_tensor].copy_(acc)


def broadcast_multigpu(tensor_list, src_rank: int = 0, src_tensor: int = 0, group_name: str = "default"):
    tensor_list = list(tensor_list)
    g = _group(group_name)
    t = tensor_list[src_tensor] if g.rank == src_rank else tensor_list[0]
    g.broadcast([t], src_rank)
    for x in tensor_list:
        if x is not t:
            x.copy_(t)


def allgather_multigpu(output_tensor_lists, input_tensor_list, group_name: str = "default"):
    """``output_tensor_lists[i][r * L + j]`` = local input ``j`` of rank ``r`` (L local tensors)."""
    g = _group(group_name)
    L = len(input_tensor_list)
    for j, inp in enumerate(input_tensor_list):
        parts = [inp.new_empty(inp.shape) for _ in range(g.world_size)]
        g.allgather([parts], [inp])
        for outs in output_tensor_lists:
            for r in range(g.world_size):
                outs[r * L + j].copy_(parts[r])


def reducescatter_multigpu(output_tensor_list, input_tensor_lists, group_name: str = "default",
                           op=ReduceOp.SUM):
    """``input_tensor_lists[i]`` holds ``world_size * L`` tensors; rank ``r`` receives the reductions
    of entries ``r * L .. r * L + L - 1`` into its ``output_tensor_list``."""
    g = _group(group_name)
    L = len(output_tensor_list)
    sums = [_local_sum([lst[k] for lst in input_tensor_lists], op) for k in range(g.world_size * L)]
    for j, out in enumerate(output_tensor_list):
        g.reducescatter([out], [[sums[r * L + j] for r in range(g.world_size)]], op)


def send_multigpu(tensor, dst_rank: int, dst_gpu_index: int = 0, group_name: str = "default", n_elements: int = 0):
    send(tensor if not n_elements else tensor.view(-1)[:n_elements], dst_rank, group_name)


def recv_multigpu(tensor, src_rank: int, src_gpu_index: int = 0, group_name: str = "default", n_elements: int = 0):
    recv(tensor if not n_elements else tensor.view(-1)[:n_elements], src_rank, group_name)


def barrier(group_name: str = "default"):
    _group(group_name).barrier()


def reduce(tensor, dst_rank: int = 0, group_name: str = "default", op=ReduceOp.SUM):
    _group(group_name).reduce([tensor], dst_rank, op)


def broadcast(tensor, src_rank: int = 0, group_name: str = "default"):
    _group(group_name).broadcast([tensor], src_rank)


def allgather(tensor_list, tensor, group_name: str = "default"):
    g = _group(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("tensor_list must have world_size entries")
    g.allgather([list(tensor_list)], [tensor])


def reducescatter(tensor, tensor_list, group_name: str = "default", op=ReduceOp.SUM):
    g = _group(group_name)
    if len(tensor_list) != g.world_size:
        raise RuntimeError("tensor_list must have world_size entries")
    g.reducescatter([tensor], [list(tensor_list)], op)


def alltoall(output, input, group_name: str = "default"):
    _group(group_name).alltoall(output, input)


def send(tensor, dst_rank: int, group_name: str = "default"):
    g = _group(group_name)
    if dst_rank == g.rank:
        raise RuntimeError("The destination rank must differ from the source rank.")
    g.send([tensor], dst_rank)


def recv(tensor, src_rank: int, group_name: str = "default"):
    g = _group(group_name)
    if src_rank == g.rank:
        raise RuntimeError("The source rank must differ from the destination rank.")
    g.recv([tensor], src_rank)


def synchronize(gpu_id: int = 0):
    torch, _ = _torch()
    torch.cuda.synchronize(gpu_id)
