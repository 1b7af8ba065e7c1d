from .collective import (allgather, allgather_multigpu, allreduce, allreduce_multigpu, alltoall, barrier, broadcast,
                         broadcast_multigpu, create_collective_group, destroy_collective_group,
                         get_collective_group_size, get_rank, gloo_available, init_collective_group,
                         is_group_initialized, nccl_available, recv, recv_multigpu, reduce, reduce_multigpu,
                         reducescatter, reducescatter_multigpu, send, send_multigpu, synchronize)
from .types import Backend, ReduceOp

__all__ = ["init_collective_group", "create_collective_group", "destroy_collective_group", "is_group_initialized",
           "get_rank", "get_collective_group_size", "allreduce", "allreduce_multigpu", "barrier", "reduce",
           "broadcast", "allgather", "reducescatter", "alltoall", "send", "recv", "synchronize", "Backend",
           "ReduceOp", "nccl_available", "gloo_available", "reduce_multigpu", "broadcast_multigpu",
           "allgather_multigpu", "reducescatter_multigpu", "send_multigpu", "recv_multigpu"]
