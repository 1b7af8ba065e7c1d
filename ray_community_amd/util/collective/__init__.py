from .collective import (allgather, allreduce, allreduce_multigpu, alltoall, barrier, broadcast,
                         create_collective_group, destroy_collective_group, get_collective_group_size, get_rank,
                         init_collective_group, is_group_initialized, recv, reduce, reducescatter, send, synchronize)
from .types import Backend, ReduceOp

__all__ = ["init_collective_group", "create_collective_group", "destroy_collective_group", "is_group_initialized",
           "get_rank", "get_collective_group_size", "allreduce", "allreduce_multigpu", "barrier", "reduce",
           "broadcast", "allgather", "reducescatter", "alltoall", "send", "recv", "synchronize", "Backend",
           "ReduceOp"]
