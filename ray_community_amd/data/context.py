"""DataContext (reference: ``python/ray/data/context.py``)."""
from __future__ import annotations

import threading
from dataclasses import dataclass, field


def _no_limits():
    from ._internal.resource_manager import ExecutionResources

    return ExecutionResources()


@dataclass
class ExecutionOptions:
    """``resource_limits``: caps for the streaming executor (``ExecutionResources(cpu=, gpu=,
    object_store_memory=)``; None = the cluster's CPUs/GPUs and
    ``object_store_memory_limit_fraction`` of its object store)."""
    resource_limits: object = field(default_factory=_no_limits)
    preserve_order: bool = True  # False: operators release blocks as they complete (no head-of-line blocking)
    locality_with_output: bool = False
    verbose_progress: bool = False


@dataclass
class DataContext:
    target_max_block_size: int = 128 * 1024 * 1024
    target_min_block_size: int = 1 * 1024 * 1024
    execution_options: ExecutionOptions = field(default_factory=ExecutionOptions)
    enable_progress_bars: bool = False
    use_push_based_shuffle: bool = False
    object_store_memory_limit_fraction: float = 0.5
    op_resource_reservation_ratio: float = 0.5
    actor_pool_idle_timeout_s: float = 1.0  # an autoscaling pool drops an actor idle this long
    # logical optimizer rules (data/_internal/logical_optimizer.py)
    enable_operator_fusion: bool = True
    enable_limit_pushdown: bool = True
    last_execution_stats: object = None  # ResourceManager.stats() of the most recent execution

    _current = None
    _lock = threading.Lock()

    @staticmethod
    def get_current() -> "DataContext":
        with DataContext._lock:
            if DataContext._current is None:
                DataContext._current = DataContext()
            return DataContext._current

    @staticmethod
    def _set_current(ctx):
        DataContext._current = ctx


DatasetContext = DataContext
