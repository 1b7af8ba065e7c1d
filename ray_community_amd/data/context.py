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
    exclude_resources: object = field(default_factory=_no_limits)
    actor_locality_enabled: bool = True

    def validate(self) -> None:
        """Limits must be non-negative (reference ``ExecutionOptions.validate``)."""
        for name in ("resource_limits", "exclude_resources"):
            r = getattr(self, name)
            for attr in ("cpu", "gpu", "object_store_memory"):
                v = getattr(r, attr, None)
                if v is not None and v < 0:
                    raise ValueError(f"ExecutionOptions.{name}.{attr} must be >= 0, got {v}")


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
    # reference DataContext knobs (python/ray/data/context.py); read by this implementation where
    # the mechanism exists, kept for compatibility where it does not
    streaming_read_buffer_size: int = 32 * 1024 * 1024
    enable_pandas_block: bool = True
    enable_tensor_extension_casting: bool = True
    enable_auto_log_stats: bool = False
    verbose_stats_logs: bool = False
    trace_allocations: bool = False
    eager_free: bool = False
    decoding_size_estimation: bool = True
    min_parallelism: int = 200
    read_op_min_num_blocks: int = 200
    large_args_threshold: int = 50 * 1024 * 1024
    scheduling_strategy: object = "SPREAD"
    scheduling_strategy_large_args: object = "DEFAULT"
    target_shuffle_max_block_size: int = 1024 * 1024 * 1024
    pipeline_push_based_shuffle_reduce_tasks: bool = True
    actor_prefetcher_enabled: bool = False
    use_polars: bool = False
    use_ray_tqdm: bool = True
    log_internal_stack_trace_to_stdout: bool = False
    max_errored_blocks: int = 0
    write_file_retry_on_errors: tuple = ("AWS Error INTERNAL_FAILURE", "AWS Error NETWORK_CONNECTION",
                                         "AWS Error SLOW_DOWN")
    actor_task_retry_on_errors: object = False
    op_resource_reservation_enabled: bool = True
    enable_get_object_locations_for_metrics: bool = False
    warn_on_driver_memory_usage_bytes: int = 2 * 1024 * 1024 * 1024
    _kv_configs: dict = field(default_factory=dict)

    def get_config(self, key: str, default=None):
        """Free-form plugin settings (reference ``DataContext.get_config``)."""
        return self._kv_configs.get(key, default)

    def set_config(self, key: str, value) -> None:
        self._kv_configs[key] = value

    def remove_config(self, key: str) -> None:
        self._kv_configs.pop(key, None)

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
