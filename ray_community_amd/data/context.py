"""DataContext (reference: ``python/ray/data/context.py``)."""
from __future__ import annotations

import threading
from dataclasses import dataclass, field


@dataclass
class ExecutionOptions:
    preserve_order: bool = True
    locality_with_output: bool = False
    verbose_progress: bool = False


@dataclass
class DataContext:
    target_max_block_size: int = 128 * 1024 * 1024
    target_min_block_size: int = 1 * 1024 * 1024
    execution_options: ExecutionOptions = field(default_factory=ExecutionOptions)
    enable_progress_bars: bool = False
    use_push_based_shuffle: bool = False

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
