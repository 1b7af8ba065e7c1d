"""AIR configs (reference: ``python/ray/air/config.py``)."""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Union


@dataclass
class ScalingConfig:
    num_workers: Optional[int] = None
    use_gpu: bool = False
    resources_per_worker: Optional[Dict[str, float]] = None
    placement_strategy: str = "PACK"
    trainer_resources: Optional[Dict[str, float]] = None
    accelerator_type: Optional[str] = None
    topology: Optional[str] = None

    def __post_init__(self):
        if self.resources_per_worker:
            if not self.use_gpu and self.resources_per_worker.get("GPU", 0) > 0:
                raise ValueError("`use_gpu` is False but `GPU` was found in `resources_per_worker`. Either set "
                                 "`use_gpu` to True or remove `GPU` from `resources_per_worker.")
            if self.use_gpu and self.resources_per_worker.get("GPU", 1) == 0:
                raise ValueError("`use_gpu` is True but `GPU` is set to 0 in `resources_per_worker`.")

    @property
    def _resources_per_worker_not_none(self):
        if self.resources_per_worker is None:
            return {"CPU": 1, "GPU": 1} if self.use_gpu else {"CPU": 1}
        r = {k: v for k, v in self.resources_per_worker.items() if v != 0}
        if self.use_gpu:
            r.setdefault("GPU", 1)
        return r

    @property
    def num_cpus_per_worker(self):
        return self._resources_per_worker_not_none.get("CPU", 0)

    @property
    def num_gpus_per_worker(self):
        return self._resources_per_worker_not_none.get("GPU", 0)

    @property
    def additional_resources_per_worker(self):
        return {k: v for k, v in self._resources_per_worker_not_none.items() if k not in ("CPU", "GPU")}

    def as_placement_group_factory(self):
        bundles = [dict(self._resources_per_worker_not_none) for _ in range(self.num_workers or 1)]
        return {"bundles": bundles, "strategy": self.placement_strategy}

    @classmethod
    def from_placement_group_factory(cls, pgf) -> "ScalingConfig":
        """Inverse of ``as_placement_group_factory``: bundles (or a PlacementGroupFactory) whose
        first bundle may be the trainer's own and the rest identical worker bundles."""
        bundles = list(getattr(pgf, "bundles", None) or (pgf.get("bundles") if isinstance(pgf, dict) else pgf))
        strategy = getattr(pgf, "strategy", None) or (pgf.get("strategy") if isinstance(pgf, dict) else None) or "PACK"
        if not bundles:
            raise ValueError("placement group factory without bundles")
        trainer = None
        workers = bundles
        if len(bundles) > 1 and bundles[0] != bundles[1]:
            trainer, workers = bundles[0], bundles[1:]
        w = dict(workers[0])
        return cls(num_workers=len(workers), use_gpu=w.get("GPU", 0) > 0, resources_per_worker=w,
                   placement_strategy=strategy, trainer_resources=trainer)

    @property
    def total_resources(self):
        out = {}
        for k, v in self._resources_per_worker_not_none.items():
            out[k] = v * (self.num_workers or 1)
        return out


@dataclass
class FailureConfig:
    max_failures: int = 0
    fail_fast: Union[bool, str] = False


@dataclass
class CheckpointConfig:
    num_to_keep: Optional[int] = None
    checkpoint_score_attribute: Optional[str] = None
    checkpoint_score_order: str = "max"
    checkpoint_frequency: int = 0
    checkpoint_at_end: Optional[bool] = None

    def __post_init__(self):
        if self.num_to_keep is not None and self.num_to_keep <= 0:
            raise ValueError(f"Received invalid num_to_keep: {self.num_to_keep}. Must be None or > 0.")
        if self.checkpoint_score_order not in ("max", "min"):
            raise ValueError("checkpoint_score_order must be either 'max' or 'min'")


@dataclass
class RunConfig:
    name: Optional[str] = None
    storage_path: Optional[str] = None
    storage_filesystem: Any = None
    callbacks: Optional[List[Any]] = None
    stop: Optional[Union[Dict, Callable, Any]] = None
    failure_config: Optional[FailureConfig] = None
    checkpoint_config: Optional[CheckpointConfig] = None
    sync_config: Any = None
    verbose: Optional[int] = None
    log_to_file: Union[bool, str] = False
    progress_reporter: Any = None

    @property
    def local_dir(self) -> Optional[str]:  # the pre-2.7 name of storage_path
        return self.storage_path

    def __post_init__(self):
        if self.failure_config is None:
            self.failure_config = FailureConfig()
        if self.checkpoint_config is None:
            self.checkpoint_config = CheckpointConfig()
        if self.storage_path is None:
            self.storage_path = os.environ.get("RCA_STORAGE_PATH", os.path.expanduser("~/rca_results"))


@dataclass
class DatasetConfig:
    fit: Optional[bool] = None
    split: Optional[bool] = None
    required: Optional[bool] = None


@dataclass
class SyncConfig:
    upload_dir: Optional[str] = None
    syncer: Any = None
    sync_period: int = 300
    sync_timeout: int = 1800
