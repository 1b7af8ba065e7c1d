"""Ray Train equivalent (reference: ``python/ray/train``)."""
from ..air.config import CheckpointConfig, DatasetConfig, FailureConfig, RunConfig, ScalingConfig, SyncConfig
from ..air.result import Result
from ._checkpoint import Checkpoint
from ._internal.backend_executor import TrainingFailedError
from ._internal.session import TrainContext, get_session
from .backend import Backend, BackendConfig
from .data_parallel_trainer import BaseTrainer, DataParallelTrainer


TRAIN_DATASET_KEY = "train"


class DataConfig:
    """Which ``datasets`` are split across the training workers (reference
    ``train/_internal/data_config.py``): ``datasets_to_split="all"`` (default) or a list of names;
    the others are given whole to every worker. ``execution_options`` are passed to the
    streaming executor of each split."""

    def __init__(self, datasets_to_split="all", execution_options=None, enable_shard_locality: bool = True):
        if datasets_to_split != "all" and not isinstance(datasets_to_split, (list, tuple)):
            raise TypeError("datasets_to_split must be 'all' or a list of dataset names")
        self.datasets_to_split = datasets_to_split if datasets_to_split == "all" else list(datasets_to_split)
        self.execution_options = execution_options
        self.enable_shard_locality = enable_shard_locality

    @staticmethod
    def default_ingest_options():
        from ..data import ExecutionOptions

        return ExecutionOptions()


class TrainingIterator:
    """Iterates the per-round worker results of a run (``train/trainer.py``), as the metrics the
    workers reported, round by round. ``Result.metrics_history`` is the same data after the fact."""

    def __init__(self, result):
        self._hist = list(getattr(result, "metrics_history", None) or [])

    def __iter__(self):
        return iter(self._hist)

    def get_final_results(self, force: bool = False):
        return self._hist[-1] if self._hist else None


def report(metrics, checkpoint=None):
    """Report metrics (and optionally a Checkpoint) from a training worker."""
    get_session().report(dict(metrics), checkpoint=checkpoint)


def get_context() -> TrainContext:
    return get_session().context


def get_checkpoint():
    return get_session().checkpoint


def get_dataset_shard(name: str = "train"):
    return get_session().dataset_shards.get(name)


__all__ = ["report", "get_context", "get_checkpoint", "get_dataset_shard", "Checkpoint", "Result", "ScalingConfig",
           "RunConfig", "CheckpointConfig", "FailureConfig", "DataParallelTrainer", "BaseTrainer", "Backend",
           "BackendConfig", "TrainingFailedError", "TrainContext", "SyncConfig", "DatasetConfig", "DataConfig",
           "TrainingIterator", "TRAIN_DATASET_KEY"]
