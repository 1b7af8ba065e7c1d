"""Ray Train equivalent (reference: ``python/ray/train``)."""
from ..air.config import CheckpointConfig, DatasetConfig, FailureConfig, RunConfig, ScalingConfig, SyncConfig
from ..air.result import Result
from ._checkpoint import Checkpoint
from ._internal.backend_executor import TrainingFailedError
from ._internal.session import TrainContext, get_session
from .backend import Backend, BackendConfig
from .data_parallel_trainer import BaseTrainer, DataParallelTrainer


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
           "BackendConfig", "TrainingFailedError", "TrainContext", "SyncConfig", "DatasetConfig"]
