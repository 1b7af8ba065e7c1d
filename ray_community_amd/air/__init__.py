from .config import CheckpointConfig, DatasetConfig, FailureConfig, RunConfig, ScalingConfig
from .result import Result

__all__ = ["ScalingConfig", "RunConfig", "CheckpointConfig", "FailureConfig", "DatasetConfig", "Result"]
