"""``ray.air.integrations.mlflow`` (reference air/integrations/mlflow.py): needs `mlflow`, which is not
installed in this environment."""
from ...tune.logger import LoggerCallback


def _missing():
    raise ImportError("`mlflow` is not installed in this environment; use the CSV / JSON / TensorBoard "
                      "logger callbacks of ray_community_amd.tune.logger instead")


class MLflowLoggerCallback(LoggerCallback):
    def __init__(self, *args, **kwargs):
        _missing()


def setup_mlflow(*args, **kwargs):
    _missing()


__all__ = ['MLflowLoggerCallback', 'setup_mlflow']
