"""``ray.air.integrations.wandb`` (reference air/integrations/wandb.py): needs `wandb`, which is not
installed in this environment."""
from ...tune.logger import LoggerCallback


def _missing():
    raise ImportError("`wandb` is not installed in this environment; use the CSV / JSON / TensorBoard "
                      "logger callbacks of ray_community_amd.tune.logger instead")


class WandbLoggerCallback(LoggerCallback):
    def __init__(self, *args, **kwargs):
        _missing()


def setup_wandb(*args, **kwargs):
    _missing()


__all__ = ['WandbLoggerCallback', 'setup_wandb']
