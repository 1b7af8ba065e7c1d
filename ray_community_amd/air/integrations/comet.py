"""``ray.air.integrations.comet`` (reference air/integrations/comet.py): needs `comet_ml`, which is not
installed in this environment."""
from ...tune.logger import LoggerCallback


def _missing():
    raise ImportError("`comet_ml` is not installed in this environment; use the CSV / JSON / TensorBoard "
                      "logger callbacks of ray_community_amd.tune.logger instead")


class CometLoggerCallback(LoggerCallback):
    def __init__(self, *args, **kwargs):
        _missing()


__all__ = ['CometLoggerCallback']
