"""``ray.tune.error`` import path."""
from . import TuneError


class TuneStopTrialError(TuneError):
    """Raised inside a trial to stop it without marking it errored."""


__all__ = ["TuneError", "TuneStopTrialError"]
