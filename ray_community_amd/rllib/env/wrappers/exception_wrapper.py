"""``ResetOnExceptionWrapper`` (reference: ``rllib/env/wrappers/exception_wrapper.py``): an env whose
``reset`` / ``step`` can raise (a flaky simulator) is reset instead of failing the runner.

``reset`` is retried up to ``max_reset_attempts`` times (then ``TooManyResetAttemptsException``);
a ``step`` that raises resets the env and ends the episode as truncated, with
``info["__terminated__"] = True`` and the traceback in ``info["exception"]``.
"""
from __future__ import annotations

import logging
import traceback

from ..envs import Wrapper

logger = logging.getLogger(__name__)


class TooManyResetAttemptsException(Exception):
    def __init__(self, max_attempts: int):
        super().__init__(f"Reached the maximum number of attempts ({max_attempts}) to reset an environment.")


class ResetOnExceptionWrapper(Wrapper):
    def __init__(self, env, max_reset_attempts: int = 5):
        super().__init__(env)
        self.max_reset_attempts = int(max_reset_attempts)

    def reset(self, **kwargs):
        for _ in range(self.max_reset_attempts):
            try:
                return self.env.reset(**kwargs)
            except Exception:  # noqa - a failing simulator: log and try again
                logger.error(traceback.format_exc())
        raise TooManyResetAttemptsException(self.max_reset_attempts)

    def step(self, action):
        try:
            return self.env.step(action)
        except Exception:  # noqa
            tb = traceback.format_exc()
            logger.error(tb)
            obs, info = self.reset()
            info = dict(info or {}, __terminated__=True, exception=tb)
            return obs, 0.0, False, True, info


__all__ = ["ResetOnExceptionWrapper", "TooManyResetAttemptsException"]
