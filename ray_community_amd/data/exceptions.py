"""Ray Data exception types (reference: ``python/ray/data/exceptions.py``).

A failure inside a user-defined function of a Data transformation (``map``, ``map_batches``,
``flat_map``, ``filter``, ``add_column``) is raised as ``RayDataUserCodeException`` -- a
``ray.exceptions.UserCodeException`` -- chained to the original error (``__cause__``), so a
driver can tell its own bug from a framework failure (``SystemException``) and still inspect the
original exception. ``omit_traceback_stdout`` wraps an entry point: the full stack trace goes to
the ``ray_community_amd.data`` logger, and the exception is re-raised without the framework frames
unless ``DataContext.log_internal_stack_trace_to_stdout`` is set.
"""
from __future__ import annotations

import functools
import logging
from typing import Callable

from ..exceptions import UserCodeException

logger = logging.getLogger("ray_community_amd.data")


class RayDataUserCodeException(UserCodeException):
    """An exception raised by user code inside a Ray Data transformation."""


class SystemException(Exception):
    """An exception from Ray Data / Ray Core internals rather than user code."""


def omit_traceback_stdout(fn: Callable) -> Callable:
    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        try:
            return fn(*args, **kwargs)
        except Exception as e:
            from .context import DataContext

            full = bool(getattr(DataContext.get_current(), "log_internal_stack_trace_to_stdout", False))
            logger.debug("Ray Data exception (full stack trace)", exc_info=True)
            if full:
                raise
            if isinstance(e, UserCodeException):
                raise e.with_traceback(None)
            raise e.with_traceback(None) from SystemException()

    return wrapper


def call_user_fn(fn: Callable, *args, **kwargs):
    """Run a transformation's UDF; its exceptions surface as ``RayDataUserCodeException``."""
    try:
        return fn(*args, **kwargs)
    except UserCodeException:
        raise
    except Exception as e:
        raise RayDataUserCodeException(f"{type(e).__name__}: {e}") from e


__all__ = ["RayDataUserCodeException", "SystemException", "UserCodeException", "omit_traceback_stdout"]
