"""API stability annotations (reference: ``python/ray/util/annotations.py``)."""
from __future__ import annotations

import functools
import warnings


def _annotate(obj, stability, message=None):
    doc = obj.__doc__ or ""
    note = f"\n\n    {stability}" + (f": {message}" if message else "")
    try:
        obj.__doc__ = doc + note
        obj._annotated = stability
    except (AttributeError, TypeError):
        pass
    return obj


def PublicAPI(*args, **kwargs):
    stability = kwargs.get("stability", "stable")
    if len(args) == 1 and not kwargs and callable(args[0]):
        return _annotate(args[0], "PublicAPI")
    return lambda obj: _annotate(obj, f"PublicAPI ({stability})")


def DeveloperAPI(*args, **kwargs):
    if len(args) == 1 and not kwargs and callable(args[0]):
        return _annotate(args[0], "DeveloperAPI")
    return lambda obj: _annotate(obj, "DeveloperAPI")


class RayDeprecationWarning(DeprecationWarning):
    """Warning category of deprecated Ray APIs (shown by default, unlike DeprecationWarning)."""


warnings.simplefilter("module", RayDeprecationWarning)


def Deprecated(*args, **kwargs):
    message = kwargs.get("message")

    def wrap(obj):
        if isinstance(obj, type):
            return _annotate(obj, "Deprecated", message)

        @functools.wraps(obj)
        def inner(*a, **k):
            warnings.warn(f"{obj.__name__} is deprecated. {message or ''}", RayDeprecationWarning, stacklevel=2)
            return obj(*a, **k)

        return _annotate(inner, "Deprecated", message)

    if len(args) == 1 and not kwargs and callable(args[0]):
        return wrap(args[0])
    return wrap


def Experimental(obj):
    return _annotate(obj, "Experimental")
