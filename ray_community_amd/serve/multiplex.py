"""Model multiplexing (reference: ``python/ray/serve/multiplex.py``): an LRU of loaded models per
replica keyed by the request's ``multiplexed_model_id``."""
from __future__ import annotations

import asyncio
import collections
import contextvars
import functools
import inspect

_MODEL_ID: contextvars.ContextVar = contextvars.ContextVar("rca_serve_model_id", default="")


def _set_model_id(mid):
    return _MODEL_ID.set(mid or "")


def _reset_model_id(tok):
    _MODEL_ID.reset(tok)


def get_multiplexed_model_id() -> str:
    return _MODEL_ID.get()


def multiplexed(_func=None, *, max_num_models_per_replica: int = 3):
    def deco(fn):
        attr = f"__rca_mux_{fn.__name__}"

        @functools.wraps(fn)
        async def wrapper(self, model_id: str):
            cache = self.__dict__.setdefault(attr, collections.OrderedDict())
            if model_id in cache:
                cache.move_to_end(model_id)
                return cache[model_id]
            m = fn(self, model_id)
            if inspect.isawaitable(m):
                m = await m
            cache[model_id] = m
            while len(cache) > max_num_models_per_replica:
                _, old = cache.popitem(last=False)
                d = getattr(old, "__del__", None)
            return m

        return wrapper

    return deco(_func) if _func is not None else deco
