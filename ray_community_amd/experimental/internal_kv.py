"""Internal key-value store on the head (reference: ``python/ray/experimental/internal_kv.py``)."""
from __future__ import annotations

from typing import List, Optional, Union


def _client():
    from .._private.worker import _core

    return _core().client


def _b(x):
    return x.encode() if isinstance(x, str) else x


def _internal_kv_initialized() -> bool:
    from .._private.worker import is_initialized

    return is_initialized()


def _internal_kv_put(key, value, overwrite: bool = True, *, namespace=None) -> bool:
    """Returns True if the key already existed (reference semantics)."""
    added = _client().call("kv_put", _b(key), _b(value), overwrite, _b(namespace))
    return not added


def _internal_kv_get(key, *, namespace=None) -> Optional[bytes]:
    return _client().call("kv_get", _b(key), _b(namespace))


def _internal_kv_exists(key, *, namespace=None) -> bool:
    return _client().call("kv_exists", _b(key), _b(namespace))


def _internal_kv_del(key, *, del_by_prefix: bool = False, namespace=None) -> int:
    return _client().call("kv_del", _b(key), _b(namespace), del_by_prefix)


def _internal_kv_list(prefix, *, namespace=None) -> List[bytes]:
    return _client().call("kv_keys", _b(prefix), _b(namespace))
