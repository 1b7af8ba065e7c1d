"""``ray.util.client_connect`` (reference: ``python/ray/util/client_connect.py``): ``connect`` /
``disconnect`` for a Ray Client session, here a thin front for ``init("ray://host:port")`` over
this framework's TCP client relay (``util/client``)."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple


def connect(conn_str: str, secure: bool = False, metadata: Optional[List[Tuple[str, str]]] = None,
            connection_retries: int = 3, job_config=None, namespace: Optional[str] = None, *,
            ignore_version: bool = False, _credentials=None,
            ray_init_kwargs: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    """Connect this process to a cluster's client server; returns the connection info."""
    from .. import init, is_initialized
    from . import client

    kw = dict(ray_init_kwargs or {})
    if is_initialized() and client.is_connected():
        if kw.get("ignore_reinit_error", False):
            return {"address": conn_str, "reused": True}
        raise RuntimeError('Ray Client is already connected. Maybe you called ray.init("ray://<address>") twice?')
    if secure or _credentials is not None:
        raise NotImplementedError("TLS client connections are not supported by the TCP client relay")
    addr = conn_str if conn_str.startswith("ray://") else f"ray://{conn_str}"
    last = None
    for _ in range(max(1, int(connection_retries))):
        try:
            ctx = init(addr, namespace=namespace, job_config=job_config, **kw)
            return {"address": addr, "namespace": namespace, "context": ctx}
        except ConnectionError as e:  # server not up yet
            last = e
            import time

            time.sleep(1.0)
    raise ConnectionError(f"could not connect to {addr} after {connection_retries} attempts") from last


def disconnect():
    """Disconnect from the client server (idempotent); same as ``ray.shutdown()`` in client mode."""
    from .. import is_initialized, shutdown

    if is_initialized():
        shutdown()


__all__ = ["connect", "disconnect"]
