"""Ray Client: drive a session from another machine through ``init("ray://host:port")``.

Reference: ``python/ray/util/client/`` (a gRPC proxy on the head, port 10001, that runs the
remote driver's API calls in the cluster). Design here:

  * **server** (``server.py``, started by ``start --head --ray-client-server-port`` or
    ``serve()`` from any process attached to the session): a TCP relay. Each remote driver gets
    its own head connection, so its object references, jobs and namespace are isolated and are
    released when its link drops. RPCs are relayed frame by frame; object descriptors are made
    location-free on the way: ``get`` replies carry the bytes of shared-memory / spilled objects
    inline, large inline ``put``\\ s are written into the node's shared-memory store.
  * **client** (:class:`RemoteCoreWorker`): the ordinary core worker over a TCP socket, with every
    object travelling inline and actor calls routed through the head (the direct caller->actor
    transport needs node-local sockets). ``remote``/``get``/``put``/``wait``/actors/placement
    groups/``get_actor``/``kill``/``cancel`` and the introspection calls all work unchanged.
GPU tensors cannot cross the link by handle: move them to the host before sending.
"""
from __future__ import annotations

import socket

from ..._private.core_worker import CoreWorker, SocketClient
from ... import exceptions as exc

DEFAULT_PORT = 10001


def parse_address(address: str):
    rest = address[len("ray://"):] if address.startswith("ray://") else address
    host, _, port = rest.rpartition(":")
    if not host:
        host, port = rest, str(DEFAULT_PORT)
    return host or "127.0.0.1", int(port)


class RemoteCoreWorker(CoreWorker):
    """Core worker of a ``ray://`` driver: no local object store, objects inline both ways."""

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.direct_actor_calls = False

    def _store_serialized(self, oid, s, copy_gpu: bool = True):
        if s.gpu_tensors:
            raise TypeError("GPU tensors cannot be sent through a ray:// client link; move them to the host first")
        b = s.to_bytes()
        return ("inline", b, len(b))

    def _materialize(self, oid, desc):
        if desc[0] != "inline":
            raise exc.RaySystemError(f"ray:// client received a node-local object descriptor ({desc[0]})")
        return super()._materialize(oid, desc)


def connect(address: str, namespace: str, log_to_driver: bool = True):
    """Open the TCP link, register as a client driver and build its core worker."""
    import os

    host, port = parse_address(address)
    s = socket.create_connection((host, port), timeout=30)
    s.settimeout(None)
    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    from ..._private.worker import _driver_push_handler

    client = SocketClient(None, "client", os.urandom(20), sock=s, on_message=_driver_push_handler(log_to_driver),
                          register_extra={"log_to_driver": bool(log_to_driver)})
    hello = client.hello
    core = RemoteCoreWorker("client", client, None, hello["node_id"], hello["job_id"], namespace,
                            session_dir=hello.get("session_dir", ""))
    return core, f"ray://{host}:{port}"


def is_connected() -> bool:
    """True when this process drives a session through a ``ray://`` link."""
    from ..._private import worker

    return bool(worker._state.get("client_mode")) and worker._state.get("core") is not None


def num_connected_contexts() -> int:
    """Client contexts this process holds (0 or 1: one ``ray://`` session per process here)."""
    from ..._private import worker as w

    core = w._state.get("core")
    return 1 if core is not None and isinstance(core, RemoteCoreWorker) else 0


class RayAPIStub:
    """The ``ray.util.client.ray`` object of the reference: ``connect(address)`` /
    ``disconnect()`` / ``is_connected()`` around ``init("ray://...")``."""

    def connect(self, conn_str: str, namespace: str = None, **kw):
        from ..._private import worker as w

        return w.init(conn_str if conn_str.startswith("ray://") else "ray://" + conn_str, namespace=namespace, **kw)

    def disconnect(self):
        from ..._private import worker as w

        w.shutdown()

    def is_connected(self) -> bool:
        return num_connected_contexts() > 0


ray = RayAPIStub()
