"""TCP relay that serves ``ray://`` drivers (reference: ``python/ray/util/client/server/``,
``proxier.py``: one proxied driver per client connection).

Per accepted connection: read the remote's REGISTER frame, open a dedicated client connection
to the head (its own holder key: the remote driver's references live and die with it), answer
with the head's hello (minus the node-local store), then relay frames both ways:
  remote -> head  RPC (``put`` with a large inline payload is first written into the node's
                  shared-memory store and forwarded as a store descriptor), REF_DELTA;
  head -> remote  REPLY (``get`` descriptors pointing at shared memory or spill files are
                  replaced by the object's bytes).
"""
from __future__ import annotations

import os
import socket
import threading
from typing import Optional

from ..._private import protocol as P
from ..._private.core_worker import INLINE_THRESHOLD, SocketClient
from . import DEFAULT_PORT


def _inline(store, oid, desc):
    kind, data, size, flags = desc
    if kind == "shm":
        b = store.read_bytes(oid) if store is not None else None
        if b is None:
            return desc  # raced with spilling: the remote asks again
        return ("inline", b, len(b), flags)
    if kind == "spill":
        with open(data, "rb") as f:
            b = f.read()
        return ("inline", b, len(b), flags)
    return desc


class _Session:
    def __init__(self, server: "ClientServer", conn: socket.socket, peer):
        self.server = server
        self.peer = peer
        self.remote = P.Connection(conn)
        self.head: Optional[SocketClient] = None
        self.store = None

    def run(self):
        try:
            msg = self.remote.recv()
            if msg[0] != P.REGISTER or msg[1] != "client":
                return
            ident = msg[2]
            extra = msg[4] if len(msg) > 4 and isinstance(msg[4], dict) else {}
            # worker log lines the head pushes are relayed to the remote driver as they are
            relay = (lambda m: self._push(m)) if extra.get("log_to_driver") else None
            self.head = SocketClient(self.server.head_address, "client", ident, on_message=relay,
                                     register_extra={"log_to_driver": bool(extra.get("log_to_driver"))})
            hello = dict(self.head.hello)
            store_name = hello.pop("store", None)
            if store_name:
                from ..._private.object_store import ObjectStore

                try:
                    self.store = ObjectStore(store_name)
                except Exception:
                    self.store = None
            hello["remote"] = True
            self.remote.send((P.REPLY, 0, True, hello))
            while True:
                msg = self.remote.recv()
                t = msg[0]
                if t == P.RPC:
                    self._rpc(*msg[1:])
                elif t == P.REF_DELTA:
                    self.head.ref_delta(msg[1], msg[2])
                # BLOCKED / other worker-only frames are meaningless for a remote driver
        except (ConnectionError, OSError, EOFError):
            pass
        finally:
            self.close()

    def _rpc(self, rid, method, args, kwargs):
        if method == "put":
            oid, desc = args[0], args[1]
            if desc[0] == "inline" and desc[2] > INLINE_THRESHOLD and self.store is not None:
                if self.store.put_bytes(oid, desc[1]):
                    args = (oid, ("shm", None, desc[2])) + tuple(args[2:])
        try:
            fut = self.head.call_async(method, *args, **kwargs)
        except Exception as e:  # noqa
            self._reply(rid, False, e)
            return

        def done(f, rid=rid, method=method, args=args):
            try:
                val = f.result()
                if method == "get":
                    val = [_inline(self.store, oid, d) for oid, d in zip(args[0], val)]
                self._reply(rid, True, val)
            except BaseException as e:  # noqa
                self._reply(rid, False, e)

        fut.add_done_callback(done)

    def _push(self, msg):
        if msg[0] == P.LOG_BATCH:
            try:
                self.remote.send(msg)
            except OSError:
                pass

    def _reply(self, rid, ok, val):
        try:
            self.remote.send((P.REPLY, rid, ok, val))
        except OSError:
            pass

    def close(self):
        try:
            self.remote.close()
        except Exception:
            pass
        if self.head is not None:
            try:
                self.head.flush_refs()
                self.head.close()
            except Exception:
                pass
        self.server._sessions.discard(self)


class ClientServer:
    """``ClientServer(head_address).start()``; ``head_address`` is the session's head socket."""

    def __init__(self, head_address: str, host: str = "127.0.0.1", port: int = DEFAULT_PORT):
        self.head_address = head_address
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(64)
        self.host, self.port = self.sock.getsockname()[:2]
        self._sessions = set()
        self._stop = False
        self._thread = None

    @property
    def address(self) -> str:
        return f"ray://{self.host}:{self.port}"

    def start(self) -> "ClientServer":
        self._thread = threading.Thread(target=self._accept_loop, name="rca-client-server", daemon=True)
        self._thread.start()
        return self

    def _accept_loop(self):
        while not self._stop:
            try:
                conn, peer = self.sock.accept()
            except OSError:
                return
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s = _Session(self, conn, peer)
            self._sessions.add(s)
            threading.Thread(target=s.run, name=f"rca-client-{peer[1]}", daemon=True).start()

    def num_clients(self) -> int:
        return len(self._sessions)

    def stop(self):
        self._stop = True
        try:
            self.sock.close()
        except OSError:
            pass
        for s in list(self._sessions):
            s.close()


def serve(address: str = f"127.0.0.1:{DEFAULT_PORT}", head_address: Optional[str] = None) -> ClientServer:
    """Start a client server for the session this process is attached to (or ``head_address``)."""
    from ..._private import worker

    if head_address is None:
        head_address = worker._state.get("address")
        if not head_address or str(head_address).startswith("ray://"):
            raise RuntimeError("serve() needs a process attached to a local session (init() first)")
    host, _, port = address.rpartition(":")
    srv = ClientServer(head_address, host or "127.0.0.1", int(port or DEFAULT_PORT)).start()
    worker._state.setdefault("client_servers", []).append(srv)
    return srv


if __name__ == "__main__":  # python -m ray_community_amd.util.client.server --address auto --port 10001
    import argparse
    import signal

    ap = argparse.ArgumentParser()
    ap.add_argument("--address", default="auto")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=DEFAULT_PORT)
    a = ap.parse_args()
    from ..._private.worker import _resolve_address

    srv = ClientServer(_resolve_address(a.address), a.host, a.port).start()
    print(srv.address, flush=True)
    ev = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: ev.set())
    signal.signal(signal.SIGINT, lambda *_: ev.set())
    ev.wait()
    srv.stop()
    os._exit(0)
