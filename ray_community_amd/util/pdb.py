"""Breakpoints inside tasks and actors (reference: ``python/ray/util/rpdb.py``, ``ray.util.pdb``).

A worker has no terminal, so ``set_trace()`` opens a pdb session on a TCP socket instead: it
binds 127.0.0.1 on a free port (``RCA_PDB_PORT`` / ``port=`` to pin it), records the breakpoint in
the session's internal KV (``list_breakpoints()`` / ``python -m ray_community_amd debug``) and prints
where to connect; any line-mode client (``nc 127.0.0.1 PORT``, ``telnet``) then drives pdb. The
session ends with ``c``/``q`` or when the client disconnects.
"""
from __future__ import annotations

import json
import os
import pdb as _pdb
import socket
import sys
import time
from typing import List, Optional

_KV_PREFIX = "RCA_PDB_"


class RemotePdb(_pdb.Pdb):
    def __init__(self, host: str = "127.0.0.1", port: int = 0, quiet: bool = False):
        self._listener = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self._listener.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self._listener.bind((host, port))
        self._listener.listen(1)
        self.host, self.port = self._listener.getsockname()
        self._quiet = quiet
        self._conn = None
        self._file = None
        self._key = None

    def listen(self, timeout: Optional[float] = None):
        self._key = _register(self.host, self.port)
        if not self._quiet:
            print(f"RemotePdb session open at {self.host}:{self.port}, use 'nc {self.host} {self.port}' "
                  f"or `python -m ray_community_amd debug` to connect", flush=True)
        self._listener.settimeout(timeout)
        self._conn, _ = self._listener.accept()
        self._listener.close()
        self._file = self._conn.makefile("rw")
        super().__init__(stdin=self._file, stdout=self._file)
        self.prompt = "(rca-pdb) "
        self.use_rawinput = False

    def _close(self):
        _unregister(self._key)
        for c in (self._file, self._conn):
            try:
                if c is not None:
                    c.close()
            except OSError:
                pass

    def do_continue(self, arg):
        r = super().do_continue(arg)
        self._close()
        return r

    do_c = do_cont = do_continue

    def do_quit(self, arg):
        r = super().do_quit(arg)
        self._close()
        return r

    do_q = do_exit = do_quit

    def do_EOF(self, arg):
        return self.do_quit(arg)


def _register(host, port) -> Optional[str]:
    try:
        from ..experimental import internal_kv

        key = f"{_KV_PREFIX}{os.getpid()}_{port}"
        internal_kv._internal_kv_put(key, json.dumps({"host": host, "port": port, "pid": os.getpid(),
                                                      "time": time.time()}), namespace="rca_pdb")
        return key
    except Exception:  # noqa  (no session: breakpoint still works, just not listed)
        return None


def _unregister(key):
    if key is None:
        return
    try:
        from ..experimental import internal_kv

        internal_kv._internal_kv_del(key, namespace="rca_pdb")
    except Exception:  # noqa
        pass


def list_breakpoints() -> List[dict]:
    """Active remote breakpoints of the session (host, port, pid)."""
    from ..experimental import internal_kv

    out = []
    for k in internal_kv._internal_kv_list(_KV_PREFIX, namespace="rca_pdb"):
        v = internal_kv._internal_kv_get(k, namespace="rca_pdb")
        if v:
            out.append(json.loads(v))
    return out


def set_trace(host: str = "127.0.0.1", port: Optional[int] = None, timeout: Optional[float] = None):
    """Break here and serve pdb on a TCP port (see module docstring)."""
    if port is None:
        port = int(os.environ.get("RCA_PDB_PORT", "0"))
    dbg = RemotePdb(host, port)
    dbg.listen(timeout)
    dbg.set_trace(sys._getframe().f_back)


def post_mortem(tb=None, host: str = "127.0.0.1", port: Optional[int] = None):
    dbg = RemotePdb(host, port or int(os.environ.get("RCA_PDB_PORT", "0")))
    dbg.listen()
    dbg.reset()
    dbg.interaction(None, tb or sys.exc_info()[2])
    dbg._close()
