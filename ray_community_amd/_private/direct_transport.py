"""Direct caller -> actor transport with caller-owned return objects.

Reference behaviour: ``src/ray/core_worker/transport/direct_actor_task_submitter.cc`` (the
caller pushes actor tasks straight to the actor's worker, ordered by per-caller sequence) and
``src/ray/core_worker/reference_count.cc`` (the submitter OWNS the returned objects). Design here:

  * every worker process listens on its own AF_UNIX socket (``DirectServer``); the head only
    resolves an actor id to (socket, incarnation) once per incarnation (``rpc_actor_address``);
  * the caller keeps one ``ActorChannel`` per actor: calls are queued IN SUBMISSION ORDER, their
    ObjectRef arguments are resolved on the caller side (an earlier call with an unresolved
    dependency holds back only this caller's later calls, never other callers'), then pushed over
    one stream, so the actor sees each caller's calls in order;
  * results come back on the same stream and land in the caller's ``OwnedTable`` -- ``get`` /
    ``wait`` on them never touch the head. An owned object is *published* to the head (declared,
    then its value put) only if its ref escapes the process: serialized into an argument, a
    ``put`` or a return value, passed to a head-scheduled task, or waited on together with
    head-managed refs. Results the head must manage anyway (shared-memory, GPU, or holding nested
    refs) are registered by the executing worker before it replies;
  * the head still sees every direct call afterwards: workers batch (task, timing, outcome)
    records to it for the state API and the timeline, off the critical path;
  * a broken stream means the actor's worker died: the channel re-resolves the actor (waiting for
    the head to restart it or declare it dead), re-sends in-flight calls that have
    ``max_task_retries`` left, and fails the others with ``ActorDiedError``.
"""
from __future__ import annotations

import collections
import concurrent.futures
import os
import socket
import threading
import time
import traceback
import logging
from typing import Dict, List, Optional

from .. import exceptions as exc
from . import protocol as P
from . import serialization as ser

log = logging.getLogger("ray_community_amd.direct")
_EXEC_POOL: Optional[concurrent.futures.ThreadPoolExecutor] = None
_EXEC_LOCK = threading.Lock()


def _bg(fn, *args):
    """Run channel state transitions off the thread that resolved a head Deferred (which may be
    the head's own loop thread holding its lock)."""
    global _EXEC_POOL
    if _EXEC_POOL is None:
        with _EXEC_LOCK:
            if _EXEC_POOL is None:
                _EXEC_POOL = concurrent.futures.ThreadPoolExecutor(max_workers=2, thread_name_prefix="rca-direct")
    _EXEC_POOL.submit(_logged, fn, *args)


def _logged(fn, *args):
    try:
        fn(*args)
    except BaseException:  # noqa  (a pool thread would swallow it silently)
        log.error("direct transport: %s failed\n%s", getattr(fn, "__name__", fn), traceback.format_exc())


def error_desc(err: BaseException):
    b = ser.serialize(err, error=True).to_bytes()
    return ("inline", b, len(b), ser.FLAG_ERROR)


# ====================================================================== caller-owned objects
class _Owned:
    __slots__ = ("desc", "callbacks", "published", "tid", "channel", "dropped")

    def __init__(self, tid, channel):
        self.desc = None          # (kind, data, size, flags) once ready
        self.callbacks = []       # fn(desc) run once when ready
        self.published = False    # the head manages (or is told about) this object
        self.tid = tid
        self.channel = channel
        self.dropped = False      # no local refs left, kept only to forward a published value


class OwnedTable:
    def __init__(self, core):
        self.core = core
        self.cond = threading.Condition(threading.Lock())
        self.objs: Dict[bytes, _Owned] = {}

    def create(self, oid, tid, channel):
        with self.cond:
            self.objs[oid] = _Owned(tid, channel)

    def get_entry(self, oid) -> Optional[_Owned]:
        return self.objs.get(oid)

    def set_ready(self, oid, desc, head_managed=False):
        """Store a result. ``head_managed``: the executing worker already registered it with the
        head (holder = this process)."""
        with self.cond:
            e = self.objs.get(oid)
            if e is not None and e.desc is not None:
                return
            forward = False
            cbs = ()
            dropped = e is None or e.dropped
            if e is not None:
                e.desc = desc
                forward = e.published and not head_managed
                if head_managed:
                    e.published = True
                cbs, e.callbacks = e.callbacks, []
                if e.dropped:
                    del self.objs[oid]
        if forward:  # the ref escaped while the call was in flight: hand the value to the head
            self.core.client.call("put", oid, desc[:3], [], False, desc[3])
        for cb in cbs:
            try:
                cb(desc)
            except Exception:  # noqa
                pass
        if dropped and (head_managed or forward):  # release this process's holder at the head
            self.core.client.ref_delta((), (oid,))

    def on_ready(self, oid, cb):
        with self.cond:
            e = self.objs.get(oid)
            if e is not None and e.desc is None:
                e.callbacks.append(cb)
                return
            desc = e.desc if e is not None else error_desc(exc.ObjectLostError(oid.hex()))
        cb(desc)

    def publish(self, oid):
        """Make the head aware of an owned object whose ref is escaping this process."""
        with self.cond:
            e = self.objs.get(oid)
            if e is None or e.published:
                return
            e.published = True
            desc = e.desc
            if desc is None:
                self.core.client.call("declare_object", oid)
                return
        self.core.client.call("put", oid, desc[:3], [], False, desc[3])

    def drop(self, oid) -> bool:
        """Local refcount reached zero. Returns True if the head must also be told (published).
        A pending object that is published (the head waits for the value this process forwards)
        or has callbacks (futures / dependent calls) stays (``dropped``) until its value arrives."""
        with self.cond:
            e = self.objs.get(oid)
            if e is None:
                return False
            if e.desc is None and (e.published or e.callbacks):
                e.dropped = True
                return False
            del self.objs[oid]
        return e.published

    def revive(self, oid) -> bool:
        """A ref to an owned object reappeared locally (count 0 -> 1). True if it is owned (the
        head holder registration is managed here, not by ref deltas)."""
        with self.cond:
            e = self.objs.get(oid)
            if e is None:
                return False
            e.dropped = False
            return True

    def _arm(self, oids, need):
        """Event set once ``need`` of ``oids`` (the ones still pending) have results. Counted
        per-object callbacks, so a getter of N refs costs O(N), not O(N) per arriving result."""
        ev = threading.Event()
        lock = threading.Lock()
        left = [need]

        def cb(_desc):
            with lock:
                left[0] -= 1
                if left[0] == 0:
                    ev.set()

        for o in oids:
            self.objs[o].callbacks.append(cb)
        return ev

    def wait_descs(self, oids, deadline):
        """Block until every oid has a result (or the deadline passes). Returns the descs."""
        with self.cond:
            missing = [o for o in dict.fromkeys(oids) if o in self.objs and self.objs[o].desc is None]
            ev = self._arm(missing, len(missing)) if missing else None
        if ev is not None:
            rem = None if deadline is None else max(0.0, deadline - time.monotonic())
            if not ev.wait(rem):
                raise exc.GetTimeoutError("Get timed out: some object(s) not ready after the timeout.")
        out = []
        for o in oids:
            e = self.objs.get(o)
            out.append(e.desc if e is not None else error_desc(exc.ObjectLostError(o.hex())))
        return out

    def wait_ready(self, oids, num_returns, deadline):
        with self.cond:
            pending = [o for o in oids if o in self.objs and self.objs[o].desc is None]
            need = num_returns - (len(oids) - len(pending))
            ev = self._arm(pending, need) if need > 0 else None
        if ev is not None:
            rem = None if deadline is None else max(0.0, deadline - time.monotonic())
            ev.wait(rem)
        objs = self.objs
        return [o for o in oids if (o not in objs) or objs[o].desc is not None]


# ====================================================================== caller side
class _Call:
    __slots__ = ("spec", "deps", "unresolved", "retries_left", "resolved_args")

    def __init__(self, spec, deps):
        self.spec = spec
        self.deps = deps                  # ObjectRefs kept alive until the call completes
        self.unresolved = 0
        self.retries_left = spec.get("max_task_retries", 0)
        self.resolved_args = list(spec["args"])


class ActorChannel:
    """Ordered direct submission to one actor from this process."""

    def __init__(self, core, aid: bytes):
        self.core = core
        self.aid = aid
        self.lock = threading.RLock()
        self.queue: "collections.deque[_Call]" = collections.deque()
        self.inflight: Dict[bytes, _Call] = {}
        self.conn: Optional[P.Connection] = None
        self.state = "new"  # new | resolving | connected | dead
        self.incarnation = -1
        self.dead_error: Optional[BaseException] = None
        self.holding = False
        self.broken_calls: List[_Call] = []

    # -------------------------------------------------------------- submit
    def submit(self, spec, deps):
        call = _Call(spec, deps)
        owned = self.core.owned
        for rid in spec["return_ids"]:
            owned.create(rid, spec["tid"], self)
        with self.lock:
            if self.state == "dead":
                self._fail(call, self.dead_error)
                return
            self._hold(True)
            self.queue.append(call)
            self._resolve_deps(call)
            self._pump()

    def _resolve_deps(self, call):
        args = call.resolved_args
        head_ids = []
        for i, a in enumerate(args):
            if a[0] != "r":
                continue
            oid = a[1]
            e = self.core.owned.get_entry(oid)
            if e is not None and e.desc is not None and e.desc[3] & ser.FLAG_GPU:
                e = None  # GPU objects: the head hands out current descriptors (spill / restore)
            if e is not None:
                if e.desc is not None:
                    args[i] = ("d", oid, e.desc)
                else:
                    call.unresolved += 1
                    self.core.owned.on_ready(oid, lambda d, i=i, oid=oid, call=call: self._dep_done(call, i, oid, d))
            else:
                head_ids.append((i, oid))
        if head_ids:
            self._resolve_at_head(call, head_ids)

    def _resolve_at_head(self, call, head_ids):
        with self.lock:
            call.unresolved += 1
        fut = self.core.client.call_async("object_descs", [o for _, o in head_ids])

        def done(f, call=call, head_ids=head_ids):  # runs on the _bg pool, never the head thread
            try:
                descs = f.result()
            except BaseException as e:  # noqa
                descs = [error_desc(e if isinstance(e, exc.RayError) else exc.RaySystemError(str(e)))] * len(head_ids)
            with self.lock:
                for (i, oid), d in zip(head_ids, descs):
                    call.resolved_args[i] = ("d", oid, d)
                call.unresolved -= 1
            self._pump_locked()

        fut.add_done_callback(lambda f, done=done: _bg(done, f))

    def _dep_done(self, call, i, oid, desc):
        if desc[3] & ser.FLAG_GPU:  # a GPU result: fetch its current descriptor from the head
            self._resolve_at_head(call, [(i, oid)])
        with self.lock:
            if not desc[3] & ser.FLAG_GPU:
                call.resolved_args[i] = ("d", oid, desc)
            call.unresolved -= 1
        _bg(self._pump_locked)

    def _pump_locked(self):
        with self.lock:
            self._pump()

    def _pump(self):
        if self.state == "new":
            self.state = "resolving"
            self._resolve_address()
            return
        if self.state != "connected":
            return
        while self.queue and self.queue[0].unresolved == 0:
            call = self.queue.popleft()
            spec = dict(call.spec)
            spec["args"] = call.resolved_args
            self.inflight[spec["tid"]] = call
            try:
                self.conn.send((P.DEXEC, spec))
            except OSError:
                self._on_break()
                return

    # -------------------------------------------------------------- address / connection
    def _resolve_address(self):
        fut = self.core.client.call_async("actor_address", self.aid, self.incarnation + 1)
        fut.add_done_callback(lambda f: _bg(self._on_address, f))

    def _on_address(self, fut):
        try:
            path, inc = fut.result()
        except BaseException as e:  # noqa
            err = e if isinstance(e, exc.RayActorError) else exc.ActorDiedError(self.aid, str(e))
            with self.lock:
                self._die(err)
            return
        try:
            s = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            s.connect(path)
            conn = P.Connection(s)
        except OSError:
            # the worker went away between the head's answer and our connect: ask again
            with self.lock:
                self.incarnation = inc
                self._resolve_address()
            return
        with self.lock:
            self.conn = conn
            self.incarnation = inc
            self.state = "connected"
            broken, self.broken_calls = self.broken_calls, []
            # calls that were in flight on the previous incarnation: resend (retries) or fail
            resend = []
            for call in broken:
                if call.retries_left != 0:
                    if call.retries_left > 0:
                        call.retries_left -= 1
                    resend.append(call)
                else:
                    self._fail(call, exc.ActorDiedError(self.aid, "The actor died while executing this call "
                                                                  "(its worker process exited); the actor has "
                                                                  "been restarted."))
            for call in reversed(resend):
                self.queue.appendleft(call)
            threading.Thread(target=self._read_loop, args=(conn,), name="rca-direct-reader", daemon=True).start()
            self._pump()

    def _read_loop(self, conn):
        owned = self.core.owned
        while True:
            try:
                msg = conn.recv()
            except Exception:
                with self.lock:
                    if self.conn is conn:
                        self._on_break()
                return
            if msg[0] != P.DDONE:
                continue
            _, tid, results, head_managed = msg
            with self.lock:
                call = self.inflight.pop(tid, None)
            if call is None:
                continue
            for rid, r in zip(call.spec["return_ids"], results):
                owned.set_ready(rid, r, head_managed)
            call.deps = None
            with self.lock:
                self._maybe_release()

    def _on_break(self):
        try:
            self.conn.close()
        except Exception:
            pass
        self.conn = None
        if self.state == "dead":
            return
        self.broken_calls.extend(self.inflight.values())
        self.inflight.clear()
        self.state = "resolving"
        self._resolve_address()

    def _die(self, err):
        self.state = "dead"
        self.dead_error = err
        calls = list(self.broken_calls) + list(self.inflight.values()) + list(self.queue)
        self.broken_calls, self.inflight = [], {}
        self.queue.clear()
        for c in calls:
            self._fail(c, err)
        self._maybe_release()

    def _fail(self, call, err):
        d = error_desc(err)
        for rid in call.spec["return_ids"]:
            self.core.owned.set_ready(rid, d)
        call.deps = None

    # -------------------------------------------------------------- cancel
    def cancel(self, tid, force):
        with self.lock:
            for c in list(self.queue):
                if c.spec["tid"] == tid:
                    self.queue.remove(c)
                    self._fail(c, exc.TaskCancelledError(tid.hex()))
                    self._maybe_release()
                    return True
            if tid in self.inflight and self.conn is not None:
                try:
                    self.conn.send((P.DCANCEL, tid, False))
                except OSError:
                    pass
                return True
        return False

    # -------------------------------------------------------------- actor lifetime
    def _hold(self, flag):
        """While calls are queued or in flight the channel holds an actor-handle reference, so an
        actor whose last user handle was dropped right after the call is not killed under it."""
        if flag and not self.holding:
            self.holding = True
            self.core.ref_add(b"A" + self.aid)
        elif not flag and self.holding:
            self.holding = False
            self.core.ref_remove(b"A" + self.aid)

    def _maybe_release(self):
        if not self.queue and not self.inflight and not self.broken_calls:
            self._hold(False)

    def close(self):
        with self.lock:
            if self.conn is not None:
                try:
                    self.conn.close()
                except Exception:
                    pass
            self.conn = None
            self.state = "dead"
            self.dead_error = exc.RaySystemError("the session was shut down")


# ====================================================================== actor-worker side
class DirectServer:
    """Accepts direct connections from callers and feeds their calls to the worker."""

    def __init__(self, worker, session_dir: str, wid: bytes):
        self.worker = worker
        path = os.path.join(session_dir or "/tmp", f"d-{wid.hex()[-16:]}.sock")
        if len(path.encode()) > 100:
            path = os.path.join("/tmp", f"rca-d-{wid.hex()[-16:]}.sock")
        if os.path.exists(path):
            os.unlink(path)
        self.path = path
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.bind(path)
        self.sock.listen(256)
        self.records: List[tuple] = []
        self.rec_lock = threading.Lock()
        threading.Thread(target=self._accept_loop, name="rca-direct-accept", daemon=True).start()
        threading.Thread(target=self._flush_loop, name="rca-direct-events", daemon=True).start()

    def _accept_loop(self):
        while True:
            try:
                s, _ = self.sock.accept()
            except OSError:
                return
            conn = P.Connection(s)
            threading.Thread(target=self._conn_loop, args=(conn,), name="rca-direct-conn", daemon=True).start()

    def _conn_loop(self, conn):
        while True:
            try:
                msg = conn.recv()
            except Exception:
                return
            t = msg[0]
            if t == P.DEXEC:
                spec = msg[1]
                spec["_reply"] = conn
                self.worker._dispatch_spec(spec)
            elif t == P.DCANCEL:
                self.worker._cancel(msg[1], msg[2])

    def record(self, spec, start, end, info):
        with self.rec_lock:
            self.records.append((spec["tid"], spec.get("name"), spec.get("actor_id"), start, end,
                                 bool(info.get("error")), info.get("error_type")))

    def _flush_loop(self):
        while True:
            time.sleep(0.1)
            self.flush()

    def flush(self):
        if not self.records:
            return
        with self.rec_lock:
            recs, self.records = self.records, []
        try:
            self.worker.client.send((P.DIRECT_EVENTS, recs))
        except OSError:
            pass

    def close(self):
        try:
            self.sock.close()
            os.unlink(self.path)
        except OSError:
            pass
