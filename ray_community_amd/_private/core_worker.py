"""Per-process core worker: ObjectRef, local reference counting, object get/put, task submission.

Reference: ``python/ray/_raylet.pyx`` (CoreWorker, ObjectRef, ObjectRefGenerator) and
``src/ray/core_worker/core_worker.cc``. The same ``CoreWorker`` class serves
  * the driver in the head's process (``DirectClient``: in-process calls into the head), and
  * worker processes / external drivers (``SocketClient``: framed RPC over a Unix socket).
Objects are read zero-copy from the node's shm store; small objects travel inline.
"""
from __future__ import annotations

import asyncio
import concurrent.futures
import hashlib
import itertools
import operator
import os
import socket
import threading
import time
import weakref
from typing import Any, Dict, List, Optional

from .. import exceptions as exc
from . import protocol as P
from . import serialization as ser
from ..util import tracing
from .ids import new_id
from .object_store import ObjectStore

INLINE_THRESHOLD = 100 * 1024

_core: Optional["CoreWorker"] = None


def global_core() -> "CoreWorker":
    if _core is None:
        raise RuntimeError("ray_community_amd is not initialized; call init() first")
    return _core


def set_global_core(c):
    global _core
    _core = c


_REF_ID = operator.attrgetter("_id")

# ====================================================================== ObjectRef
class ObjectRef:
    __slots__ = ("_id", "_core", "__weakref__")
    # ``ObjectRef[int]`` in annotations (the reference's typing stub ``ray.types.ObjectRef[T]``)
    __class_getitem__ = classmethod(__import__("types").GenericAlias)

    def __init__(self, oid: bytes, _register=True):
        self._id = oid
        c = _core
        self._core = c
        if _register and c is not None:
            c.ref_add(oid)

    def __del__(self):
        c = self._core
        if c is not None:
            try:
                c.ref_remove(self._id)
            except Exception:
                pass

    def binary(self):
        return self._id

    def hex(self):
        return self._id.hex()

    def task_id(self):
        """``TaskID`` of the task that returns this object (None for ``put`` objects)."""
        from .ids import TaskID, task_id_of

        t = task_id_of(self._id)
        return TaskID(t) if t is not None else None

    def __hash__(self):
        return hash(self._id)

    def __eq__(self, other):
        return isinstance(other, ObjectRef) and other._id == self._id

    def __repr__(self):
        return f"ObjectRef({self._id.hex()})"

    def __reduce__(self):
        ctx = ser.current_context()
        if ctx is not None:
            ctx.contained.append(self._id)
        c = _core
        if c is not None and self._id in c.owned.objs:
            c.owned.publish(self._id)  # a caller-owned result escapes this process
        return (_rebuild_ref, (self._id,))

    # futures / asyncio integration
    def future(self) -> concurrent.futures.Future:
        return global_core().as_future(self)

    def __await__(self):
        return asyncio.wrap_future(self.future()).__await__()

    def _on_completed(self, cb):
        f = self.future()
        f.add_done_callback(lambda fut: cb(fut.result()))


def _rebuild_ref(oid):
    return ObjectRef(oid)


class ObjectRefGenerator:
    """Iterator over the outputs of a ``num_returns="streaming"`` task (reference:
    ``ObjectRefGenerator`` in ``_raylet.pyx``). Yields ObjectRefs as the task produces them."""

    def __init__(self, tid: bytes, main_ref: ObjectRef):
        self._tid = tid
        self._main = main_ref
        self._i = 0
        self._done = False

    def __iter__(self):
        return self

    def __next__(self):
        return self._next_sync(None)

    def _next_sync(self, timeout_s=None):
        if self._done:
            raise StopIteration
        core = global_core()
        oid = core.client.call("gen_next", self._tid, self._i, timeout_s)
        if oid is None:
            self._done = True
            # surface a generator failure (stored on the task's main return object)
            core.get([self._main], timeout=None, _raise=True)
            raise StopIteration
        self._i += 1
        ref = ObjectRef(oid)
        core.ref_remove_server_pin(oid)
        return ref

    def __aiter__(self):
        return self

    def _next_or_none(self):
        try:
            return self._next_sync(None)
        except StopIteration:  # cannot cross an executor future: signal the end with None
            return None

    async def __anext__(self):
        loop = asyncio.get_running_loop()
        ref = await loop.run_in_executor(None, self._next_or_none)
        if ref is None:
            raise StopAsyncIteration
        return ref

    def completed(self):
        return self._main

    def is_finished(self):
        return self._done

    def __del__(self):
        # dropped before the end of the stream: a producer paused on backpressure would otherwise
        # hold its worker forever (reference: DelObjectRefStream)
        if self._done:
            return
        try:
            core = global_core()
            if core is not None and not core._shutdown:
                core.client.call_async("gen_drop", self._tid)
        except Exception:
            pass


class DynamicObjectRefGenerator:
    """Return value of a ``num_returns="dynamic"`` task: an iterable of ObjectRefs."""

    def __init__(self, refs):
        self._refs = list(refs)

    def __iter__(self):
        return iter(self._refs)

    def __len__(self):
        return len(self._refs)


# ====================================================================== clients
class DirectClient:
    """In-process calls into the head (driver co-located with the head)."""

    def __init__(self, head):
        self.head = head
        self.key = "driver"  # this process's holder key at the head

    def call(self, method, *args, **kwargs):
        head = self.head
        with head.lock:
            res = getattr(head, "rpc_" + method)(self.key, *args, **kwargs)
        if res.__class__.__name__ == "Deferred":
            if res.done:  # resolved inside the call (e.g. wait/get on ready objects)
                if not res.ok:
                    raise res.value
                return res.value
            ev = threading.Event()
            res.add(lambda d: ev.set())
            ev.wait()
            if not res.ok:
                raise res.value
            return res.value
        return res

    def call_async(self, method, *args):
        fut = concurrent.futures.Future()
        head = self.head
        try:
            with head.lock:
                res = getattr(head, "rpc_" + method)(self.key, *args)
        except Exception as e:
            fut.set_exception(e)
            return fut
        if res.__class__.__name__ == "Deferred":
            def done(d):
                if d.ok:
                    fut.set_result(d.value)
                else:
                    fut.set_exception(d.value)
            res.add(done)
        else:
            fut.set_result(res)
        return fut

    def ref_delta(self, adds, removes):
        head = self.head
        with head.lock:
            for o in adds:
                head._add_holder(o, self.key)
            for o in removes:
                head._remove_holder(o, self.key)

    def submit(self, spec):
        head = self.head
        with head.lock:
            head._submit(spec, self.key)

    def close(self):
        pass


class _RefList(list):
    """The remainder list ``wait()`` returns: a plain list that can be weakly referenced, so the
    polling fast path can recognise it without keeping its refs alive."""

    __slots__ = ("__weakref__",)


class SocketClient:
    """Framed RPC client over the head's Unix socket (workers and external drivers), or over a
    pre-connected stream socket (``sock``: the TCP link of a ``ray://`` remote driver)."""

    def __init__(self, sock_path, kind, ident, on_message=None, register_extra=None, sock=None):
        if sock is None:
            sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            sock.connect(sock_path)
        s = sock
        self.conn = P.Connection(s)
        self._req = itertools.count(1)
        self._pending: Dict[int, concurrent.futures.Future] = {}
        self._lock = threading.Lock()
        self.on_message = on_message
        self.kind = kind
        self.key = ("w:" + ident.hex()) if kind == "worker" else ("client:" + ident.hex())
        self._closed = False
        self._adds: List[bytes] = []
        self._removes: List[bytes] = []
        self._rlock = threading.Lock()
        self.hello = None
        if kind == "client":
            f = concurrent.futures.Future()
            self._pending[0] = f
        self._reader = threading.Thread(target=self._read_loop, name="rca-client-reader", daemon=True)
        self._reader.start()
        self.conn.send((P.REGISTER, kind, ident, os.getpid(), register_extra))
        if kind == "client":
            self.hello = f.result(timeout=30)
        self._flusher = threading.Thread(target=self._flush_loop, name="rca-ref-flush", daemon=True)
        self._flusher.start()

    def _read_loop(self):
        while True:
            try:
                msg = self.conn.recv()
            except Exception:
                self._closed = True
                with self._lock:
                    for f in self._pending.values():
                        if not f.done():
                            f.set_exception(exc.RaySystemError("connection to the head was lost"))
                if self.on_message is not None:
                    try:
                        self.on_message((P.EXIT,))
                    except Exception:
                        pass
                return
            if msg[0] == P.REPLY:
                _, rid, ok, val = msg
                with self._lock:
                    f = self._pending.pop(rid, None)
                if f is not None:
                    if ok:
                        f.set_result(val)
                    else:
                        f.set_exception(val if isinstance(val, BaseException) else exc.RaySystemError(str(val)))
            elif self.on_message is not None:
                self.on_message(msg)

    def _flush_loop(self):
        while not self._closed:
            time.sleep(0.005)
            self.flush_refs()

    def flush_refs(self):
        if not self._adds and not self._removes:
            return
        with self._rlock:
            adds, self._adds = self._adds, []
            removes, self._removes = self._removes, []
        if adds or removes:
            try:
                self.conn.send((P.REF_DELTA, adds, removes))
            except OSError:
                pass

    def call_async(self, method, *args, **kwargs):
        rid = next(self._req)
        f = concurrent.futures.Future()
        with self._lock:
            self._pending[rid] = f
        self.flush_refs()
        if self._closed:
            raise exc.RaySystemError("connection to the head was lost")
        self.conn.send((P.RPC, rid, method, args, kwargs))
        return f

    def call(self, method, *args, **kwargs):
        return self.call_async(method, *args, **kwargs).result()

    def ref_delta(self, adds, removes):
        with self._rlock:
            self._adds.extend(adds)
            self._removes.extend(removes)

    def submit(self, spec):
        # fire-and-forget submission; errors surface through the return objects
        self.call_async("submit", spec)

    def send(self, msg):
        self.flush_refs()
        self.conn.send(msg)

    def close(self):
        self._closed = True
        self.conn.close()


# ====================================================================== CoreWorker
class TaskContext(threading.local):
    def __init__(self):
        self.task_id = None
        self.actor_id = None
        self.task_name = None
        self.put_index = 0
        self.pg_id = None        # placement group the running task / actor belongs to
        self.capture_pg = None   # strategy children inherit (placement_group_capture_child_tasks)
        self.runtime_env = None


class CoreWorker:
    def __init__(self, mode: str, client, store: ObjectStore, node_id: str, job_id: bytes, namespace: str = "",
                 worker_id: Optional[bytes] = None, session_dir: str = ""):
        self.mode = mode  # "driver" | "worker" | "client"
        self.client = client
        self.store = store
        self.node_id = node_id
        self.job_id = job_id
        self.namespace = namespace
        self.worker_id = worker_id or new_id()
        self.session_dir = session_dir
        self._refs: Dict[bytes, int] = {}
        self._ref_lock = threading.Lock()
        self._ready_known = set()  # head-managed objects a wait() saw ready (dropped with the last ref)
        self._wait_rest = None  # (weakref to list, len): the remainder the last wait() returned, all owned + unique
        self.ctx = TaskContext()
        self.registered_functions = set()
        self.actor_id = None
        self.gpu_ids = ()
        self.assigned_resources = {}
        self.current_actor = None
        self._shutdown = False
        from .direct_transport import OwnedTable

        self.owned = OwnedTable(self)
        self.channels: Dict[bytes, Any] = {}
        self._chan_lock = threading.Lock()
        self.direct_actor_calls = os.environ.get("RCA_DIRECT_ACTOR_CALLS", "1") != "0"
        # normal tasks over leased workers (direct_transport.TaskLeaseChannel), per resource shape
        self.direct_task_calls = os.environ.get("RCA_DIRECT_TASK_CALLS", "1") != "0"
        self.task_channels: Dict[tuple, Any] = {}
        self.worker_links: Dict[str, Any] = {}
        # (tid, name, None, start, end, failed, error type, worker id, node) of leased tasks this
        # process submitted, batched to the head (state API / timeline)
        self.task_records: List[tuple] = []
        self._records_armed = False
        # ray.put of host objects does not wait for the head: the registration is sent on this
        # process's (ordered) head connection and acknowledged later. A ref that escapes this
        # process -- serialized into any value, or passed as a task / actor argument over a direct
        # channel -- first waits for the acks of the puts it names (``sync_puts``), so no other
        # process can ask the head for an object it has not registered yet.
        self._unacked: Dict[bytes, Any] = {}
        self._put_lock = threading.Lock()
        # inline descriptors of this process's own live puts: ray.get on them is local
        self._put_cache: Dict[bytes, tuple] = {}
        # puts the head REJECTED (the error arrives only on the ack future): the next get / wait of
        # such a ref raises it instead of answering from _put_cache
        self._put_errors: Dict[bytes, BaseException] = {}
        # shm-store descriptors this process already resolved through the head, for refs it holds:
        # a repeated get maps the object straight from the shared-memory store (the native pin
        # fails if it was spilled / evicted / freed since, and then the head is asked again)
        self._shm_descs: Dict[bytes, tuple] = {}
        ser.set_escape_hook(self.sync_puts)

    # -------------------------------------------------------------- reference counting
    def ref_add(self, oid):
        with self._ref_lock:
            n = self._refs.get(oid, 0)
            self._refs[oid] = n + 1
        if n == 0:
            if oid in self.owned.objs and self.owned.revive(oid):
                return
            self.client.ref_delta((oid,), ())

    def ref_remove(self, oid):
        if self._shutdown:
            return
        with self._ref_lock:
            n = self._refs.get(oid, 0) - 1
            if n <= 0:
                self._refs.pop(oid, None)
            else:
                self._refs[oid] = n
        if n == 0:
            self._ready_known.discard(oid)
            self._put_cache.pop(oid, None)
            self._put_errors.pop(oid, None)
            self._shm_descs.pop(oid, None)
            if oid in self.owned.objs and not self.owned.drop(oid):
                return  # a caller-owned result the head never heard of
            self.client.ref_delta((), (oid,))

    def ref_remove_server_pin(self, oid):
        """The head pre-registered this process as a holder when it handed out ``oid``;
        ObjectRef creation already counted it — nothing to undo (holder sets are idempotent)."""

    def local_ref_count(self, oid):
        return self._refs.get(oid, 0)

    # -------------------------------------------------------------- objects
    def gpu_info(self, oid):
        """HBM accounting record of a GPU object this process owns (None for host objects)."""
        from .gpu_store import local_store

        return local_store().info(oid)

    def _store_serialized(self, oid, s: ser.Serialized, copy_gpu: bool = True):
        if s.gpu_tensors:
            # CUDA tensors stay in HBM, owned by this process's GPU object store; the wire bytes
            # (host parts + IPC export table) travel inline
            from .gpu_store import local_store

            b = local_store().add(oid, s, copy=copy_gpu and os.environ.get("RCA_GPU_PUT_COPY", "1") != "0")
            return ("inline", b, len(b))
        if s.total_size <= INLINE_THRESHOLD:
            b = s.to_bytes()
            return ("inline", b, len(b))
        if self.store.put_serialized(oid, s):
            return ("shm", None, s.total_size)
        # store full: ask the head to spill, retry, else write a spill file directly
        for _ in range(3):
            self.client.call("make_room", s.total_size)
            if self.store.put_serialized(oid, s):
                return ("shm", None, s.total_size)
        path = os.path.join(self.session_dir or "/tmp", "spill", oid.hex())
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "wb") as f:
            f.write(s.to_bytes())
        return ("spill", path, s.total_size)

    def put(self, value, _owner_address=None) -> ObjectRef:
        if isinstance(value, ObjectRef):
            raise TypeError("Calling put() on an ObjectRef is not allowed.")
        oid = new_id()
        s = ser.serialize(value)
        is_gpu = bool(s.gpu_tensors)
        desc = self._store_serialized(oid, s)
        ref = ObjectRef(oid, _register=False)
        with self._ref_lock:
            self._refs[oid] = self._refs.get(oid, 0) + 1
        if is_gpu:
            self.client.call("put", oid, desc, s.contained, self.gpu_info(oid), s.flags)
            return ref
        fut = self.client.call_async("put", oid, desc, s.contained, False, s.flags)
        if not fut.done():
            with self._put_lock:
                self._unacked[oid] = fut
            if desc[0] == "inline":
                self._put_cache[oid] = (desc[0], desc[1], desc[2], s.flags)
            fut.add_done_callback(lambda f, o=oid: self._acked(o, f))
            return ref
        if fut.exception() is not None:
            raise fut.exception()
        if desc[0] == "inline":
            self._put_cache[oid] = (desc[0], desc[1], desc[2], s.flags)
        return ref

    def _acked(self, oid, fut=None):
        err = None
        if fut is not None and not fut.cancelled():
            err = fut.exception()
        with self._put_lock:
            self._unacked.pop(oid, None)
            if err is not None:
                # the head never registered it: the locally cached value must not be served
                self._put_cache.pop(oid, None)
                self._put_errors[oid] = err

    def forget_puts(self, oids):
        """``ray.internal.free``: freed objects are no longer answered from the local caches."""
        for o in oids:
            self._put_cache.pop(o, None)
            self._shm_descs.pop(o, None)

    def _raise_put_errors(self, oids):
        pe = self._put_errors
        if pe:
            for o in oids:
                e = pe.get(o)
                if e is not None:
                    raise e

    def sync_puts(self, oids=None):
        """Wait until the head has registered this process's puts among ``oids`` (all if None)."""
        if not self._unacked:
            return
        if threading.current_thread() is getattr(self.client, "_reader", None):
            return  # the acks arrive on this very thread; its messages are ordered after the puts anyway
        with self._put_lock:
            if oids is None:
                futs = list(self._unacked.values())
            else:
                futs = [f for f in (self._unacked.get(o) for o in oids) if f is not None]
        for f in futs:
            f.result()

    def free_gpu_objects(self, oids):
        from .gpu_store import local_store

        local_store().free(oids)

    def gpu_command(self, cmd, oids):
        """The head asks this owner to spill GPU objects to pinned host memory or restore them."""
        from .gpu_store import local_store

        st = local_store()
        if cmd == "spill":
            done = [o for o in oids if st.spill(o)]
            self.client.call_async("gpu_spilled", done)
        elif cmd == "restore":
            for o in oids:
                b = st.restore(o)
                self.client.call_async("gpu_restored", o, ("inline", b, len(b)) if b is not None else None,
                                       self.gpu_info(o))

    def _note_shm(self, oids, descs):
        refs = self._refs
        for o, d in zip(oids, descs):
            if d is not None and d[0] == "shm" and not (d[3] & ser.FLAG_GPU) and refs.get(o):
                self._shm_descs[o] = d

    def _materialize(self, oid, desc):
        kind, data, size, flags = desc
        if kind == "inline":
            value, _ = ser.deserialize(data)
        elif kind == "shm":
            view = self.store.pin(oid)
            if view is None:
                # raced with spilling (or a cached descriptor went stale): ask again (the head
                # restores it)
                self._shm_descs.pop(oid, None)
                d2 = self.client.call("get", [oid], None)[0]
                if d2[0] == "shm":
                    view = self.store.pin(oid)
                    if view is None:
                        raise exc.ObjectLostError(oid.hex())
                else:
                    return self._materialize(oid, d2)
            value, _ = ser.deserialize(memoryview(view))
        elif kind == "spill":
            with open(data, "rb") as f:
                value, _ = ser.deserialize(f.read())
        else:
            raise exc.RaySystemError(f"bad object descriptor {kind}")
        if flags & ser.FLAG_ERROR:
            return _ErrorValue(value)
        return value

    def get(self, refs, timeout=None, _raise=True):
        single = isinstance(refs, ObjectRef)
        if single:
            refs = [refs]
        for r in refs:
            if not isinstance(r, ObjectRef):
                raise TypeError(f"get() expects ObjectRefs, got {type(r)}")
        if not refs:
            return []
        oids = [r._id for r in refs]
        descs = self._get_descs(oids, timeout)
        out = []
        for oid, d in zip(oids, descs):
            v = self._materialize(oid, d)
            if isinstance(v, _ErrorValue):
                if _raise:
                    raise v.as_exception()
                v = v.err
            out.append(v)
        return out[0] if single else out

    def _get_descs(self, oids, timeout):
        """Descriptors for ``oids``: caller-owned results from the local table (no head round
        trip), the rest from the head."""
        self._raise_put_errors(oids)
        pc, sc = self._put_cache, self._shm_descs
        if pc or sc:
            hit = [pc.get(o) or sc.get(o) for o in oids]
            if None not in hit:
                return hit
        owned = self.owned.objs
        local = [o for o in oids if o in owned]
        if not local:
            descs = self.client.call("get", oids, timeout)
            self._note_shm(oids, descs)
            return descs
        deadline = None if timeout is None else time.monotonic() + timeout
        remote = [o for o in oids if o not in owned]
        got = {}
        if remote:
            for o, d in zip(remote, self.client.call("get", remote, timeout)):
                got[o] = d
        blocking = self.mode == "worker" and any(owned.get(o) is not None and owned[o].desc is None for o in local)
        if blocking:
            self.client.send((P.BLOCKED, True))
        try:
            for o, d in zip(local, self.owned.wait_descs(local, deadline)):
                got[o] = d
        finally:
            if blocking:
                self.client.send((P.BLOCKED, False))
        # GPU objects are managed by the head (spill / restore / owner death): ask it
        gpu = [o for o in local if got[o][3] & ser.FLAG_GPU]
        if gpu:
            rem = None if deadline is None else max(0.0, deadline - time.monotonic())
            for o, d in zip(gpu, self.client.call("get", gpu, rem)):
                got[o] = d
        return [got[o] for o in oids]

    def as_future(self, ref) -> concurrent.futures.Future:
        out = concurrent.futures.Future()
        if ref._id in self.owned.objs:
            def ready(d, oid=ref._id):
                if d[3] & ser.FLAG_GPU:  # GPU objects: current descriptor from the head
                    g = self.client.call_async("get", [oid], None)
                    g.add_done_callback(lambda f: _finish(f, oid))
                    return
                try:
                    v = self._materialize(oid, d)
                    if isinstance(v, _ErrorValue):
                        out.set_exception(v.as_exception())
                    else:
                        out.set_result(v)
                except BaseException as e:  # noqa
                    out.set_exception(e)

            def _finish(f, oid):
                try:
                    v = self._materialize(oid, f.result()[0])
                    if isinstance(v, _ErrorValue):
                        out.set_exception(v.as_exception())
                    else:
                        out.set_result(v)
                except BaseException as e:  # noqa
                    out.set_exception(e)

            self.owned.on_ready(ref._id, ready)
            return out
        f = self.client.call_async("get", [ref._id], None)

        def done(fut):
            try:
                d = fut.result()[0]
                v = self._materialize(ref._id, d)
                if isinstance(v, _ErrorValue):
                    out.set_exception(v.as_exception())
                else:
                    out.set_result(v)
            except BaseException as e:  # noqa
                out.set_exception(e)

        f.add_done_callback(done)
        return out

    def wait(self, refs, num_returns=1, timeout=None, fetch_local=True):
        if isinstance(refs, ObjectRef):
            raise TypeError("wait() expected a list of ObjectRefs")
        # Polling fast path (``ready, rest = wait(rest)``): ``refs`` is the unchanged remainder list
        # an earlier call returned, so its refs are known unique and all owned here; if its head
        # is already ready, answer with one slice instead of re-validating the whole list
        # (O(N) per call instead of five O(N) passes).
        # Only a weak reference to that list is cached: a caller that drops ``rest`` must release
        # its refs (free-on-last-ref), not have them pinned here until the next wait().
        last = self._wait_rest
        same = (num_returns == 1 and last is not None and refs is last[0]() and len(refs) == last[1] and refs)
        if same:
            e = self.owned.objs.get(refs[0]._id)
            if e is not None and e.desc is not None:
                rest = _RefList(refs[1:])
                self._wait_rest = (weakref.ref(rest), len(rest))
                return [refs[0]], rest
        self._wait_rest = None
        refs = list(refs)
        ids = list(map(_REF_ID, refs))  # C-level pass (wait() is called once per completion when polling)
        self._raise_put_errors(ids)
        owned = self.owned.objs
        if same:  # the unchanged remainder of an earlier wait: unique and all owned here already
            sids = None
        else:
            sids = set(ids)
            if len(sids) != len(ids):
                raise ValueError("Wait requires a list of unique object refs.")
            if num_returns <= 0:
                raise ValueError("Invalid number of objects to return %d." % num_returns)
            if num_returns > len(refs):
                raise ValueError("num_returns cannot be greater than the number of objects provided.")
        if sids is None or sids <= owned.keys():
            deadline = None if timeout is None else time.monotonic() + timeout
            got = self.owned.wait_ready(ids, num_returns, deadline)
        else:
            local = [o for o in ids if o in owned]
            for o in local:  # mixed with head-managed refs: let the head track them all
                self.owned.publish(o)
            # objects seen ready by an earlier wait stay ready while referenced: polling a shrinking
            # list (``ready, rest = wait(rest)``) is answered locally after one head round trip
            rk = self._ready_known
            known = [o for o in ids if o in rk]
            if len(known) >= num_returns:
                got = known
            else:
                got = self.client.call("wait", ids, num_returns, timeout, fetch_local, True)
                rk.update(got)
        if len(got) > num_returns:
            got = got[:num_returns]
        if len(got) <= 4:  # the polling case: split by position instead of two filtering passes
            idx = sorted(ids.index(o) for o in got)
            ready = [refs[i] for i in idx]
            not_ready, prev = _RefList(), 0
            for i in idx:
                not_ready.extend(refs[prev:i])
                prev = i + 1
            not_ready.extend(refs[prev:])
            if sids is None or sids <= owned.keys():
                self._wait_rest = (weakref.ref(not_ready), len(not_ready))
            return ready, not_ready
        rs = set(got)
        ready = [r for r in refs if r._id in rs]
        not_ready = [r for r in refs if r._id not in rs]
        return ready, not_ready

    # -------------------------------------------------------------- functions
    def function_id(self, blob: bytes) -> bytes:
        return hashlib.sha1(blob).digest()

    # -------------------------------------------------------------- args
    def encode_args(self, args, kwargs):
        out = []
        contained = []
        deps = []
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, ObjectRef):
                out.append(("r", a._id))
                deps.append(a)
                if self._unacked:
                    self.sync_puts((a._id,))
                continue
            s = ser.serialize(a)
            if s.gpu_tensors:
                # GPU tensors passed by value become GPU objects owned by this process (snapshot)
                ref = self._put_serialized(s)
                out.append(("r", ref._id))
                deps.append(ref)
                continue
            if s.total_size > INLINE_THRESHOLD:
                ref = self._put_serialized(s)
                out.append(("r", ref._id))
                deps.append(ref)
                continue
            out.append(("v", s.to_bytes()))
            contained.extend(s.contained)
        return out, list(kwargs.keys()), contained, deps

    def _put_serialized(self, s):
        oid = new_id()
        is_gpu = bool(s.gpu_tensors)
        desc = self._store_serialized(oid, s)
        ref = ObjectRef(oid, _register=False)
        with self._ref_lock:
            self._refs[oid] = self._refs.get(oid, 0) + 1
        self.client.call("put", oid, desc, s.contained, self.gpu_info(oid) if is_gpu else False, s.flags)
        return ref

    def submit_spec(self, spec, deps=()):
        spec["parent"] = self.ctx.task_id
        spec["caller_node"] = self.node_id
        trace = tracing.submission_context()
        if trace is not None:
            spec["trace"] = trace
        if self.direct_task_calls and _leasable(spec):
            return self._submit_leased(spec, deps)
        owned = self.owned.objs
        for a in spec["args"]:
            if a[0] == "r" and a[1] in owned:
                self.owned.publish(a[1])  # the head schedules this task: it must know its inputs
        self.client.submit(spec)

    def flush_task_records(self):
        self._records_armed = False
        if not self.task_records:
            return
        recs, self.task_records = self.task_records, []
        try:
            self.client.call_async("direct_task_records", recs)
        except Exception:  # noqa  (the session is going away)
            pass

    def _submit_leased(self, spec, deps):
        blob = spec.pop("fblob", None)
        if blob is not None:  # workers fetch functions they have not seen from the head
            self.client.call("register_function", spec["fid"], blob)
        spec["owner_key"] = self.client.key
        res = spec.get("resources") or {}
        key = tuple(sorted((k, v) for k, v in res.items() if v > 0))
        ch = self.task_channels.get(key)
        if ch is None:
            from .direct_transport import TaskLeaseChannel

            with self._chan_lock:
                ch = self.task_channels.get(key)
                if ch is None:
                    ch = self.task_channels[key] = TaskLeaseChannel(self, dict(key))
        ch.submit(spec, list(deps))

    def submit_actor_task(self, spec, deps):
        """Actor calls go straight to the actor's worker (``direct_transport.ActorChannel``);
        generator methods keep the head-routed path."""
        if not self.direct_actor_calls or spec.get("generator") is not None:
            return self.submit_spec(spec, deps)
        spec["parent"] = self.ctx.task_id
        spec["caller_node"] = self.node_id
        spec["owner_key"] = self.client.key
        trace = tracing.submission_context()
        if trace is not None:
            spec["trace"] = trace
        aid = spec["actor_id"]
        ch = self.channels.get(aid)
        if ch is None:
            from .direct_transport import ActorChannel

            with self._chan_lock:
                ch = self.channels.get(aid)
                if ch is None:
                    ch = ActorChannel(self, aid)
                    self.channels[aid] = ch
        # object refs nested in the arguments stay pinned at the head until the call returns (the
        # head-routed path pins ``contained`` in its submit; the caller may drop its refs first)
        nested = tuple(o for o in spec.get("contained") or () if o[:1] != b"A")
        rids = spec.get("return_ids")
        if nested and rids:
            self.client.call_async("pin_objects", nested, 1)
        ch.submit(spec, list(deps))
        if nested and rids:
            self.owned.on_ready(rids[0], lambda _d, c=nested: self.client.call_async("pin_objects", c, -1))

    def cancel(self, oid, force=False, recursive=True):
        e = self.owned.objs.get(oid)
        if e is not None:
            if e.desc is not None or e.channel is None:
                return False
            return e.channel.cancel(e.tid, force)
        return self.client.call("cancel", oid, force, recursive)

    def shutdown(self):
        self._shutdown = True
        for ch in list(self.channels.values()):
            ch.close()
        self.channels.clear()
        for ch in list(self.task_channels.values()):
            ch.close()
        self.task_channels.clear()
        for link in list(self.worker_links.values()):
            link.close()
        self.worker_links.clear()


def _leasable(spec) -> bool:
    """Normal tasks that run on a leased worker pushed by their caller: plain CPU-shaped tasks
    (no placement group / strategy, runtime_env, GPU, generator, or refs nested in inline args,
    which the head pins while a head-scheduled task runs)."""
    if spec["kind"] != "task" or spec.get("generator") is not None or spec.get("strategy") is not None:
        return False
    if spec.get("runtime_env") or spec.get("contained") or spec.get("max_calls") or spec.get("label_selector"):
        return False  # (max_calls: the worker retires after N calls; label selectors: node choice -- head-scheduled)
    for k in (spec.get("resources") or {}):
        if k == "GPU" or k.startswith("GPU_group") or k.startswith("accelerator_type"):
            return False
    return True


class _ErrorValue:
    __slots__ = ("err",)

    def __init__(self, err):
        self.err = err

    def as_exception(self):
        e = self.err
        if isinstance(e, exc.RayTaskError):
            return e.as_instanceof_cause()
        return e
