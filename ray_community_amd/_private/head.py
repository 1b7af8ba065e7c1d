"""The head service: GCS tables + raylet (scheduler, worker pool, object directory) in one.

Reference counterparts: ``src/ray/gcs/gcs_server/*`` (actor / placement-group / node / KV tables),
``src/ray/raylet/{node_manager,worker_pool,local_task_manager}.cc``, and the ownership /
reference-counting logic of ``src/ray/core_worker/{reference_count,task_manager}.cc``.

Design: one head per session, living in the driver process (or in its own process via
``ray_community_amd.scripts start --head``). A selector thread serves worker connections; driver
API calls enter the same state machine directly under ``self.lock``. Resource accounting and
queueing are delegated to the C++ ``Scheduler``; objects live in the C++ shm store. Node
"virtualisation" (``cluster_utils.Cluster``) = extra scheduler nodes with their own worker pools.
"""
from __future__ import annotations

import collections
import json
import logging
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import threading
import time
import traceback
from typing import Any, Callable, Dict, List, Optional, Set

from .. import exceptions as exc
from . import protocol as P
from .gc_tuning import restore_gc, tune_gc
from .log_monitor import LogMonitor, read_log
from .ids import new_id
from .object_store import ObjectStore, default_store_capacity, native
from .serialization import FLAG_ERROR, serialize

log = logging.getLogger("ray_community_amd.head")

DRIVER = "driver"
INLINE_THRESHOLD = 100 * 1024

# object states
PENDING, READY, FREED = 0, 1, 2
# task states
T_WAIT_DEPS, T_QUEUED, T_WAIT_WORKER, T_RUNNING, T_FINISHED, T_FAILED, T_CANCELLED = range(7)
TASK_STATE_NAMES = ["PENDING_ARGS_AVAIL", "PENDING_NODE_ASSIGNMENT", "PENDING_WORKER", "RUNNING", "FINISHED",
                    "FAILED", "CANCELLED"]
# actor states
A_PENDING, A_ALIVE, A_RESTARTING, A_DEAD = "PENDING_CREATION", "ALIVE", "RESTARTING", "DEAD"


class Deferred:
    __slots__ = ("callbacks", "done", "value", "ok")

    def __init__(self):
        self.callbacks = []
        self.done = False
        self.value = None
        self.ok = True

    def resolve(self, value, ok=True):
        if self.done:
            return
        self.done = True
        self.value = value
        self.ok = ok
        cbs, self.callbacks = self.callbacks, []
        for cb in cbs:
            cb(self)

    def add(self, cb):
        if self.done:
            cb(self)
        else:
            self.callbacks.append(cb)


class ObjEntry:
    # holders / pins live in the native reference table (Head.refs, _native/ref_table.cpp)
    __slots__ = ("oid", "state", "desc", "waiters", "contained", "task", "gpu_owner", "size",
                 "flags", "created", "gpu", "node")

    def __init__(self, oid, task=None):
        self.oid = oid
        self.state = PENDING
        self.desc = None
        self.waiters: List[Callable] = []
        self.contained: List[bytes] = []
        self.task = task
        self.gpu_owner = None
        self.size = 0
        self.flags = 0
        self.created = time.time()
        self.gpu = None  # GPU object accounting: {"nbytes", "gpus", "state", "last", "maps": {reader: n}}
        self.node = None  # node whose store holds the value (lost with the node)


class TaskState:
    __slots__ = ("tid", "spec", "state", "deps", "retries_left", "worker", "node", "demand", "owner", "key", "gpus",
                 "times", "children", "parent", "cancelled", "blocked", "gen_items", "gen_done", "gen_waiters",
                 "gen_consumed", "gen_bp_waiters", "gen_dropped",
                 "error_type", "attempt", "reply")

    def __init__(self, tid, spec, owner):
        self.tid = tid
        self.spec = spec
        self.state = T_WAIT_DEPS
        self.deps: Set[bytes] = set()
        self.retries_left = spec.get("max_retries", 0)
        self.worker = None
        self.node = None
        self.demand = {}
        self.owner = owner
        self.key = None
        self.gpus = ()
        self.times = {"submit": time.time()}
        self.children: List[bytes] = []
        self.parent = spec.get("parent")
        self.cancelled = False
        self.blocked = False
        self.gen_items: List[bytes] = []
        self.gen_consumed = 0          # items handed to the consumer (streaming backpressure)
        self.gen_bp_waiters: List = []  # (needed count, Deferred) of a paused producer
        self.gen_dropped = False  # the consumer dropped its ObjectRefGenerator (or its owner died)
        self.gen_done = False
        self.gen_waiters: Dict[int, List[Deferred]] = {}
        self.error_type = None
        self.attempt = 0
        self.reply: Optional[Deferred] = None  # leases: the grant reply


class ActorState:
    """Runtime handles of one actor (call queue, in-flight calls, waiters). What the actor is
    looked up by -- state, node, name, placement group, handle holders -- lives in the native
    actor directory (``Head.actor_dir``, _native/actor_table.cpp); ``state`` and ``node`` write
    through to it."""

    def __init__(self, aid, spec, owner, directory=None):
        self.aid = aid
        self.spec = spec
        self._dir = None
        self._state = A_PENDING
        self._node = None
        self.worker = None
        self.queue: collections.deque = collections.deque()
        self.inflight: Dict[bytes, TaskState] = {}
        self.restarts_left = spec.get("max_restarts", 0)
        self.num_restarts = 0
        self.name = spec.get("actor_name")
        self.namespace = spec.get("namespace", "")
        self.detached = spec.get("lifetime") == "detached"
        self.owner = owner
        self.demand = {}
        self.gpus = ()
        self.death_cause = None
        self.ready_waiters: List[Deferred] = []
        self.creation_task: Optional[TaskState] = None
        self.pid = None
        self.killed = False
        self.addr_waiters: List[tuple] = []  # (Deferred, min incarnation) of direct-call channels
        if directory is not None:
            st = spec.get("strategy") or {}
            directory.add(aid, self.name, self.namespace, owner, st.get("pg_id") if st.get("kind") == "pg" else None,
                          A_PENDING, spec.get("class_name") or "", self.detached)
            self._dir = directory

    @property
    def state(self):
        return self._state

    @state.setter
    def state(self, v):
        self._state = v
        if self._dir is not None:
            self._dir.set_state(self.aid, v)

    @property
    def node(self):
        return self._node

    @node.setter
    def node(self, v):
        self._node = v
        if self._dir is not None:
            self._dir.set_node(self.aid, v)


class WorkerState:
    def __init__(self, wid, node_id, env_key, proc, gpus):
        self.wid = wid
        self.node_id = node_id
        self.env_key = env_key
        self.proc = proc
        self.conn: Optional[socket.socket] = None
        self.reader = P.FrameReader()
        self.send_lock = threading.Lock()
        self.pid = proc.pid if proc else None
        self.state = "starting"
        self.task: Optional[TaskState] = None
        self.actor: Optional[ActorState] = None
        self.known_functions: Set[bytes] = set()
        self.gpus = gpus
        self.idle_since = time.time()
        self.dead = False
        self.gpu_objects: Set[bytes] = set()
        self.out = collections.deque()
        self.direct_addr: Optional[str] = None


def _pool_key(env_key) -> str:
    """The worker-pool index's flat string for a (runtime_env json, GPU ids) env key."""
    env, gpus = env_key
    return env + "\x00" + ",".join(str(g) for g in gpus)


class NodeState:
    def __init__(self, node_id, resources, labels=None, is_head=False):
        self.node_id = node_id
        self.resources = dict(resources)
        self.labels = labels or {}
        self.is_head = is_head
        self.dispatch_q: Dict[Any, collections.deque] = collections.defaultdict(collections.deque)
        self.gpu_free = [1.0] * int(resources.get("GPU", 0))
        self.alive = True
        self.start_time = time.time()


class Head:
    def __init__(self, session_dir: str, resources: dict, object_store_memory: Optional[int] = None,
                 namespace: str = "", system_config: Optional[dict] = None, job_id: Optional[bytes] = None,
                 labels: Optional[dict] = None):
        self.lock = threading.RLock()
        self.session_dir = session_dir
        os.makedirs(session_dir, exist_ok=True)
        self.spill_dir = os.path.join(session_dir, "spill")
        os.makedirs(self.spill_dir, exist_ok=True)
        self.logs_dir = os.path.join(session_dir, "logs")
        os.makedirs(self.logs_dir, exist_ok=True)
        self.config = dict(system_config or {})
        # in-process head (local ray.init inside the user's driver): raise the threshold only,
        # no freeze, and put the driver's setting back at shutdown
        self._prev_gc = tune_gc(self.config, freeze=False)
        self.namespace = namespace
        self.job_id = job_id or new_id()
        self.sched = native().Scheduler(float(self.config.get("scheduler_spread_threshold", 0.5)))
        self.label_selectors: Dict[str, list] = {}  # synthetic resource name -> selector clauses
        cap = object_store_memory or default_store_capacity()
        # random, not derived from new_id(): its last bytes are a per-process counter, so two
        # sessions on one machine would pick the same segment name and unlink each other's store
        self.store_name = "/rca_" + os.urandom(8).hex()
        self.store = ObjectStore(self.store_name, cap, create=True)
        self.store_capacity = cap
        self.objects: Dict[bytes, ObjEntry] = {}
        # who keeps each object alive (holder keys + anonymous pins) and where its value lives:
        # C++ (_native/ref_table.cpp), with a holder -> objects index so a process death frees
        # what it held without scanning every object
        self.refs = native().RefTable()
        self.tasks: Dict[bytes, TaskState] = {}
        self.task_keys: Dict[int, TaskState] = {}
        self._key = 0
        self.actors: Dict[bytes, ActorState] = {}
        # actor directory: name / node / placement-group / handle-holder indexes (C++)
        self.actor_dir = native().ActorDirectory(A_DEAD)
        self.workers: Dict[bytes, WorkerState] = {}
        # worker-pool index (C++: idle stacks per (node, env key), spawned-not-registered counts,
        # idle reaping); the WorkerState objects stay in self.workers
        self.wpool = native().WorkerPool()
        self.nodes: Dict[str, NodeState] = {}
        # placement-group table (C++: records, name index, pending FIFO, state counts); the
        # pg.ready() waiters stay here
        self.pg_dir = native().PgDirectory()
        self.pg_waiters: Dict[bytes, list] = {}
        self.kv = native().KvTable()  # internal KV (GCS InternalKV)
        self.functions: Dict[bytes, bytes] = {}
        self.events: collections.deque = collections.deque(maxlen=int(self.config.get("task_events_max", 100000)))
        self.finished_tasks: collections.deque = collections.deque(maxlen=10000)
        # lineage of reconstructable task outputs: tid -> [spec, owner, attempts left]; bounded LRU
        self.lineage: "collections.OrderedDict[bytes, list]" = collections.OrderedDict()
        self.lineage_max = int(self.config.get("max_lineage_entries", 100000))
        # caller key -> {oid: n}: pins taken for direct actor calls' nested refs (rpc_pin_objects),
        # released here if the caller dies before its own unpin
        self.call_pins: Dict[str, Dict[bytes, int]] = {}
        self.num_reconstructions = 0
        # records of directly transported actor calls (state API / timeline), batched by workers
        self.direct_tasks: collections.deque = collections.deque(maxlen=int(self.config.get("direct_task_records", 10000)))
        # worker leases of direct task submitters: lease id -> TaskState (kind "lease")
        self.leases: Dict[bytes, TaskState] = {}
        self.leases_by_owner: Dict[str, Set[bytes]] = {}
        self.lease_fates: Dict[bytes, BaseException] = {}
        self.lease_fate_waiters: Dict[bytes, List[Deferred]] = {}
        self.timers: List[tuple] = []
        self.spilled_bytes = 0
        self.num_spilled = 0
        self.num_restored = 0
        self.driver_gpu_objects: Set[bytes] = set()
        self.driver_free_gpu_cb = None
        self.driver_gpu_cmd_cb = None
        # GPU object store accounting (per physical GPU), see _private/gpu_store.py
        self.gpu_budget = int(self.config.get("gpu_object_store_memory") or _default_gpu_budget())
        self.gpu_usage: Dict[str, int] = {}
        self.gpu_objects: Dict[bytes, ObjEntry] = {}
        self.gpu_spilled_bytes = 0
        self.gpu_num_spilled = 0
        self.gpu_num_restored = 0
        self.driver_task_cancel_cb = None
        self.shutting_down = False
        from .memory_monitor import MemoryMonitor

        self.memory_monitor = MemoryMonitor(self.config)
        self._oom_log: collections.deque = collections.deque(maxlen=1000)
        # cluster events for the state API (node added/removed, worker died, OOM kills)
        self.cluster_events: collections.deque = collections.deque(maxlen=10000)
        self.spans: collections.deque = collections.deque(maxlen=int(self.config.get("max_spans", 200000)))
        # head node
        self.head_node_id = new_id().hex()
        self._add_node(self.head_node_id, resources, labels, is_head=True)
        # network
        self.sock_path = os.path.join(session_dir, "head.sock")
        if len(self.sock_path.encode()) > 100:  # sun_path is 108 bytes: fall back to a short name
            self.sock_path = os.path.join(tempfile.gettempdir(), f"rca-{os.urandom(6).hex()}.sock")
        if os.path.exists(self.sock_path):
            os.unlink(self.sock_path)
        self.listener = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.listener.bind(self.sock_path)
        self.listener.listen(1024)
        self.listener.setblocking(False)
        # native epoll reactor (_native/reactor.cpp): accepts, reads and splits frames in C++
        # with the GIL released; the loop gets every frame that arrived in one batch
        self.reactor = native().Reactor()
        self.reactor.add(self.listener.fileno(), -1, True)
        self.conns: Dict[int, tuple] = {}  # fd -> (socket, ClientConn)
        self.conn_worker: Dict[int, WorkerState] = {}
        self.clients: Dict[int, "ClientConn"] = {}
        self._thread = threading.Thread(target=self._loop, name="rca-head", daemon=True)
        self._thread.start()
        # worker stdout/stderr -> drivers (log_to_driver); see _private/log_monitor.py
        self.log_monitor = LogMonitor(self._describe_worker_logs, self.lock,
                                      float(self.config.get("log_monitor_interval_s", 0.1)))
        if self.config.get("log_monitor", True):
            self.log_monitor.start()
        prestart = int(self.config.get("prestart_workers", min(2, int(resources.get("CPU", 1)))))
        with self.lock:
            for _ in range(prestart):
                self._start_worker(self.nodes[self.head_node_id], self._env_key({}, ()), ())

    # ================================================================== nodes
    def _add_node(self, node_id, resources, labels=None, is_head=False):
        res = {k: float(v) for k, v in resources.items() if v}
        res.setdefault("memory", 8e9)
        res[f"node:{node_id}"] = 1.0
        if is_head:
            res["node:__internal_head__"] = 1.0
        for name, clauses in getattr(self, "label_selectors", {}).items():
            if self._selector_matches(labels, clauses):
                res[name] = 1e6
        self.sched.add_node(node_id, res)
        self.nodes[node_id] = NodeState(node_id, {k: v for k, v in res.items() if not k.startswith("__labelsel:")},
                                        labels, is_head)
        self._cluster_event("INFO", "NODE", f"node {node_id[:8]} added", node_id=node_id)
        return node_id

    # ------------------------------------------------------------ label selectors
    # ``label_selector`` / ``NodeLabelSchedulingStrategy`` hard constraints become a synthetic
    # resource per distinct selector, present (with a capacity no task exhausts) exactly on the
    # nodes whose labels match; the native scheduler then only places the task on those nodes.
    @staticmethod
    def _label_clause_ok(labels, key, op, values):
        have = labels.get(key)
        if op == "in":
            return have is not None and have in values
        if op == "not_in":
            return have is None or have not in values
        if op == "exists":
            return have is not None
        if op == "not_exists":
            return have is None
        raise ValueError(f"unknown label operator {op}")

    def _selector_matches(self, labels, clauses):
        return all(self._label_clause_ok(labels or {}, k, op, vals) for k, op, vals in clauses)

    def _selector_resource(self, clauses) -> str:
        import hashlib

        canon = json.dumps(sorted([k, op, sorted(vals)] for k, op, vals in clauses))
        name = "__labelsel:" + hashlib.sha1(canon.encode()).hexdigest()[:16]
        if name not in self.label_selectors:
            self.label_selectors[name] = clauses
            for nid, n in self.nodes.items():
                if n.alive and self._selector_matches(n.labels, clauses):
                    self.sched.adjust(nid, {name: 1e6})
        return name

    def add_node(self, resources: dict, labels=None) -> str:
        with self.lock:
            nid = new_id().hex()
            self._add_node(nid, resources, labels)
            self._schedule()
            return nid

    def remove_node(self, node_id: str):
        with self.lock:
            node = self.nodes.get(node_id)
            if node is None or node.is_head:
                return
            node.alive = False
            self.sched.remove_node(node_id)
            self.wpool.drop_node(node_id)
            self._cluster_event("ERROR", "NODE", f"node {node_id[:8]} removed", node_id=node_id)
            for w in list(self.workers.values()):
                if w.node_id == node_id and not w.dead:
                    self._kill_worker(w)
            # objects in the node's store are gone with it: reconstruct from lineage or fail
            on_node = (self.objects.get(o) for o in self.refs.objects_on_node(node_id))
            for e in [e for e in on_node if e is not None and e.node == node_id and e.state == READY and e.desc
                      and e.desc[0] in ("shm", "spill")]:
                self._lose_object(e)
            self._schedule()

    # ================================================================== main loop
    def _loop(self):
        reactor = self.reactor
        loads = P.loads
        while not self.shutting_down:
            try:
                events = reactor.poll(50)
            except Exception:  # noqa
                if self.shutting_down:
                    return
                raise
            if events:
                self._on_events(events, loads)
            if self.timers:
                self._fire_timers()
            self._reap_idle()
            self.memory_monitor.poll(self)

    def _on_events(self, events, loads):
        conns = self.conns
        batch = []  # consecutive frames handled under one lock acquisition
        for kind, token, fd, payload in events:
            if kind == 0:
                ent = conns.get(fd)
                if ent is not None:
                    try:
                        batch.append((ent[1], loads(payload)))
                    except Exception:
                        log.error("head: undecodable frame\n%s", traceback.format_exc())
                continue
            if batch:
                self._handle_batch(batch)
                batch = []
            if kind == 2:
                c = socket.socket(fileno=fd)
                c.setblocking(True)
                cc = ClientConn(c)
                conns[fd] = (c, cc)
                self.reactor.add(fd, fd)
            elif kind == 1:
                ent = conns.pop(fd, None)
                if ent is not None:
                    self._on_disconnect(ent[0], ent[1])
        if batch:
            self._handle_batch(batch)

    def _handle_batch(self, batch):
        with self.lock:
            for cc, msg in batch:
                try:
                    self._handle(cc, msg)
                except Exception:
                    log.error("head: error handling %s\n%s", msg[0], traceback.format_exc())

    def wake(self):
        try:
            self.reactor.wake()
        except Exception:  # noqa
            pass

    def _on_disconnect(self, sock, cc):
        try:
            self.reactor.remove(sock.fileno())
        except Exception:
            pass
        try:
            sock.close()
        except Exception:
            pass
        with self.lock:
            if cc.worker is not None:
                self._on_worker_death(cc.worker, "worker process exited")
            elif cc.client_key is not None:
                if getattr(cc, "log_sink", None) is not None:
                    self.log_monitor.remove_sink(cc.log_sink)
                self._return_leases_of(cc.client_key)
                self._release_call_pins(cc.client_key)
                self._drop_streams_of(cc.client_key)
                self._drop_holder_everywhere(cc.client_key)
                self._schedule()

    def _send(self, cc_or_worker, msg):
        conn = cc_or_worker.conn if isinstance(cc_or_worker, WorkerState) else cc_or_worker
        if conn is None:
            return
        try:
            conn.send(msg)
        except OSError:
            pass

    # ================================================================== message dispatch
    def _handle(self, cc, msg):
        t = msg[0]
        if t == P.TASK_DONE:
            self._on_task_done(cc.worker, msg[1], msg[2], msg[3])
        elif t == P.RPC:
            _, req_id, method, args, kwargs = msg
            caller = cc.key()
            try:
                fn = getattr(self, "rpc_" + method)
                res = fn(caller, *args, **kwargs)
            except Exception as e:
                self._send(cc, (P.REPLY, req_id, False, e))
                return
            if isinstance(res, Deferred):
                res.add(lambda d, cc=cc, req_id=req_id: self._send(cc, (P.REPLY, req_id, d.ok, d.value)))
            else:
                self._send(cc, (P.REPLY, req_id, True, res))
        elif t == P.REF_DELTA:
            key = cc.key()
            for oid in msg[1]:
                self._add_holder(oid, key)
            for oid in msg[2]:
                self._remove_holder(oid, key)
        elif t == P.GEN_ITEM:
            self._on_gen_item(msg[1], msg[2], msg[3])
        elif t == P.BLOCKED:
            self._on_blocked(cc.worker, msg[1])
        elif t == P.DIRECT_EVENTS:
            self._on_direct_events(cc.worker, msg[1])
        elif t == P.REGISTER:
            self._on_register(cc, msg)
        elif t == P.LOG:
            pass

    def _on_register(self, cc, msg):
        _, kind, ident, pid = msg[:4]
        if kind == "worker":
            w = self.workers.get(ident)
            if w is None or w.dead:
                self._send(cc.conn, (P.EXIT,))  # a late/stale worker; it may already be gone
                return
            cc.worker = w
            self.start_failures = 0
            w.conn = cc.conn
            extra = msg[4] if len(msg) > 4 and isinstance(msg[4], dict) else {}
            w.direct_addr = extra.get("direct_addr")
            w.pid = pid
            w.state = "idle"
            self.wpool.add_starting(w.node_id, _pool_key(w.env_key), -1)
            self._worker_available(w)
        else:  # client driver
            cc.client_key = "client:" + ident.hex()
            extra = msg[4] if len(msg) > 4 and isinstance(msg[4], dict) else {}
            if extra.get("log_to_driver"):
                cc.log_sink = lambda batches, cc=cc: self._send(cc, (P.LOG_BATCH, batches))
                self.log_monitor.add_sink(cc.log_sink)
            cc.conn.send((P.REPLY, 0, True, {"store": self.store_name, "node_id": self.head_node_id,
                                              "job_id": self.job_id, "namespace": self.namespace,
                                              "session_dir": self.session_dir}))

    # ================================================================== objects
    def _obj(self, oid, create=True, task=None) -> Optional[ObjEntry]:
        e = self.objects.get(oid)
        if e is None and create:
            e = ObjEntry(oid, task)
            self.objects[oid] = e  # its reference record is created by the first holder or pin
        return e

    def _add_holder(self, oid, key):
        e = self.objects.get(oid)
        if e is None:
            if oid[:1] == b"A":
                a = self.actors.get(oid[1:])
                if a is not None:
                    self.actor_dir.add_handle(a.aid, key)
            return
        if e.state != FREED:
            self.refs.add_holder(oid, key)

    def _remove_holder(self, oid, key):
        if oid[:1] == b"A" and len(oid) == 21:
            a = self.actors.get(oid[1:])
            if a is not None:
                self.actor_dir.remove_handle(a.aid, key)
                self._maybe_kill_unreferenced(a)
            return
        e = self.objects.get(oid)
        if e is None:
            return
        if self.refs.remove_holder(oid, key):
            self._maybe_free(e)

    def _pin(self, oid, n=1) -> bool:
        e = self.objects.get(oid)
        if e is not None:
            self.refs.pin(oid, n)
            return True
        if oid[:1] == b"A" and len(oid) == 21:
            a = self.actors.get(oid[1:])
            if a is not None:
                a.pins = getattr(a, "pins", 0) + n
                return True
        return False

    def _unpin(self, oid, n=1):
        e = self.objects.get(oid)
        if e is not None:
            if self.refs.pin(oid, -n):
                self._maybe_free(e)
        elif oid[:1] == b"A" and len(oid) == 21:
            a = self.actors.get(oid[1:])
            if a is not None:
                a.pins = getattr(a, "pins", 0) - n
                self._maybe_kill_unreferenced(a)

    def _maybe_kill_unreferenced(self, a):
        if self.actor_dir.num_handles(a.aid) or getattr(a, "pins", 0) > 0 or a.detached or a.state == A_DEAD or a.name:
            return
        if a.queue or a.inflight:
            return  # submitted calls keep the actor alive until they finish (re-checked on completion)
        self._kill_actor(a, no_restart=True, reason="all handles to the actor went out of scope")

    def _maybe_free(self, e: ObjEntry):
        if e.state == FREED or self.refs.referenced(e.oid):
            return
        if e.state == PENDING:
            return  # freed when the producing task completes (result discarded)
        self._free(e)

    def _free(self, e: ObjEntry):
        e.state = FREED
        d = e.desc
        if d is not None:
            if d[0] == "shm":
                self.store.delete(e.oid)
            elif d[0] == "spill":
                try:
                    os.unlink(d[1])
                except OSError:
                    pass
        if e.gpu_owner is not None:
            self._gpu_unaccount(e)
            self._free_gpu_object(e.gpu_owner, e.oid)
        e.desc = None
        for c in e.contained:
            self._unpin(c)
        e.contained = []
        self.objects.pop(e.oid, None)
        self.refs.erase(e.oid)

    def _free_gpu_object(self, owner, oid):
        if owner == DRIVER:
            if self.driver_free_gpu_cb:
                self.driver_free_gpu_cb([oid])
            return
        w = self.workers.get(owner)
        if w is not None and not w.dead:
            self._send(w, (P.FREE_GPU, [oid]))

    def _drop_holder_everywhere(self, key):
        for e in list(self.gpu_objects.values()):
            if e.gpu is not None:
                e.gpu["maps"].pop(key, None)
        for oid in self.refs.drop_holder(key):  # only the objects this holder kept alive
            e = self.objects.get(oid)
            if e is not None:
                self._maybe_free(e)
        for aid in self.actor_dir.drop_holder(key):  # only the actors this holder had handles to
            a = self.actors.get(aid)
            if a is not None:
                self._maybe_kill_unreferenced(a)

    def _set_ready(self, e: ObjEntry, desc, contained=(), gpu_owner=None, flags=0, gpu_info=None):
        if e.state == FREED:
            return
        if gpu_owner is not None and isinstance(gpu_info, dict):
            self._gpu_account(e, gpu_info)
        e.desc = desc
        e.flags = flags
        e.size = desc[2] or 0
        e.contained = list(contained)
        for c in e.contained:
            self._pin(c)
        e.gpu_owner = gpu_owner
        e.state = READY
        ws, e.waiters = e.waiters, []
        for cb in ws:
            cb(e)
        if not self.refs.referenced(e.oid):
            self._free(e)

    def _set_error(self, e: ObjEntry, err: BaseException):
        b = serialize(err, error=True).to_bytes()
        self._set_ready(e, ("inline", b, len(b)), flags=FLAG_ERROR)

    def _when_ready(self, oids, cb_each):
        for oid in oids:
            e = self.objects.get(oid)
            if e is None or e.state != PENDING:
                cb_each(oid)
            else:
                e.waiters.append(lambda e, oid=oid: cb_each(oid))

    def _desc_for(self, oid, caller):
        """Descriptor handed to a reader (+ holder registration for refs nested inside)."""
        e = self.objects.get(oid)
        if e is None or e.state == FREED:
            err = exc.ObjectLostError(oid.hex())
            b = serialize(err, error=True).to_bytes()
            return ("inline", b, len(b), FLAG_ERROR)
        for c in e.contained:
            ce = self.objects.get(c)
            if ce is not None:
                self.refs.add_holder(c, caller)
        d = e.desc
        if d[0] == "spill" and self.config.get("restore_spilled", True):
            self._restore(e)
            d = e.desc
        g = e.gpu
        if g is not None:
            g["last"] = time.time()
            if caller != self._gpu_owner_key(e):  # the reader maps the owner's HBM until it unmaps
                g["maps"][caller] = g["maps"].get(caller, 0) + 1
        return (d[0], d[1], d[2], e.flags)

    # -------------------------------------------------------------- put
    def rpc_put(self, caller, oid, desc, contained, is_gpu=False, flags=0):
        e = self._obj(oid)
        self.refs.add_holder(oid, caller)
        owner = None
        if is_gpu:
            if caller == DRIVER:
                owner = DRIVER
            elif caller.startswith("w:"):
                owner = bytes.fromhex(caller[2:])
                w = self.workers.get(owner)
                if w is not None:
                    w.gpu_objects.add(oid)
        self._set_ready(e, tuple(desc), contained, owner, flags, gpu_info=is_gpu)
        return True

    # -------------------------------------------------------------- lineage reconstruction
    def _record_lineage(self, ts):
        """Keep the spec of a finished retryable task so its outputs can be recomputed if lost
        (reference ``src/ray/core_worker/object_recovery_manager.cc``). Bounded LRU: an evicted
        entry makes a later loss fail with ObjectReconstructionFailedLineageEvictedError."""
        spec = ts.spec
        ent = self.lineage.get(ts.tid)
        if ent is None:
            self.lineage[ts.tid] = [spec, ts.owner, int(spec.get("max_retries", 0))]
        self.lineage.move_to_end(ts.tid)
        while len(self.lineage) > self.lineage_max:
            self.lineage.popitem(last=False)

    def _lose_object(self, e):
        """A READY object's value is gone (its node died / its spill file vanished)."""
        if e.desc and e.desc[0] == "shm":
            self.store.delete(e.oid)
        tid = e.task
        ent = self.lineage.get(tid) if tid else None
        if ent is None:
            err = (exc.ObjectReconstructionFailedLineageEvictedError(e.oid.hex()) if tid and tid in self.tasks
                   else exc.ObjectLostError(e.oid.hex()))
            self._fail_lost(e, err)
            return
        if ent[2] == 0:
            self._fail_lost(e, exc.ObjectReconstructionFailedMaxAttemptsExceededError(e.oid.hex()))
            return
        self._reconstruct(tid)

    def _fail_lost(self, e, err):
        b = serialize(err, error=True).to_bytes()
        e.desc = ("inline", b, len(b))
        e.flags = FLAG_ERROR

    def _reconstruct(self, tid):
        """Re-execute the producing task (same task id and return ids); readers of its outputs
        wait on them as on any pending object. Lost inputs are reconstructed first."""
        ent = self.lineage.get(tid)
        if ent is None:
            return
        ts_old = self.tasks.get(tid)
        if ts_old is not None and ts_old.state not in (T_FINISHED, T_FAILED, T_CANCELLED):
            return  # already being recomputed
        spec, owner, left = ent
        if left > 0:
            ent[2] = left - 1
        self.num_reconstructions += 1
        for rid in spec["return_ids"]:
            e = self.objects.get(rid)
            if e is not None and e.state == READY:
                if e.desc and e.desc[0] == "shm":
                    self.store.delete(rid)
                for c in e.contained:
                    self._unpin(c)
                e.contained = []
                e.state = PENDING
                e.desc = None
        for a in spec["args"]:
            if a[0] == "r":
                d = self.objects.get(a[1])
                if d is not None and d.state == READY and d.desc and d.desc[0] in ("shm", "spill") and \
                        d.node is not None and not self.nodes.get(d.node, NodeState("x", {})).alive:
                    self._lose_object(d)
        self._event(ts_old or TaskState(tid, spec, owner), "reconstruct")
        re_spec = dict(spec)
        re_spec["max_retries"] = 0
        self._submit(re_spec, owner)

    def rpc_lineage_stats(self, caller):
        return {"entries": len(self.lineage), "reconstructions": self.num_reconstructions}

    # -------------------------------------------------------------- GPU object store (HBM budget)
    def _gpu_owner_key(self, e):
        o = e.gpu_owner
        return None if o is None else (DRIVER if o == DRIVER else "w:" + o.hex())

    def _gpu_account(self, e, info):
        e.gpu = {"nbytes": int(info.get("nbytes", 0)), "gpus": list(info.get("gpus") or ["0"]), "state": "hbm",
                 "last": time.time(), "maps": {}, "counted": True}
        self.gpu_objects[e.oid] = e
        share = e.gpu["nbytes"] // max(1, len(e.gpu["gpus"]))
        for g in e.gpu["gpus"]:
            self.gpu_usage[g] = self.gpu_usage.get(g, 0) + share
        for g in e.gpu["gpus"]:
            self._gpu_enforce_budget(g)

    def _gpu_unaccount(self, e):
        g = e.gpu
        if g is None:
            return
        self.gpu_objects.pop(e.oid, None)
        if g["counted"]:
            share = g["nbytes"] // max(1, len(g["gpus"]))
            for d in g["gpus"]:
                self.gpu_usage[d] = max(0, self.gpu_usage.get(d, 0) - share)
        e.gpu = None

    def _gpu_enforce_budget(self, gpu):
        budget = self.gpu_budget
        if not budget or self.gpu_usage.get(gpu, 0) <= budget:
            return
        over = self.gpu_usage[gpu] - budget
        # least recently used, not mapped by any reader, resident on this GPU
        cands = sorted((e for e in self.gpu_objects.values() if e.gpu["state"] == "hbm" and gpu in e.gpu["gpus"]
                        and e.state == READY and not any(e.gpu["maps"].values())), key=lambda e: e.gpu["last"])
        by_owner: Dict[Any, List[bytes]] = {}
        for e in cands:
            if over <= 0:
                break
            e.gpu["state"] = "spilling"
            by_owner.setdefault(e.gpu_owner, []).append(e.oid)
            over -= e.gpu["nbytes"] // max(1, len(e.gpu["gpus"]))
        for owner, oids in by_owner.items():
            self._gpu_command(owner, "spill", oids)

    def _gpu_command(self, owner, cmd, oids):
        if owner == DRIVER:
            if self.driver_gpu_cmd_cb is not None:
                threading.Thread(target=self.driver_gpu_cmd_cb, args=(cmd, oids), daemon=True).start()
            return
        w = self.workers.get(owner)
        if w is not None and not w.dead:
            self._send(w, (P.GPU_CMD, cmd, oids))

    def rpc_gpu_spilled(self, caller, oids):
        for oid in oids:
            e = self.objects.get(oid)
            if e is None or e.gpu is None or not e.gpu["counted"]:
                continue
            if e.gpu["state"] == "spilling":
                e.gpu["state"] = "host"
            e.gpu["counted"] = False
            share = e.gpu["nbytes"] // max(1, len(e.gpu["gpus"]))
            for d in e.gpu["gpus"]:
                self.gpu_usage[d] = max(0, self.gpu_usage.get(d, 0) - share)
            self.gpu_spilled_bytes += e.gpu["nbytes"]
            self.gpu_num_spilled += 1
        return True

    def _gpu_request_restore(self, e):
        if e.gpu["state"] == "restoring":
            return
        e.gpu["state"] = "restoring"
        e.state = PENDING  # readers wait on the restore like on a producing task
        self._gpu_command(e.gpu_owner, "restore", [e.oid])

    def rpc_gpu_restored(self, caller, oid, desc, info):
        e = self.objects.get(oid)
        if e is None or e.gpu is None or e.gpu["state"] != "restoring":
            return False
        if desc is None:
            self._set_error(e, exc.ObjectLostError(oid.hex()))
            return False
        g = e.gpu
        g["state"] = "hbm"
        g["last"] = time.time()
        if not g["counted"]:
            g["counted"] = True
            share = g["nbytes"] // max(1, len(g["gpus"]))
            for d in g["gpus"]:
                self.gpu_usage[d] = self.gpu_usage.get(d, 0) + share
        self.gpu_num_restored += 1
        e.desc = tuple(desc)
        e.state = READY
        ws, e.waiters = e.waiters, []
        for cb in ws:
            cb(e)
        for d in g["gpus"]:
            self._gpu_enforce_budget(d)
        return True

    def rpc_gpu_unmapped(self, caller, oid):
        e = self.objects.get(oid)
        if e is not None and e.gpu is not None:
            n = e.gpu["maps"].get(caller, 0) - 1
            if n > 0:
                e.gpu["maps"][caller] = n
            else:
                e.gpu["maps"].pop(caller, None)
        return True

    def rpc_gpu_store_stats(self, caller):
        return {"budget_per_gpu": self.gpu_budget, "usage": dict(self.gpu_usage), "objects": len(self.gpu_objects),
                "spilled_bytes": self.gpu_spilled_bytes, "num_spilled": self.gpu_num_spilled,
                "num_restored": self.gpu_num_restored,
                "on_host": sum(1 for e in self.gpu_objects.values() if e.gpu["state"] == "host")}

    def rpc_make_room(self, caller, nbytes):
        """Spill LRU objects until ``nbytes`` could fit (best effort). Returns freed bytes."""
        return self._spill(nbytes)

    def _spill(self, nbytes):
        freed = 0
        cands = self.store.lru_candidates(256)
        for oid, size in cands:
            e = self.objects.get(oid)
            if e is None or e.state != READY or e.desc[0] != "shm":
                continue
            data = self.store.read_bytes(oid)
            if data is None:
                continue
            path = os.path.join(self.spill_dir, oid.hex())
            with open(path, "wb") as f:
                f.write(data)
            e.desc = ("spill", path, size)
            self.store.delete(oid)
            self.spilled_bytes += size
            self.num_spilled += 1
            freed += size
            if freed >= nbytes * 1.2 + (1 << 20):
                break
        return freed

    def _restore(self, e):
        path, size = e.desc[1], e.desc[2]
        try:
            with open(path, "rb") as f:
                data = f.read()
        except OSError:
            self._lose_object(e)  # the spill file is gone: reconstruct from lineage or fail
            return
        ok = self.store.put_bytes(e.oid, data)
        if not ok:
            self._spill(len(data))
            ok = self.store.put_bytes(e.oid, data)
        if ok:
            e.desc = ("shm", None, size)
            self.num_restored += 1
            try:
                os.unlink(path)
            except OSError:
                pass

    # -------------------------------------------------------------- get / wait
    def rpc_get(self, caller, oids, timeout=None, _block=True):
        d = Deferred()
        remaining = {o for o in oids}
        for oid in oids:
            e = self.objects.get(oid)
            if e is not None and e.state == READY and e.gpu is not None and e.gpu["state"] != "hbm":
                self._gpu_request_restore(e)  # spilled to pinned host: back into HBM first
            if e is not None and e.state == PENDING:
                continue
            remaining.discard(oid)
        if not remaining:
            d.resolve([self._desc_for(o, caller) for o in oids])
            return d
        state = {"n": len(remaining)}

        def one(oid):
            if oid in remaining:
                remaining.discard(oid)
                state["n"] -= 1
                if state["n"] == 0 and not d.done:
                    d.resolve([self._desc_for(o, caller) for o in oids])

        self._when_ready(list(remaining), one)
        if timeout is not None and not d.done:
            self._add_timer(timeout, lambda: d.resolve(exc.GetTimeoutError(
                f"Get timed out: some object(s) not ready after {timeout}s."), ok=False))
        if _block:
            self._maybe_block(caller, d)
        return d

    def _maybe_block(self, caller, d):
        """A worker waiting in get/wait inside a normal task lends its CPU back (no deadlock when
        tasks wait on tasks) and re-acquires it once the wait is over."""
        if d.done or not caller.startswith("w:"):
            return
        w = self.workers.get(bytes.fromhex(caller[2:]))
        if w is None or w.task is None:
            return
        self._on_blocked(w, True)
        d.add(lambda _d, w=w: self._on_blocked(w, False))

    def rpc_wait(self, caller, oids, num_returns, timeout=None, fetch_local=True, all_ready=False):
        """``all_ready``: when enough objects are already ready, return EVERY ready one (in input
        order) so the caller can answer its next waits on the same list locally."""
        d = Deferred()
        objs = self.objects
        ready, pending = [], []
        for o in oids:
            e = objs.get(o)
            if e is None or e.state != PENDING:
                ready.append(o)
                if len(ready) >= num_returns and not all_ready:  # the first num_returns ready, in order
                    d.resolve(ready)
                    return d
            else:
                pending.append(e)
        if len(ready) >= num_returns:
            d.resolve(ready)
            return d
        if timeout == 0:
            d.resolve(ready)
            return d
        rs = set(ready)
        order = list(ready)

        def detach():
            # drop this wait's callbacks from objects still pending: repeated waits on a
            # shrinking list (the common polling pattern) must not pile up dead callbacks
            for e in pending:
                if e.state == PENDING:
                    try:
                        e.waiters.remove(cb)
                    except ValueError:
                        pass

        def cb(e):
            if d.done or e.oid in rs:
                return
            rs.add(e.oid)
            order.append(e.oid)
            if len(order) >= num_returns:
                d.resolve(order[:num_returns])
                detach()

        for e in pending:
            e.waiters.append(cb)
        if timeout is not None and not d.done:
            def expire():
                if not d.done:
                    d.resolve(list(order))
                    detach()
            self._add_timer(timeout, expire)
        self._maybe_block(caller, d)
        return d

    def rpc_object_locations(self, caller, oids):
        """{oid: {"node_ids": [...], "object_size": n}} for known objects (reference:
        ``experimental/locations.py``): objects in the node's shm store (or spilled from it) report
        that node; small inline objects live in their owner's memory and report no node."""
        out = {}
        for o in oids:
            e = self.objects.get(o)
            if e is None or e.state == PENDING:
                continue
            kind = e.desc[0] if e.desc else None
            nodes = [self.head_node_id.hex() if isinstance(self.head_node_id, bytes) else self.head_node_id] \
                if kind in ("shm", "spill") else []
            out[o] = {"node_ids": nodes, "object_size": int(e.size or 0)}
        return out

    def rpc_object_ready(self, caller, oid):
        e = self.objects.get(oid)
        return e is None or e.state != PENDING

    def rpc_free(self, caller, oids):
        for oid in oids:
            e = self.objects.get(oid)
            if e is not None:
                self.refs.clear_refs(oid)
                if e.state == READY:
                    self._free(e)

    # ================================================================== functions
    def rpc_register_function(self, caller, fid, blob):
        self.functions.setdefault(fid, blob)
        return True

    # ================================================================== task submission
    def rpc_submit(self, caller, spec):
        self._submit(spec, caller)
        return None

    def _submit(self, spec, owner):
        tid = spec["tid"]
        if spec["kind"] == "actor_creation" and spec.get("actor_name"):
            ns = spec.get("namespace", "")
            if not self.actor_dir.name_available(ns, spec["actor_name"]):
                raise ValueError(f"The name {spec['actor_name']} (namespace={ns}) is already taken.")
        if spec.get("fblob") is not None:
            self.functions.setdefault(spec["fid"], spec.pop("fblob"))
        ts = TaskState(tid, spec, owner)
        self.tasks[tid] = ts
        parent = spec.get("parent")
        if parent is not None and parent in self.tasks:
            self.tasks[parent].children.append(tid)
        for rid in spec["return_ids"]:
            self._obj(rid, task=tid)
            self.refs.add_holder(rid, owner)
        if spec.get("generator") == "streaming":
            pass
        for c in spec.get("contained", ()):
            self._pin(c)
        deps = [a[1] for a in spec["args"] if a[0] == "r"]
        for d in deps:
            self._pin(d)
        self._event(ts, "submit")
        kind = spec["kind"]
        if kind == "actor_creation":
            self._create_actor(spec, owner, ts)
        pending = {d for d in deps if (self.objects.get(d) is not None and self.objects[d].state == PENDING)}
        ts.deps = pending
        if kind == "actor_task":
            a = self.actors.get(spec["actor_id"])
            if a is None or a.state == A_DEAD:
                self._fail_task(ts, exc.ActorDiedError(spec["actor_id"], self._actor_death_msg(a)))
                return
            a.queue.append(ts)
            ts.state = T_QUEUED
            if pending:
                self._when_ready(list(pending), lambda oid, ts=ts, a=a: self._actor_dep_ready(a, ts, oid))
            self._pump_actor(a)
            return
        if pending:
            self._when_ready(list(pending), lambda oid, ts=ts: self._dep_ready(ts, oid))
        else:
            self._enqueue(ts)

    def _dep_ready(self, ts, oid):
        ts.deps.discard(oid)
        if not ts.deps and ts.state == T_WAIT_DEPS and not ts.cancelled:
            self._enqueue(ts)

    def _actor_dep_ready(self, a, ts, oid):
        ts.deps.discard(oid)
        self._pump_actor(a)

    def _demand_of(self, spec):
        res = dict(spec.get("resources") or {})
        strat = spec.get("strategy") or {}
        clauses = list(spec.get("label_selector") or ())
        if strat.get("kind") == "labels":
            clauses += list(strat.get("hard") or ())
        if clauses:
            res[self._selector_resource(clauses)] = 0.001
        if strat.get("kind") == "pg":
            pgid = strat["pg_id"].hex()
            idx = strat.get("bundle_index", -1)
            out = {}
            for k, v in res.items():
                if v <= 0:
                    continue
                out[f"{k}_group_{idx}_{pgid}" if idx is not None and idx >= 0 else f"{k}_group_{pgid}"] = v
            out[f"bundle_group_{idx}_{pgid}" if idx is not None and idx >= 0 else f"bundle_group_{pgid}"] = 0.001
            return out
        return {k: v for k, v in res.items() if v > 0}

    def _enqueue(self, ts):
        spec = ts.spec
        ts.demand = self._demand_of(spec)
        ts.state = T_QUEUED
        self._key += 1
        ts.key = self._key
        self.task_keys[ts.key] = ts
        strat = spec.get("strategy") or {}
        kind = strat.get("kind")
        code = 0
        aff = ""
        soft = False
        if kind == "spread":
            code = 1
        elif kind == "node_affinity":
            code = 2
            aff = strat["node_id"]
            soft = bool(strat.get("soft"))
        preferred = spec.get("caller_node") or self.head_node_id
        if not self.sched.is_feasible(ts.demand) and not (kind == "node_affinity" and soft):
            if kind == "pg" and self.pg_dir.state(strat["pg_id"]) == "PENDING":
                pass  # wait for the placement group to be placed
            elif kind == "node_affinity" and not soft:
                self._fail_task(ts, exc.TaskUnschedulableError(
                    f"node {aff} is not alive or infeasible for {ts.demand}"))
                return
            else:
                log.warning("task %s demands %s which no node can satisfy; it stays pending",
                            spec.get("name"), ts.demand)
        self.sched.enqueue(ts.key, ts.demand, code, preferred, aff, soft)
        self._schedule()

    def _schedule(self):
        if self.shutting_down:
            return
        for key, node_id in self.sched.schedule(0):
            ts = self.task_keys.pop(key, None)
            if ts is None:
                self.sched.release(node_id, {})
                continue
            if ts.cancelled:
                self.sched.release(node_id, ts.demand)
                continue
            ts.node = node_id
            node = self.nodes[node_id]
            ts.gpus = self._assign_gpus(node, ts.demand, ts.spec)
            ts.state = T_WAIT_WORKER
            self._event(ts, "scheduled")
            env_key = self._env_key(ts.spec.get("runtime_env") or {}, ts.gpus)
            if ts.spec["kind"] == "actor_creation":
                a = self.actors.get(ts.spec["actor_id"])
                if a is None or a.state == A_DEAD:
                    self.sched.release(node_id, ts.demand)
                    self._release_gpus(node_id, ts.gpus, ts.demand)
                    continue
                a.node = node_id
                a.demand = ts.demand
                a.gpus = ts.gpus
                # dedicated worker: reuse an idle CPU worker if the env matches, else spawn
                w = self._pop_idle(node, env_key)
                if w is None:
                    node.dispatch_q[env_key].append(ts)
                    self._start_worker(node, env_key, ts.gpus, ts.spec.get("runtime_env") or {})
                else:
                    self._dispatch(w, ts)
                continue
            w = self._pop_idle(node, env_key)
            if w is not None:
                self._dispatch(w, ts)
            else:
                node.dispatch_q[env_key].append(ts)
                need = len(node.dispatch_q[env_key])
                if self.wpool.starting(node.node_id, _pool_key(env_key)) < need:
                    self._start_worker(node, env_key, ts.gpus, ts.spec.get("runtime_env") or {})
        self._try_place_pgs()

    def _assign_gpus(self, node, demand, spec):
        g = 0.0
        for k, v in demand.items():
            if k == "GPU" or (k.startswith("GPU_group_")):
                g = max(g, v)
        if g <= 0:
            return ()
        free = node.gpu_free
        if g >= 1:
            n = int(round(g))
            ids = [i for i, c in enumerate(free) if c >= 0.9999][:n]
            for i in ids:
                free[i] = 0.0
            return tuple(ids)
        cands = sorted([i for i, c in enumerate(free) if c >= g - 1e-9], key=lambda i: free[i])
        if not cands:
            return ()
        i = cands[0]
        free[i] -= g
        return (i,)

    def _release_gpus(self, node_id, gpus, demand):
        node = self.nodes.get(node_id)
        if node is None or not gpus:
            return
        g = 0.0
        for k, v in demand.items():
            if k == "GPU" or k.startswith("GPU_group_"):
                g = max(g, v)
        per = 1.0 if g >= 1 else g
        for i in gpus:
            if i < len(node.gpu_free):
                node.gpu_free[i] = min(1.0, node.gpu_free[i] + per)

    def _env_key(self, runtime_env, gpus):
        env = json.dumps(runtime_env, sort_keys=True, default=str) if runtime_env else ""
        return (env, tuple(gpus))

    def _pop_idle(self, node, env_key):
        key = _pool_key(env_key)
        while True:
            wid = self.wpool.pop_idle(node.node_id, key)
            if wid is None:
                return None
            w = self.workers.get(wid)
            if w is not None and not w.dead:
                return w

    # ================================================================== worker pool
    def _start_worker(self, node, env_key, gpus, runtime_env=None):
        wid = new_id()
        env = dict(os.environ)
        env["RCA_HEAD_SOCK"] = self.sock_path
        env["RCA_WORKER_ID"] = wid.hex()
        env["RCA_NODE_ID"] = node.node_id
        env["RCA_STORE"] = self.store_name
        env["RCA_SESSION_DIR"] = self.session_dir
        env["RCA_JOB_ID"] = self.job_id.hex()
        env["RCA_NAMESPACE"] = self.namespace
        env["RCA_SYS_PATH"] = json.dumps([p for p in sys.path if p])
        pkg_parent = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        pp = env.get("PYTHONPATH", "")
        env["PYTHONPATH"] = pkg_parent + (os.pathsep + pp if pp else "")
        env["RCA_GPU_IDS"] = ",".join(str(g) for g in gpus)
        env.setdefault("PYTHONUNBUFFERED", "1")
        if gpus:
            env["HIP_VISIBLE_DEVICES"] = worker_hip_visible_devices(gpus, os.environ)
            env.pop("CUDA_VISIBLE_DEVICES", None)
        else:
            if self.config.get("hide_gpus_from_cpu_workers", True):
                env["HIP_VISIBLE_DEVICES"] = ""
                env["ROCR_VISIBLE_DEVICES_RCA_HIDDEN"] = "1"
        renv = runtime_env or {}
        for k, v in (renv.get("env_vars") or {}).items():
            env[str(k)] = str(v)
        if renv.get("working_dir"):
            from ..runtime_env import prepare_working_dir

            try:
                env["RCA_WORKING_DIR"] = prepare_working_dir(str(renv["working_dir"]), self.session_dir)
            except Exception:
                env["RCA_WORKING_DIR"] = str(renv["working_dir"])
        if renv.get("pip") or renv.get("worker_process_setup_hook") or renv.get("_rca_setup_hook_blob"):
            env["RCA_RUNTIME_ENV"] = json.dumps({k: renv[k] for k in ("pip", "worker_process_setup_hook",
                                                                      "_rca_setup_hook_blob") if k in renv})
        if renv.get("py_modules"):
            env["RCA_PY_MODULES"] = json.dumps([str(p) for p in renv["py_modules"]])
        out_path = os.path.join(self.logs_dir, f"worker-{wid.hex()}.out")
        try:
            logf = open(out_path, "ab")
        except OSError:
            logf = subprocess.DEVNULL
        cmd = [sys.executable, "-u", "-m", "ray_community_amd._private.worker_main"]
        proc = subprocess.Popen(cmd, env=env, stdout=logf, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                                cwd=os.getcwd(), start_new_session=True)
        if logf is not subprocess.DEVNULL:
            logf.close()
        w = WorkerState(wid, node.node_id, env_key, proc, gpus)
        w.log_path = out_path
        self.workers[wid] = w
        self.wpool.add_starting(node.node_id, _pool_key(env_key), 1)
        return w

    def _worker_available(self, w: WorkerState):
        if w.dead or w.actor is not None or getattr(w, "retiring", False):
            return  # (retiring: the worker hit a function's max_calls and is exiting)
        node = self.nodes.get(w.node_id)
        if node is None or not node.alive:
            self._kill_worker(w)
            return
        q = node.dispatch_q.get(w.env_key)
        while q:
            ts = q.popleft()
            if ts.cancelled or ts.state != T_WAIT_WORKER:
                continue
            self._dispatch(w, ts)
            return
        w.state = "idle"
        w.task = None
        w.idle_since = time.time()
        self.wpool.push_idle(node.node_id, _pool_key(w.env_key), w.wid, w.idle_since)

    def _reap_idle(self):
        now = time.time()
        if getattr(self, "_last_reap", 0) > now - 0.5:
            return
        self._last_reap = now
        with self.lock:
            for w in list(self.workers.values()):
                if w.state == "starting" and w.proc is not None and w.proc.poll() is not None:
                    self.start_failures = getattr(self, "start_failures", 0) + 1
                    reason = (f"worker failed to start (exit code {w.proc.returncode}); "
                              f"see {getattr(w, 'log_path', '')}")
                    if self.start_failures >= 5:
                        self._fail_unstartable(w, reason)
                    self._on_worker_death(w, reason)
        keep = int(self.config.get("max_idle_workers", 16))
        timeout = float(self.config.get("idle_worker_timeout_s", 60))
        with self.lock:
            for node in self.nodes.values():
                for wid in self.wpool.reap(node.node_id, keep, timeout, now):
                    w = self.workers.get(wid)
                    if w is not None:
                        self._kill_worker(w)

    def _fail_unstartable(self, w, reason):
        """Workers for this env keep crashing at startup: fail the work queued for them."""
        node = self.nodes.get(w.node_id)
        if node is None:
            return
        tail = ""
        try:
            with open(getattr(w, "log_path", ""), "rb") as f:
                tail = f.read()[-2000:].decode(errors="replace")
        except OSError:
            pass
        err = exc.RuntimeEnvSetupError(f"{reason}\n{tail}")
        q = node.dispatch_q.get(w.env_key)
        while q:
            ts = q.popleft()
            self._release_task_resources(ts)
            if ts.spec["kind"] == "actor_creation":
                a = self.actors.get(ts.spec["actor_id"])
                if a is not None:
                    a.death_cause = str(err)
                    a.killed = True
                    self._on_actor_worker_death(a, str(err), None)
            self._fail_task(ts, err)
        self.start_failures = 0

    def _kill_worker(self, w: WorkerState):
        if w.dead:
            return
        try:
            if w.conn is not None:
                w.conn.send((P.EXIT,))
        except OSError:
            pass
        try:
            if w.proc is not None:
                w.proc.kill()
        except Exception:
            pass

    # ================================================================== dispatch / completion
    def _dispatch(self, w: WorkerState, ts: TaskState):
        spec = ts.spec
        if spec["kind"] == "lease":
            self._grant_lease(w, ts)
            return
        ts.worker = w.wid
        ts.state = T_RUNNING
        ts.attempt += 1
        ts.times["start"] = time.time()
        w.state = "busy"
        w.task = ts
        args = []
        for a in spec["args"]:
            if a[0] == "r":
                args.append(("d", a[1], self._desc_for(a[1], "w:" + w.wid.hex())))
            else:
                args.append(a)
        msg = dict(spec)
        msg["args"] = args
        msg["gpu_ids"] = ts.gpus
        msg["node_id"] = ts.node
        fid = spec.get("fid")
        if fid is not None and fid not in w.known_functions:
            msg["fblob"] = self.functions.get(fid)
            w.known_functions.add(fid)
        if spec["kind"] == "actor_creation":
            a = self.actors[spec["actor_id"]]
            a.worker = w.wid
            a.pid = w.pid
            w.actor = a
        self._event(ts, "running", worker=w)
        self._send(w, (P.EXECUTE, msg))

    def _on_task_done(self, w: WorkerState, tid, results, info):
        if info.get("retire") and w is not None:
            w.retiring = True
        sp = info.get("spans")
        if sp:
            self.spans.extend(sp)
        ts = self.tasks.get(tid)
        if w is not None and w.task is ts:
            w.task = None
        if ts is None:
            return
        if ts.blocked:
            ts.blocked = False
        spec = ts.spec
        kind = spec["kind"]
        failed = info.get("error", False)
        retry_exc = info.get("retryable", False)
        if failed and retry_exc and ts.retries_left != 0 and not ts.cancelled and kind == "task":
            ts.retries_left -= 1
            self._release_task_resources(ts)
            self._event(ts, "retry")
            if w is not None:
                self._worker_available(w)
            ts.state = T_WAIT_DEPS
            self._enqueue(ts)
            return
        ts.state = T_FAILED if failed else T_FINISHED
        ts.times["end"] = time.time()
        ts.error_type = info.get("error_type")
        if kind == "task" and not failed and spec.get("max_retries", 0) != 0 and spec.get("generator") is None:
            self._record_lineage(ts)
        self._event(ts, "failed" if failed else "finished", worker=w)
        gpu_owner = ("w:" + w.wid.hex()) if w is not None else None
        for rid, res in zip(spec["return_ids"], results):
            e = self.objects.get(rid)
            if e is None:
                if res[0] == "shm":
                    self.store.delete(rid)
                continue
            desc, contained, flags, is_gpu = res[0:3], res[3], res[4], res[5]
            owner = w.wid if (is_gpu and w is not None) else None
            if owner is not None:
                w.gpu_objects.add(rid)
            e.node = ts.node
            if ts.node is not None:
                self.refs.set_node(rid, ts.node)
            self._set_ready(e, tuple(desc), contained, owner, flags, gpu_info=is_gpu)
        if spec.get("generator") == "streaming":
            ts.gen_done = True
            self._flush_gen_waiters(ts)
            self._release_gen_producer(ts, self.GEN_STOP_DROPPED)
        self._finish_task_bookkeeping(ts)
        if kind == "actor_creation":
            a = self.actors.get(spec["actor_id"])
            if a is None:
                return
            if failed:
                a.death_cause = info.get("error_msg", "actor constructor failed")
                self._kill_actor(a, no_restart=True, reason=a.death_cause, init_failed=True)
            else:
                a.state = A_ALIVE
                for d in a.ready_waiters:
                    d.resolve(True)
                a.ready_waiters = []
                self._flush_addr_waiters(a)
                self._pump_actor(a)
            return
        if kind == "actor_task":
            a = self.actors.get(spec["actor_id"])
            if a is not None:
                a.inflight.pop(tid, None)
                if info.get("actor_exit"):
                    self._kill_actor(a, no_restart=True, reason="exit_actor() called", graceful=True)
                else:
                    self._maybe_kill_unreferenced(a)
            return
        self._release_task_resources(ts)
        if w is not None:
            self._worker_available(w)
        self._schedule()

    def _finish_task_bookkeeping(self, ts):
        spec = ts.spec
        for a in spec["args"]:
            if a[0] == "r":
                self._unpin(a[1])
        for c in spec.get("contained", ()):
            self._unpin(c)
        self.finished_tasks.append(ts.tid)
        while len(self.finished_tasks) > 9000:
            old = self.finished_tasks.popleft()
            self.tasks.pop(old, None)

    def _release_task_resources(self, ts):
        if ts.node is not None and ts.demand is not None:
            if not ts.blocked:
                self.sched.release(ts.node, ts.demand)
            else:
                rest = {k: v for k, v in ts.demand.items() if k != "CPU" and not k.startswith("CPU_group")}
                self.sched.release(ts.node, rest)
            self._release_gpus(ts.node, ts.gpus, ts.demand)
            ts.demand = {}
            ts.gpus = ()

    def _fail_task(self, ts, err):
        ts.state = T_FAILED
        ts.times["end"] = time.time()
        ts.error_type = type(err).__name__
        for rid in ts.spec["return_ids"]:
            e = self.objects.get(rid)
            if e is not None and e.state == PENDING:
                self._set_error(e, err)
        if ts.spec.get("generator") == "streaming":
            ts.gen_done = True
            self._flush_gen_waiters(ts)
            self._release_gen_producer(ts, self.GEN_STOP_DROPPED)
        self._event(ts, "failed")
        self._finish_task_bookkeeping(ts)

    def _on_blocked(self, w, flag):
        if w is None or w.task is None:
            return
        ts = w.task
        if ts.spec["kind"] not in ("task", "lease") or ts.node is None:
            return
        cpu = {k: v for k, v in ts.demand.items() if k == "CPU" or k.startswith("CPU_group")}
        if not cpu:
            return
        if flag and not ts.blocked:
            ts.blocked = True
            self.sched.release(ts.node, cpu)
            self._schedule()
        elif not flag and ts.blocked:
            ts.blocked = False
            self.sched.acquire(ts.node, cpu, True)

    def _cluster_event(self, severity, source, message, **fields):
        ev = {"event_id": new_id().hex(), "time": time.time(), "severity": severity, "source_type": source,
              "message": message}
        ev.update(fields)
        self.cluster_events.append(ev)

    def rpc_cluster_events(self, caller):
        return list(self.cluster_events)

    def _on_worker_death(self, w: WorkerState, reason):
        if w.dead:
            return
        w.dead = True
        if not self.shutting_down:
            oom = getattr(w, "oom_killed", None)
            self._cluster_event("ERROR" if oom else "WARNING", "WORKER",
                                f"worker {w.wid.hex()[:8]} (pid {w.pid}) died: "
                                f"{'killed by the memory monitor' if oom else reason}",
                                node_id=w.node_id, pid=w.pid, worker_id=w.wid.hex())
        node = self.nodes.get(w.node_id)
        if w.state == "starting":
            self.wpool.add_starting(w.node_id, _pool_key(w.env_key), -1)
        self.wpool.remove(w.wid)
        self.workers.pop(w.wid, None)
        self._drop_streams_of("w:" + w.wid.hex())
        # GPU objects owned by the worker are lost
        for oid in list(w.gpu_objects):
            e = self.objects.get(oid)
            if e is not None and e.state in (READY, PENDING) and (e.state == READY or e.gpu is not None):
                self._gpu_unaccount(e)
                e.gpu_owner = None
                e.desc = ("inline", serialize(exc.OwnerDiedError(oid.hex()), error=True).to_bytes(), 0)
                e.flags = FLAG_ERROR
                if e.state == PENDING:  # readers were waiting on a restore from the dead owner
                    e.state = READY
                    ws, e.waiters = e.waiters, []
                    for cb in ws:
                        cb(e)
        ts = w.task
        w.task = None
        if getattr(w, "oom_killed", None):
            reason = f"killed by the memory monitor (node memory usage {w.oom_killed[0]:.2f} >= " \
                     f"threshold {w.oom_killed[1]:.2f})"
        self._return_leases_of("w:" + w.wid.hex())  # leases this worker held as a submitter
        self._release_call_pins("w:" + w.wid.hex())
        if w.actor is not None:
            a = w.actor
            self._on_actor_worker_death(a, reason, ts)
        elif ts is not None and ts.spec["kind"] == "lease":
            self._lease_worker_died(w, ts, reason)
        elif ts is not None and ts.state == T_RUNNING:
            self._release_task_resources(ts)
            if ts.cancelled:
                self._fail_task(ts, exc.TaskCancelledError(ts.tid.hex()))
            elif ts.retries_left != 0:
                ts.retries_left -= 1
                self._event(ts, "retry")
                ts.state = T_WAIT_DEPS
                self._enqueue(ts)
            elif getattr(w, "oom_killed", None):
                u, thr = w.oom_killed
                self._fail_task(ts, exc.OutOfMemoryError(
                    f"Task {ts.spec.get('name')} was killed by the memory monitor: node memory usage {u:.2f} "
                    f"exceeded the threshold {thr:.2f} (memory_usage_threshold) and its retries are exhausted. "
                    "Reduce the task's memory, lower its parallelism, or raise max_retries."))
            else:
                self._fail_task(ts, exc.WorkerCrashedError(
                    f"The worker died unexpectedly while executing task {ts.spec.get('name')} ({reason})."))
        self._schedule()
        # keep the pool warm for queued work
        if node is not None and node.alive:
            for key, q in node.dispatch_q.items():
                if q and self.wpool.starting(node.node_id, _pool_key(key)) < len(q):
                    self._start_worker(node, key, q[0].gpus, q[0].spec.get("runtime_env") or {})

    # ================================================================== streaming generators
    def _on_gen_item(self, tid, index, res):
        ts = self.tasks.get(tid)
        oid = res[6]
        e = self._obj(oid, task=tid)
        if ts is not None:
            self.refs.add_holder(oid, ts.owner)
            while len(ts.gen_items) <= index:
                ts.gen_items.append(None)
            ts.gen_items[index] = oid
        desc, contained, flags = res[0:3], res[3], res[4]
        self._set_ready(e, tuple(desc), contained, None, flags)
        if ts is not None:
            self._flush_gen_waiters(ts)

    def _gen_consumed(self, ts, index):
        """The consumer was handed item ``index``: wake a producer paused on backpressure."""
        if index + 1 > ts.gen_consumed:
            ts.gen_consumed = index + 1
            if ts.gen_bp_waiters:
                keep = []
                for need, d in ts.gen_bp_waiters:
                    if ts.gen_consumed >= need:
                        d.resolve(ts.gen_consumed)
                    else:
                        keep.append((need, d))
                ts.gen_bp_waiters = keep

    # what a paused producer is told when it must stop instead of producing more
    GEN_STOP_DROPPED, GEN_STOP_CANCELLED = -1, -2

    def rpc_gen_wait_consumed(self, caller, tid, need):
        """``_generator_backpressure_num_objects``: the producer blocks until the consumer has
        taken ``need`` items (reference: ``src/ray/core_worker/generator_waiter.h``). Answers a
        negative code instead when the stream is gone: the task was cancelled, or its consumer
        dropped the generator / died (reference: ``HandleDelObjectRefStream`` releasing the waiter)."""
        ts = self.tasks.get(tid)
        d = Deferred()
        if ts is None:
            d.resolve(self.GEN_STOP_DROPPED)
        elif ts.cancelled:
            d.resolve(self.GEN_STOP_CANCELLED)
        elif ts.gen_dropped:
            d.resolve(self.GEN_STOP_DROPPED)
        elif ts.gen_consumed >= need:
            d.resolve(ts.gen_consumed)
        else:
            ts.gen_bp_waiters.append((need, d))
        return d

    def _release_gen_producer(self, ts, code):
        """Wake a producer paused on backpressure with a stop ``code``: nothing will ever consume
        what it is waiting to produce, and a blocked producer would hold its worker forever."""
        waiters, ts.gen_bp_waiters = ts.gen_bp_waiters, []
        for _need, d in waiters:
            d.resolve(code)

    def rpc_gen_drop(self, caller, tid):
        """The consumer's ObjectRefGenerator was garbage-collected before the stream ended."""
        ts = self.tasks.get(tid)
        if ts is not None and not ts.gen_done:
            ts.gen_dropped = True
            self._release_gen_producer(ts, self.GEN_STOP_DROPPED)
        return True

    def _drop_streams_of(self, owner_key):
        """An owner process is gone: release the paused producers of the streams it consumed."""
        for ts in list(self.tasks.values()):
            if ts.gen_bp_waiters and ts.owner == owner_key and not ts.gen_done:
                ts.gen_dropped = True
                self._release_gen_producer(ts, self.GEN_STOP_DROPPED)

    def _flush_gen_waiters(self, ts):
        for idx in list(ts.gen_waiters):
            if idx < len(ts.gen_items) and ts.gen_items[idx] is not None:
                for d in ts.gen_waiters.pop(idx):
                    d.resolve(ts.gen_items[idx])
                self._gen_consumed(ts, idx)
            elif ts.gen_done:
                for d in ts.gen_waiters.pop(idx):
                    d.resolve(None)

    def rpc_gen_next(self, caller, tid, index, timeout=None):
        ts = self.tasks.get(tid)
        d = Deferred()
        if ts is None:
            d.resolve(None)
            return d
        if index < len(ts.gen_items) and ts.gen_items[index] is not None:
            oid = ts.gen_items[index]
            if oid in self.objects:
                self.refs.add_holder(oid, caller)
            d.resolve(oid)
            self._gen_consumed(ts, index)
            return d
        if ts.gen_done:
            # error of the generator task is surfaced through its return object
            d.resolve(None)
            return d
        ts.gen_waiters.setdefault(index, []).append(d)
        if timeout is not None:
            self._add_timer(timeout, lambda: d.resolve(exc.GetTimeoutError("generator next timed out"), ok=False))
        return d

    # ================================================================== actors
    def _create_actor(self, spec, owner, ts):
        aid = spec["actor_id"]
        if aid in self.actor_dir:  # a re-submitted creation spec: keep the registered actor
            self.actor_dir.remove(aid)
        a = ActorState(aid, spec, owner, self.actor_dir)  # raises if the name is taken (live holder)
        a.creation_task = ts
        self.actors[aid] = a

    def rpc_actor_name_available(self, caller, name, namespace):
        return self.actor_dir.name_available(namespace, name)

    def _pump_actor(self, a: ActorState):
        if a.state != A_ALIVE:
            return
        w = self.workers.get(a.worker)
        if w is None or w.dead:
            return
        # per-caller order: a call with unresolved dependencies holds back only the LATER calls
        # of the same caller; other callers' calls proceed
        blocked = set()
        rest = collections.deque()
        q = a.queue
        while q:
            ts = q.popleft()
            if ts.cancelled:
                continue
            if ts.deps or ts.owner in blocked:
                blocked.add(ts.owner)
                rest.append(ts)
                continue
            a.inflight[ts.tid] = ts
            ts.node = a.node
            self._dispatch_actor_task(w, ts)
        a.queue = rest

    def _dispatch_actor_task(self, w, ts):
        spec = ts.spec
        ts.worker = w.wid
        ts.state = T_RUNNING
        ts.times["start"] = time.time()
        args = []
        for x in spec["args"]:
            if x[0] == "r":
                args.append(("d", x[1], self._desc_for(x[1], "w:" + w.wid.hex())))
            else:
                args.append(x)
        msg = dict(spec)
        msg["args"] = args
        self._event(ts, "running", worker=w)
        self._send(w, (P.EXECUTE, msg))

    def _on_actor_worker_death(self, a: ActorState, reason, running_ts):
        if a.state == A_DEAD:
            return
        inflight = list(a.inflight.values())
        a.inflight.clear()
        if a.node is not None and not getattr(a, "_res_released", False):
            self.sched.release(a.node, a.demand)
            self._release_gpus(a.node, a.gpus, a.demand)
        a.worker = None
        can_restart = (not a.killed) and (a.restarts_left != 0)
        if running_ts is not None and running_ts.spec["kind"] == "actor_creation" and running_ts.state == T_RUNNING:
            can_restart = can_restart and True
        if can_restart:
            if a.restarts_left > 0:
                a.restarts_left -= 1
            a.num_restarts += 1
            a.state = A_RESTARTING
            self._event_actor(a, "restarting")
            # in-flight calls: retry if allowed, else fail
            retry = []
            for ts in inflight:
                mtr = ts.spec.get("max_task_retries", 0)
                if mtr != 0:
                    ts.spec["max_task_retries"] = mtr - 1 if mtr > 0 else mtr
                    ts.state = T_QUEUED
                    retry.append(ts)
                else:
                    self._fail_task(ts, exc.ActorDiedError(a.aid, f"The actor died: {reason}"))
            for ts in reversed(retry):
                a.queue.appendleft(ts)
            cts = a.creation_task
            cts.state = T_WAIT_DEPS
            cts.retries_left = 0
            # the creation task's args are still pinned (never finished bookkeeping twice)
            self._enqueue(cts)
        else:
            a.state = A_DEAD
            a.death_cause = a.death_cause or reason
            self._event_actor(a, "dead")
            err = exc.ActorDiedError(a.aid, self._actor_death_msg(a))
            for ts in inflight:
                self._fail_task(ts, err)
            while a.queue:
                self._fail_task(a.queue.popleft(), err)
            cts = a.creation_task
            if cts is not None and cts.state in (T_RUNNING, T_WAIT_WORKER, T_QUEUED, T_WAIT_DEPS):
                self._fail_task(cts, exc.ActorDiedError(a.aid, self._actor_death_msg(a), actor_init_failed=True))
            for d in a.ready_waiters:
                d.resolve(exc.ActorDiedError(a.aid, self._actor_death_msg(a)), ok=False)
            a.ready_waiters = []
            self._flush_addr_waiters(a)

    def _actor_death_msg(self, a):
        if a is None:
            return "The actor is dead (unknown actor)."
        return f"The actor {a.spec.get('class_name', '')} ({a.aid.hex()}) died: {a.death_cause or 'unknown cause'}"

    def _kill_actor(self, a: ActorState, no_restart=True, reason="ray.kill() called", init_failed=False,
                    graceful=False):
        if a.state == A_DEAD:
            return
        if no_restart:
            a.killed = True
            a.restarts_left = 0
        a.death_cause = reason
        w = self.workers.get(a.worker) if a.worker else None
        if w is not None and not w.dead:
            if graceful:
                self._send(w, (P.EXIT,))
            else:
                self._kill_worker(w)
            # death is finalised when the connection drops
            if no_restart:
                # pending (not yet dispatched) calls fail right away
                err = exc.ActorDiedError(a.aid, self._actor_death_msg(a), actor_init_failed=init_failed)
                while a.queue:
                    self._fail_task(a.queue.popleft(), err)
        else:
            cts = a.creation_task
            if cts is not None and cts.key is not None and cts.key in self.task_keys:
                self.sched.cancel(cts.key)
                self.task_keys.pop(cts.key, None)
            if cts is not None:
                for node in self.nodes.values():
                    for q in node.dispatch_q.values():
                        if cts in q:
                            q.remove(cts)
                            if cts.node:
                                self.sched.release(cts.node, cts.demand)
                                self._release_gpus(cts.node, cts.gpus, cts.demand)
                            a._res_released = True
            self._on_actor_worker_death(a, reason, None)

    def rpc_kill_actor(self, caller, aid, no_restart=True):
        a = self.actors.get(aid)
        if a is None:
            raise ValueError("unknown actor")
        self._kill_actor(a, no_restart=no_restart)
        return True

    def rpc_get_actor(self, caller, name, namespace):
        aid = self.actor_dir.by_name(namespace, name)
        a = self.actors.get(aid) if aid else None
        if a is None or a.state == A_DEAD:
            return None
        self.actor_dir.add_handle(a.aid, caller)
        return {"actor_id": a.aid, "meta": a.spec.get("class_meta")}

    def rpc_actor_handle(self, caller, aid):
        """Handle metadata of an actor by id (``get_runtime_context().current_actor``)."""
        a = self.actors.get(aid)
        if a is None or a.state == A_DEAD:
            return None
        self.actor_dir.add_handle(a.aid, caller)
        return {"actor_id": a.aid, "meta": a.spec.get("class_meta")}

    def rpc_actor_ready(self, caller, aid):
        a = self.actors.get(aid)
        d = Deferred()
        if a is None:
            d.resolve(exc.ActorDiedError(aid, "unknown actor"), ok=False)
        elif a.state == A_ALIVE:
            d.resolve(True)
        elif a.state == A_DEAD:
            d.resolve(exc.ActorDiedError(aid, self._actor_death_msg(a)), ok=False)
        else:
            a.ready_waiters.append(d)
        return d

    # -------------------------------------------------------------- direct actor calls
    def rpc_actor_address(self, caller, aid, min_incarnation=0):
        """Direct-call endpoint of an actor: resolves to (socket path, incarnation) once the actor
        is ALIVE in an incarnation >= ``min_incarnation`` (a caller whose stream broke asks for
        the next one), or fails with ActorDiedError once it is dead for good."""
        d = Deferred()
        a = self.actors.get(aid)
        if a is None:
            d.resolve(exc.ActorDiedError(aid, "The actor is dead (unknown actor)."), ok=False)
            return d
        a.addr_waiters.append((d, min_incarnation))
        self._flush_addr_waiters(a)
        return d

    def _flush_addr_waiters(self, a):
        if not a.addr_waiters:
            return
        keep = []
        for d, inc in a.addr_waiters:
            if d.done:
                continue
            if a.state == A_DEAD:
                d.resolve(exc.ActorDiedError(a.aid, self._actor_death_msg(a)), ok=False)
                continue
            w = self.workers.get(a.worker) if a.worker else None
            if a.state == A_ALIVE and a.num_restarts >= inc and w is not None and not w.dead and w.direct_addr:
                d.resolve((w.direct_addr, a.num_restarts))
            else:
                keep.append((d, inc))
        a.addr_waiters = keep

    def rpc_object_descs(self, caller, oids):
        """Descriptors of ``oids`` once all are ready (like ``get`` but without lending the
        caller's CPU: a direct-call submitter resolving the arguments of a queued call)."""
        return self.rpc_get(caller, oids, None, _block=False)

    def rpc_declare_object(self, caller, oid):
        """A caller-owned (direct-call) result whose ref escaped before its value arrived."""
        self._obj(oid)
        self.refs.add_holder(oid, caller)
        return True

    def rpc_pin_objects(self, caller, oids, n):
        """Pin (n > 0) / unpin (n < 0) objects for the duration of a direct actor call that carries
        them nested in its arguments: the head-routed path pins a spec's ``contained`` refs in
        ``_submit``, but a direct call never passes the head, and the owner may drop its last ref
        before the callee deserializes the argument."""
        held = self.call_pins.setdefault(caller, {})
        for o in oids:
            if n > 0:
                if self._pin(o, n):
                    held[o] = held.get(o, 0) + n
            else:
                k = min(-n, held.get(o, 0))
                if k <= 0:
                    continue
                self._unpin(o, k)
                if held[o] == k:
                    del held[o]
                else:
                    held[o] -= k
        if not held:
            self.call_pins.pop(caller, None)
        return True

    def _release_call_pins(self, key):
        """The caller died: drop the pins its in-flight direct actor calls held."""
        for o, k in (self.call_pins.pop(key, None) or {}).items():
            self._unpin(o, k)

    def rpc_put_owned(self, caller, items, owner_key, lineage=None):
        """A worker registers direct-call results the head must manage (shm, GPU, nested refs) on
        behalf of the calling process ``owner_key`` before replying to it. ``lineage``: the spec
        of a retryable leased task, kept so lost outputs can be recomputed like head-run ones."""
        gpu_owner = bytes.fromhex(caller[2:]) if caller.startswith("w:") else None
        w = self.workers.get(gpu_owner) if gpu_owner else None
        tid = None
        if lineage is not None:
            tid = lineage["tid"]
            self.lineage[tid] = [lineage, owner_key, int(lineage.get("max_retries", 0))]
            self.lineage.move_to_end(tid)
            while len(self.lineage) > self.lineage_max:
                self.lineage.popitem(last=False)
        for oid, desc, contained, is_gpu, flags in items:
            e = self._obj(oid)
            self.refs.add_holder(oid, owner_key)
            if tid is not None:
                e.task = tid
            if w is not None:
                e.node = w.node_id
                self.refs.set_node(oid, w.node_id)
            owner = None
            if is_gpu and w is not None:
                owner = gpu_owner
                w.gpu_objects.add(oid)
            self._set_ready(e, tuple(desc), contained, owner, flags, gpu_info=is_gpu)
        return True

    def rpc_actor_exit(self, caller):
        """``exit_actor()`` / ``__ray_terminate__`` inside a directly called actor."""
        w = self.workers.get(bytes.fromhex(caller[2:])) if caller.startswith("w:") else None
        if w is not None and w.actor is not None:
            self._kill_actor(w.actor, no_restart=True, reason="exit_actor() called", graceful=True)
        return True

    # -------------------------------------------------------------- worker leases (direct tasks)
    def rpc_lease(self, caller, resources, caller_node=None):
        """Lease a worker for normal tasks of one resource shape (reference:
        ``NodeManager::HandleRequestWorkerLease`` + ``NormalTaskSubmitter``). The lease goes
        through the ordinary scheduler like a task; once a worker is assigned the caller gets
        ``(lease_id, worker_id, direct socket, node_id)`` and pushes its tasks to the worker
        itself until it returns the lease. The lease holds the shape's resources meanwhile."""
        lid = new_id()
        spec = {"tid": lid, "kind": "lease", "name": "lease", "resources": dict(resources or {}), "args": (),
                "return_ids": (), "caller_node": caller_node, "max_retries": -1}
        ts = TaskState(lid, spec, caller)
        d = Deferred()
        ts.reply = d
        self.leases[lid] = ts
        self.leases_by_owner.setdefault(caller, set()).add(lid)
        self._enqueue(ts)
        return d

    def _grant_lease(self, w, ts):
        ts.worker = w.wid
        ts.state = T_RUNNING
        ts.times["start"] = time.time()  # memory-monitor victim order: newest first
        w.state = "busy"
        w.task = ts
        d = ts.reply
        if d is not None and not d.done:
            d.resolve((ts.tid, w.wid, w.direct_addr, ts.node))

    def _end_lease(self, ts, make_available=True):
        self.leases.pop(ts.tid, None)
        s = self.leases_by_owner.get(ts.owner)
        if s is not None:
            s.discard(ts.tid)
            if not s:
                self.leases_by_owner.pop(ts.owner, None)
        d = ts.reply
        if d is not None and not d.done:
            d.resolve(None)  # cancelled before a worker was assigned
        state = ts.state
        if state in (T_QUEUED, T_WAIT_DEPS):
            ts.cancelled = True
            if ts.key is not None and self.sched.cancel(ts.key):
                self.task_keys.pop(ts.key, None)
        elif state == T_WAIT_WORKER:
            ts.cancelled = True
            self._release_task_resources(ts)
        elif state == T_RUNNING:
            self._release_task_resources(ts)
            w = self.workers.get(ts.worker)
            if w is not None and w.task is ts:
                w.task = None
                if make_available:
                    self._worker_available(w)
        ts.state = T_FINISHED

    def rpc_return_lease(self, caller, lid):
        ts = self.leases.get(lid)
        if ts is not None:
            self._end_lease(ts)
            self._schedule()
        return True

    def rpc_lease_fate(self, caller, lid):
        """Why a leased worker went away (the caller saw its stream break): the error its
        in-flight task fails with. Resolved once the head has processed the worker's death."""
        d = Deferred()
        fate = self.lease_fates.get(lid)
        if fate is not None:
            d.resolve(fate)
        else:
            self.lease_fate_waiters.setdefault(lid, []).append(d)
            self._add_timer(10.0, lambda: None if d.done else d.resolve(
                exc.WorkerCrashedError("The worker executing this task died unexpectedly.")))
        return d

    def _lease_worker_died(self, w, ts, reason):
        if getattr(w, "oom_killed", None):
            u, thr = w.oom_killed
            err = exc.OutOfMemoryError(
                f"A task was killed by the memory monitor: node memory usage {u:.2f} exceeded the threshold "
                f"{thr:.2f} (memory_usage_threshold) and its retries are exhausted. Reduce the task's memory, "
                "lower its parallelism, or raise max_retries.")
        else:
            err = exc.WorkerCrashedError(f"The worker died unexpectedly while executing a task ({reason}).")
        self.lease_fates[ts.tid] = err
        while len(self.lease_fates) > 10000:
            self.lease_fates.pop(next(iter(self.lease_fates)))
        for d in self.lease_fate_waiters.pop(ts.tid, ()):
            d.resolve(err)
        self._end_lease(ts, make_available=False)

    def _return_leases_of(self, owner):
        """The lease owner is gone (disconnected or dead). A granted lease's worker may still be
        running a task the owner pushed to it directly -- the head cannot tell -- so, as the
        reference does for leased workers of a dead owner, the worker is killed: returning it to
        the idle pool would over-commit its resources and queue new tasks behind the orphan."""
        for lid in list(self.leases_by_owner.get(owner, ())):
            ts = self.leases.get(lid)
            if ts is None:
                continue
            w = self.workers.get(ts.worker) if ts.state == T_RUNNING else None
            if w is not None and not w.dead and w.task is ts:
                self._end_lease(ts, make_available=False)
                self._kill_worker(w)
            else:
                self._end_lease(ts)

    def rpc_get_function(self, caller, fid):
        """Function blob for a worker that received a task directly (not through the head)."""
        return self.functions.get(fid)

    def rpc_direct_task_records(self, caller, records):
        """(tid, name, None, start, end, failed, error type, worker id, node) of leased tasks,
        reported by their caller."""
        for tid, name, aid, start, end, failed, etype, wid, node in records:
            w = self.workers.get(wid)
            self.direct_tasks.append((tid, name, aid, start, end, failed, etype, wid, node))
            pid = w.pid if w is not None else None
            self.events.append((start, tid, "running", name, pid, node))
            self.events.append((end, tid, "failed" if failed else "finished", name, pid, node))
        return True

    def _on_direct_events(self, w, records):
        pid = w.pid if w is not None else None
        node = w.node_id if w is not None else None
        wid = w.wid if w is not None else None
        for tid, name, aid, start, end, failed, etype in records:
            self.direct_tasks.append((tid, name, aid, start, end, failed, etype, wid, node))
            self.events.append((start, tid, "running", name, pid, node))
            self.events.append((end, tid, "failed" if failed else "finished", name, pid, node))

    def rpc_actor_info(self, caller, aid):
        a = self.actors.get(aid)
        if a is None:
            return None
        return {"state": a.state, "num_restarts": a.num_restarts, "node_id": a.node, "pid": a.pid,
                "name": a.name, "death_cause": a.death_cause}

    # ================================================================== cancel
    def rpc_cancel(self, caller, oid, force=False, recursive=True):
        e = self.objects.get(oid)
        tid = e.task if e is not None else None
        ts = self.tasks.get(tid) if tid else None
        if ts is None:
            return False
        self._cancel_task(ts, force, recursive)
        return True

    def _cancel_task(self, ts, force, recursive):
        if ts.state in (T_FINISHED, T_FAILED, T_CANCELLED):
            return
        ts.cancelled = True
        if ts.gen_bp_waiters:
            self._release_gen_producer(ts, self.GEN_STOP_CANCELLED)
        if recursive:
            for c in ts.children:
                cts = self.tasks.get(c)
                if cts is not None:
                    self._cancel_task(cts, force, recursive)
        kind = ts.spec["kind"]
        if ts.state in (T_WAIT_DEPS, T_QUEUED, T_WAIT_WORKER):
            if ts.key is not None and self.sched.cancel(ts.key):
                self.task_keys.pop(ts.key, None)
            if ts.state == T_WAIT_WORKER and ts.node:
                self.sched.release(ts.node, ts.demand)
                self._release_gpus(ts.node, ts.gpus, ts.demand)
            if kind == "actor_task":
                a = self.actors.get(ts.spec["actor_id"])
                if a is not None and ts in a.queue:
                    a.queue.remove(ts)
            self._fail_task(ts, exc.TaskCancelledError(ts.tid.hex()))
            ts.state = T_CANCELLED
            self._schedule()
            return
        if ts.state == T_RUNNING:
            w = self.workers.get(ts.worker)
            if kind == "actor_task":
                if w is not None:
                    self._send(w, (P.CANCEL, ts.tid, False))
                return
            if w is not None:
                if force:
                    self._kill_worker(w)
                else:
                    self._send(w, (P.CANCEL, ts.tid, False))

    # ================================================================== placement groups
    def rpc_create_pg(self, caller, pg_id, bundles, strategy, name="", lifetime=None):
        infeasible = any(not self.sched.is_feasible({k: v for k, v in b.items() if v > 0}) for b in bundles)
        self.pg_dir.add(pg_id, name or "", strategy, list(bundles), lifetime, time.time(), infeasible)
        self._try_place_pgs()
        return True

    def _try_place_pgs(self):
        pending = self.pg_dir.pending()
        if not pending:
            return
        placed_any = False
        for pg_id in pending:
            if self.pg_dir.state(pg_id) != "PENDING":
                continue
            bundles = [{k: float(v) for k, v in b.items() if v > 0} for b in self.pg_dir.bundles(pg_id)]
            nodes = self.sched.create_pg(pg_id.hex(), bundles, self.pg_dir.strategy(pg_id))
            if nodes is None:
                continue
            self.pg_dir.set_nodes(pg_id, list(nodes))
            self.pg_dir.set_state(pg_id, "CREATED")  # leaves the pending queue
            # per-bundle GPU bookkeeping happens at task grant time (node.gpu_free)
            for d in self.pg_waiters.pop(pg_id, ()):
                d.resolve(True)
            placed_any = True
        if placed_any:
            self._schedule()

    def rpc_pg_ready(self, caller, pg_id, timeout=None):
        st = self.pg_dir.state(pg_id)
        d = Deferred()
        if st in ("", "REMOVED"):
            d.resolve(ValueError("placement group removed"), ok=False)
        elif st == "CREATED":
            d.resolve(True)
        else:
            self.pg_waiters.setdefault(pg_id, []).append(d)
            if timeout is not None:
                self._add_timer(timeout, lambda: d.resolve(False))
        return d

    def rpc_remove_pg(self, caller, pg_id):
        st = self.pg_dir.state(pg_id)
        if not st:
            return False
        # kill actors placed in the group (the directory's placement-group index)
        for aid in self.actor_dir.in_pg(pg_id):
            a = self.actors.get(aid)
            if a is not None and a.state != A_DEAD:
                self._kill_actor(a, no_restart=True, reason="placement group removed")
        if st == "CREATED":
            self.sched.remove_pg(pg_id.hex())
        self.pg_dir.set_state(pg_id, "REMOVED")  # also leaves the pending queue
        for d in self.pg_waiters.pop(pg_id, ()):
            d.resolve(False)
        self._schedule()
        return True

    def rpc_pg_table(self, caller, pg_id=None):
        if pg_id is not None:
            return self.pg_dir.info(pg_id)
        return self.pg_dir.table()

    def rpc_get_named_pg(self, caller, name):
        pg_id = self.pg_dir.by_name(name)
        if pg_id is None:
            return None
        return {"pg_id": pg_id, "bundles": self.pg_dir.bundles(pg_id), "strategy": self.pg_dir.strategy(pg_id)}

    # ================================================================== cluster info
    def rpc_cluster_resources(self, caller):
        tot = collections.Counter()
        for nid, res in self.sched.totals().items():
            for k, v in res.items():
                if "_group_" in k or k.startswith("__labelsel:"):
                    continue
                tot[k] += v
        return dict(tot)

    def rpc_available_resources(self, caller):
        tot = collections.Counter()
        for nid, res in self.sched.available().items():
            for k, v in res.items():
                if "_group_" in k or k.startswith("__labelsel:"):
                    continue
                if v > 0:
                    tot[k] += v
        return dict(tot)

    # ================================================================== autoscaler load
    def rpc_resource_demands(self, caller):
        """Unmet demand for the autoscaler: resource shapes of queued (not yet scheduled) tasks and
        actors, and the bundles of pending placement groups (``[{res: amount}, ...]`` per group)."""
        tasks = []
        for ts in self.task_keys.values():
            if ts.cancelled or ts.state in (T_CANCELLED,):
                continue
            d = {k: v for k, v in (ts.demand or {}).items() if v > 0 and "_group_" not in k and not k.startswith("node:")}
            if d:
                tasks.append(d)
        pgs = []
        for pg_id in self.pg_dir.pending():
            if self.pg_dir.state(pg_id) == "PENDING":
                pgs.append({"strategy": self.pg_dir.strategy(pg_id),
                            "bundles": [{k: float(v) for k, v in b.items() if v > 0} for b in self.pg_dir.bundles(pg_id)]})
        return {"tasks": tasks, "placement_groups": pgs}

    def rpc_node_load(self, caller):
        """Per alive node: totals, availability and whether any worker is executing work."""
        totals, avail = self.sched.totals(), self.sched.available()
        busy = collections.Counter()
        for w in self.workers.values():
            if not w.dead and (w.task is not None or w.actor is not None):
                busy[w.node_id] += 1
        out = []
        for nid, n in self.nodes.items():
            if not n.alive:
                continue
            clean = lambda r: {k: v for k, v in r.items() if "_group_" not in k and not k.startswith("node:")}  # noqa
            out.append({"node_id": nid, "is_head": n.is_head, "labels": dict(n.labels or {}),
                        "total": clean(totals.get(nid, n.resources)), "available": clean(avail.get(nid, {})),
                        "busy_workers": busy[nid]})
        return out

    def rpc_nodes(self, caller):
        totals = self.sched.totals()
        out = []
        for nid, n in self.nodes.items():
            out.append({"NodeID": nid, "Alive": n.alive, "NodeManagerAddress": "127.0.0.1",
                        "NodeManagerHostname": socket.gethostname(),
                        "Resources": {k: v for k, v in totals.get(nid, n.resources).items() if "_group_" not in k},
                        "Labels": n.labels, "alive": n.alive, "IsHead": n.is_head,
                        "ObjectStoreSocketName": self.store_name})
        return out

    # ================================================================== KV
    # byte keys/values in namespaces, in C++ (_native/kv_table.cpp: ordered per namespace, so
    # prefix listing / deletion touch only the matching range); str keys are stored as UTF-8
    def rpc_kv_put(self, caller, key, value, overwrite=True, namespace=None):
        return self.kv.put(key, value, overwrite, namespace)

    def rpc_kv_get(self, caller, key, namespace=None):
        return self.kv.get(key, namespace)

    def rpc_kv_del(self, caller, key, namespace=None, del_by_prefix=False):
        return self.kv.delete(key, namespace, del_by_prefix)

    def rpc_kv_keys(self, caller, prefix, namespace=None):
        return self.kv.keys(prefix, namespace)

    def rpc_kv_exists(self, caller, key, namespace=None):
        return self.kv.exists(key, namespace)

    # ================================================================== state / observability
    def _event(self, ts, what, worker=None):
        if ts.spec["kind"] == "lease":
            return
        self.events.append((time.time(), ts.tid, what, ts.spec.get("name"), worker.pid if worker else None,
                            ts.node))

    def _event_actor(self, a, what):
        self.events.append((time.time(), a.aid, "actor_" + what, a.spec.get("class_name"), a.pid, a.node))

    def rpc_list_tasks(self, caller, limit=10000):
        out = []
        for ts in list(self.tasks.values())[-limit:]:
            out.append({"task_id": ts.tid.hex(), "name": ts.spec.get("name"), "state": TASK_STATE_NAMES[ts.state],
                        "type": {"task": "NORMAL_TASK", "actor_task": "ACTOR_TASK",
                                 "actor_creation": "ACTOR_CREATION_TASK"}[ts.spec["kind"]],
                        "node_id": ts.node, "worker_id": ts.worker.hex() if ts.worker else None,
                        "actor_id": ts.spec.get("actor_id").hex() if ts.spec.get("actor_id") else None,
                        "required_resources": ts.spec.get("resources"), "error_type": ts.error_type,
                        "attempt_number": max(0, ts.attempt - 1),
                        "start_time_ms": int(ts.times.get("start", 0) * 1000),
                        "end_time_ms": int(ts.times.get("end", 0) * 1000),
                        "func_or_class_name": ts.spec.get("name")})
        for tid, name, aid, start, end, failed, etype, wid, node in list(self.direct_tasks)[-limit:]:
            out.append({"task_id": tid.hex(), "name": name, "state": "FAILED" if failed else "FINISHED",
                        "type": "ACTOR_TASK" if aid else "NORMAL_TASK", "node_id": node,
                        "worker_id": wid.hex() if wid else None,
                        "actor_id": aid.hex() if aid else None, "required_resources": {}, "error_type": etype,
                        "attempt_number": 0, "start_time_ms": int(start * 1000), "end_time_ms": int(end * 1000),
                        "func_or_class_name": name})
        return out[-limit:]

    def rpc_list_actors(self, caller):
        out = []
        for a in self.actors.values():
            out.append({"actor_id": a.aid.hex(), "class_name": a.spec.get("class_name"), "state": a.state,
                        "name": a.name or "", "namespace": a.namespace, "pid": a.pid, "node_id": a.node,
                        "num_restarts": a.num_restarts, "death_cause": a.death_cause,
                        "is_detached": a.detached, "required_resources": a.spec.get("resources"),
                        "annotations": dict(getattr(a, "annotations", None) or {})})
        return out

    def rpc_actor_annotate(self, caller, aid, key, message):
        """``ray.show_in_dashboard`` from inside an actor: a message kept on its state record."""
        a = self.actors.get(aid)
        if a is not None:
            if getattr(a, "annotations", None) is None:
                a.annotations = {}
            a.annotations[key] = message
        return True

    def rpc_list_objects(self, caller):
        out = []
        for e in self.objects.values():
            out.append({"object_id": e.oid.hex(), "object_size": e.size,
                        "task_status": "FINISHED" if e.state == READY else "PENDING",
                        "reference_type": "LOCAL_REFERENCE" if self.refs.num_holders(e.oid) else "PINNED_IN_MEMORY",
                        "num_holders": self.refs.num_holders(e.oid), "pins": self.refs.pins(e.oid),
                        "storage": e.desc[0] if e.desc else None, "gpu": e.gpu_owner is not None})
        return out

    def rpc_list_workers(self, caller):
        return [{"worker_id": w.wid.hex(), "pid": w.pid, "node_id": w.node_id, "state": w.state,
                 "is_actor": w.actor is not None, "gpu_ids": list(w.gpus), "worker_type": "WORKER",
                 "is_alive": not w.dead, "runtime_env": json.loads(w.env_key[0]) if w.env_key[0] else {},
                 "log_file": os.path.basename(getattr(w, "log_path", "") or "")}
                for w in self.workers.values()]

    # ------------------------------------------------------------------ worker logs
    def _describe_worker_logs(self):
        out = {}
        for w in self.workers.values():
            path = getattr(w, "log_path", None)
            if path is None:
                continue
            if w.actor is not None:
                label = w.actor.spec.get("class_name")
            elif w.task is not None and w.task.spec.get("kind") != "lease":
                label = w.task.spec.get("name")  # (a leased worker announces its tasks itself)
            else:
                label = None
            out[w.wid] = (path, w.pid, label, w.node_id, not w.dead)
        return out

    def rpc_list_logs(self, caller, node_id=None, glob=None):
        """``{node_id: [file names]}`` of the session's log directory (reference: ``list_logs``)."""
        import fnmatch

        try:
            names = sorted(os.listdir(self.logs_dir))
        except OSError:
            names = []
        if glob:
            names = [n for n in names if fnmatch.fnmatch(n, glob)]
        by_node = collections.defaultdict(list)
        owner = {os.path.basename(getattr(w, "log_path", "") or ""): w.node_id for w in self.workers.values()}
        for n in names:
            by_node[owner.get(n, self.head_node_id)].append(n)
        if node_id is not None:
            return {node_id: by_node.get(node_id, [])}
        return dict(by_node)

    def rpc_get_log(self, caller, filename=None, actor_id=None, task_id=None, pid=None, worker_id=None, tail=-1):
        """Lines of one worker log, located by file name, actor, task, worker id or pid."""
        path = None
        if filename is not None:
            path = os.path.join(self.logs_dir, os.path.basename(filename))
        else:
            if task_id is not None and worker_id is None:
                ts = self.tasks.get(bytes.fromhex(task_id)) if isinstance(task_id, str) else self.tasks.get(task_id)
                if ts is not None and ts.worker is not None:
                    worker_id = ts.worker.hex()
                else:
                    for rec in self.direct_tasks:
                        if rec[0].hex() == task_id and rec[7] is not None:
                            worker_id = rec[7].hex()
                if worker_id is None:
                    raise ValueError(f"no worker is known for task {task_id}")
            if actor_id is not None:
                a = self.actors.get(bytes.fromhex(actor_id) if isinstance(actor_id, str) else actor_id)
                if a is None:
                    raise ValueError(f"actor {actor_id} not found")
                pid = a.pid
            for w in self.workers.values():
                if (worker_id is not None and w.wid.hex() == worker_id) or (pid is not None and w.pid == pid):
                    path = getattr(w, "log_path", None)
                    break
            if path is None and worker_id is not None:
                path = os.path.join(self.logs_dir, f"worker-{worker_id}.out")
        if path is None or not os.path.exists(path):
            raise ValueError("log file not found")
        return read_log(path, tail)

    def rpc_store_stats(self, caller):
        s = dict(self.store.stats())
        s.update({"spilled_bytes": self.spilled_bytes, "num_spilled": self.num_spilled,
                  "num_restored": self.num_restored, "num_tracked_objects": len(self.objects)})
        return s

    def rpc_timeline(self, caller):
        evs = []
        open_ = {}
        for t, tid, what, name, pid, node in self.events:
            if what == "running":
                open_[tid] = (t, name, pid, node)
            elif what in ("finished", "failed") and tid in open_:
                st, nm, p, nd = open_.pop(tid)
                evs.append({"name": nm or "task", "cat": "task", "ph": "X", "ts": st * 1e6, "dur": (t - st) * 1e6,
                            "pid": nd or "node", "tid": p or 0, "args": {"task_id": tid.hex(), "state": what}})
        for sp in self.spans:  # tracing spans and profile() events
            evs.append({"name": sp["name"], "cat": sp.get("kind", "span"), "ph": "X", "ts": sp["start"] * 1e6,
                        "dur": ((sp["end"] or sp["start"]) - sp["start"]) * 1e6, "pid": "spans", "tid": sp["pid"],
                        "args": {"trace_id": sp["trace_id"], "span_id": sp["span_id"], "parent_id": sp["parent_id"],
                                 **{k: str(v) for k, v in (sp.get("attributes") or {}).items()}}})
        return evs

    def rpc_add_spans(self, caller, spans):
        self.spans.extend(spans)
        return True

    def rpc_spans(self, caller):
        return list(self.spans)

    def rpc_ping(self, caller):
        return "pong"

    # ------------------------------------------------------------------ metrics
    def rpc_metrics_push(self, caller, source, text):
        if not hasattr(self, "_metrics_text"):
            self._metrics_text = {}
        self._metrics_text[source] = (time.time(), text)
        return True

    def rpc_metrics_text(self, caller):
        """Prometheus exposition: built-in cluster gauges + the latest push of every process."""
        from collections import Counter

        lines = []

        def gauge(name, help_, samples):
            lines.append(f"# HELP {name} {help_}")
            lines.append(f"# TYPE {name} gauge")
            for tags, v in samples:
                t = ",".join(f'{k}="{val}"' for k, val in tags.items())
                lines.append(f"{name}{{{t}}} {v}" if t else f"{name} {v}")

        total, avail = self.rpc_cluster_resources(caller), self.rpc_available_resources(caller)
        gauge("rca_cluster_resources_total", "Total logical resources", [({"resource": k}, v) for k, v in total.items()])
        gauge("rca_cluster_resources_available", "Available logical resources",
              [({"resource": k}, v) for k, v in avail.items()])
        st = self.store.stats()
        gauge("rca_object_store_used_bytes", "Shared-memory object store bytes in use", [({}, st.get("used", 0))])
        gauge("rca_object_store_capacity_bytes", "Object store capacity", [({}, st.get("capacity", 0))])
        gauge("rca_object_store_spilled_bytes", "Bytes spilled to disk", [({}, self.spilled_bytes)])
        tc = Counter(TASK_STATE_NAMES[t.state] for t in self.tasks.values())
        gauge("rca_tasks", "Tasks by state", [({"state": k}, v) for k, v in tc.items()])
        ac = self.actor_dir.state_counts()
        gauge("rca_actors", "Actors by state", [({"state": k}, v) for k, v in ac.items()])
        gauge("rca_workers", "Worker processes", [({"node_id": "all"}, len(self.workers))])
        ps = self.wpool.stats()
        gauge("rca_idle_workers", "Idle pooled worker processes", [({"node_id": n}, v["idle"]) for n, v in ps.items()])
        gauge("rca_starting_workers", "Worker processes spawned but not yet registered",
              [({"node_id": n}, v["starting"]) for n, v in ps.items()])
        # GPU object store (HBM-resident objects, per physical GPU) and its host spill traffic
        gauge("rca_gpu_object_store_hbm_bytes", "HBM bytes held by GPU objects",
              [({"gpu": str(k)}, v) for k, v in self.gpu_usage.items()])
        gauge("rca_gpu_object_store_budget_bytes", "GPU object store budget per GPU (0 = unlimited)",
              [({}, self.gpu_budget)])
        gauge("rca_gpu_object_store_objects", "GPU objects by residence",
              [({"state": st}, sum(1 for e in self.gpu_objects.values() if e.gpu["state"] == st))
               for st in ("hbm", "host")])
        gauge("rca_gpu_object_store_spilled_bytes_total", "Bytes of GPU objects spilled HBM -> host",
              [({}, self.gpu_spilled_bytes)])
        gauge("rca_gpu_object_store_spills_total", "GPU objects spilled to host", [({}, self.gpu_num_spilled)])
        gauge("rca_gpu_object_store_restores_total", "GPU objects restored to HBM", [({}, self.gpu_num_restored)])
        # node + MI355X telemetry (sysfs / amd-smi / psutil; reference METRICS_GAUGES names)
        from . import node_telemetry

        if not hasattr(self, "_telemetry"):
            self._telemetry = node_telemetry.TelemetryCache()
        node, gpus = self._telemetry.get()
        lines.extend(node_telemetry.prometheus_lines(node, gpus, ip="127.0.0.1",
                                                     session=os.path.basename(self.session_dir or "")))
        seen = set()
        now = time.time()
        for src, (t, text) in list(getattr(self, "_metrics_text", {}).items()):
            if now - t > 300:
                continue
            for ln in text.splitlines():
                if ln.startswith("#"):
                    if ln in seen:
                        continue
                    seen.add(ln)
                    lines.append(ln)
                elif ln.strip():
                    name, _, rest = ln.partition("{") if "{" in ln.split(" ")[0] else (ln.split(" ")[0], "", "")
                    if rest:
                        lines.append(f'{name}{{source="{src}",{rest}')
                    else:
                        lines.append(f'{ln.split(" ")[0]}{{source="{src}"}} {ln.split(" ", 1)[1]}')
        return "\n".join(lines) + "\n"

    # ================================================================== timers
    def _add_timer(self, delay, fn):
        self.timers.append((time.time() + delay, fn))
        self.wake()

    def _fire_timers(self):
        now = time.time()
        with self.lock:
            due = [t for t in self.timers if t[0] <= now]
            if not due:
                return
            self.timers = [t for t in self.timers if t[0] > now]
            for _, fn in due:
                try:
                    fn()
                except Exception:
                    log.error("timer failed\n%s", traceback.format_exc())

    # ================================================================== shutdown
    def shutdown(self):
        with self.lock:
            if self.shutting_down:
                return
            self.shutting_down = True
            for w in list(self.workers.values()):
                try:
                    if w.conn is not None:
                        w.conn.send((P.EXIT,))
                except OSError:
                    pass
        deadline = time.time() + 2.0
        for w in list(self.workers.values()):
            if w.proc is None:
                continue
            try:
                w.proc.wait(timeout=max(0.05, deadline - time.time()))
            except Exception:
                try:
                    os.killpg(w.proc.pid, 9)
                except Exception:
                    try:
                        w.proc.kill()
                    except Exception:
                        pass
        for w in list(self.workers.values()):
            if w.proc is not None:
                try:
                    w.proc.wait(timeout=1)
                except Exception:
                    pass
        self._thread.join(timeout=2)
        self.log_monitor.stop()  # drains what the workers wrote before they exited
        for c, _cc in list(self.conns.values()):
            try:
                c.close()
            except OSError:
                pass
        self.conns.clear()
        try:
            self.reactor.close()
        except Exception:
            pass
        try:
            self.listener.close()
            os.unlink(self.sock_path)
        except OSError:
            pass
        self.store.unlink()
        if self.config.get("cleanup_session_dir", True):
            shutil.rmtree(self.spill_dir, ignore_errors=True)
        restore_gc(self._prev_gc)
        self._prev_gc = None


class ClientConn:
    """Head-side view of one socket (a worker or an external driver)."""

    def __init__(self, sock):
        self.conn = P.Connection(sock)
        self.reader = P.FrameReader()
        self.worker: Optional[WorkerState] = None
        self.client_key: Optional[str] = None
        self.log_sink = None

    def key(self):
        if self.worker is not None:
            return "w:" + self.worker.wid.hex()
        return self.client_key or "anon"

    def send(self, msg):
        self.conn.send(msg)


def _default_gpu_budget() -> int:
    """30 % of one GPU's HBM (read from sysfs: no HIP initialisation in the head), 0 = unlimited."""
    env = os.environ.get("RCA_GPU_OBJECT_STORE_MEMORY")
    if env:
        return int(float(env))
    try:
        import glob

        for f in sorted(glob.glob("/sys/class/drm/card*/device/mem_info_vram_total")):
            with open(f) as fh:
                v = int(fh.read().strip())
            if v > 0:
                return int(v * 0.3)
    except (OSError, ValueError):
        pass
    return 0


def worker_hip_visible_devices(gpus, environ) -> str:
    """``HIP_VISIBLE_DEVICES`` for a worker that owns the head's logical GPUs ``gpus``.

    The head's logical GPU ``g`` is the g-th device the head process itself sees. ROCm applies the
    two masks in layers: ``ROCR_VISIBLE_DEVICES`` filters the agents the ROCr runtime exposes, and
    ``HIP_VISIBLE_DEVICES`` (or ``CUDA_VISIBLE_DEVICES``) then indexes INTO that filtered set. The
    worker inherits the parent's ``ROCR_VISIBLE_DEVICES`` unchanged, so its HIP-level ids are:
      * the parent's HIP/CUDA mask entry ``g`` when the parent has one;
      * otherwise plain ``g`` -- never a ROCR id (with ``ROCR_VISIBLE_DEVICES=4,5`` the worker's
        devices are HIP 0 and 1; ``HIP_VISIBLE_DEVICES=4`` would select nothing).
    """
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = environ.get(var)
        if v:
            vis = [x.strip() for x in v.split(",") if x.strip()]
            return ",".join(vis[g] if g < len(vis) else str(g) for g in gpus)
    return ",".join(str(g) for g in gpus)
