"""Streaming executor: a scheduling thread over an operator topology (reference:
``python/ray/data/_internal/execution/streaming_executor.py:55`` ``StreamingExecutor`` and its
``_scheduling_loop_step`` :262, ``streaming_executor_state.py`` ``select_operator_to_run``,
``operators/actor_pool_map_operator.py:458-545`` autoscaling actor pools).

Design (not a translation -- the reference drives Ray's C++ task submission from a Python loop
over ``OpState`` queues; this one does the same against this runtime's task/actor API):

* The plan is a chain of physical operators: ``InputOp`` (read tasks or existing refs),
  ``TaskMapOp`` (fused task-compute map chain, one task per block), ``ActorPoolMapOp``
  (callable-class UDFs on an autoscaling actor pool), ``LimitOp``, ``AllToAllOp`` (barrier:
  repartition / shuffle / sort / groupby exchanges) and the streaming n-ary ``UnionOp`` /
  ``ZipOp``, whose other inputs are datasets executing concurrently (``_SideInput``).
* One background thread runs the loop: retire finished tasks (one non-blocking ``wait`` over
  every operator's outstanding metadata refs), move outputs downstream, autoscale actor pools,
  and dispatch new tasks downstream-first while the resource manager's budgets
  (``resource_manager.py``: CPU/GPU limits, per-operator object-store shares, concurrency caps)
  and each operator's output-queue bound allow. The consumer pulls finished blocks from a
  bounded queue, so a slow consumer backpressures the whole pipeline.
* Ordering: with ``DataContext.execution_options.preserve_order`` (default True here) every
  operator releases outputs in input order (a reorder buffer keyed by sequence number);
  with False they flow out as they complete, so one slow task or actor no longer holds back
  the others (head-of-line blocking).
* Actor pools scale between ``min_size`` and ``max_size``: up by one actor when work is queued
  and every live actor is saturated (``max_tasks_in_flight_per_actor``) and the newest actor
  is ready; down when an actor has been idle for ``actor_pool_idle_timeout_s`` and nothing is
  queued. Pool sizes over time are kept in the operator's stats.
"""
from __future__ import annotations

import collections
import queue
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

_DONE = object()


class _Bundle:
    __slots__ = ("seq", "block", "meta")

    def __init__(self, seq, block, meta):
        self.seq = seq
        self.block = block
        self.meta = meta


class PhysicalOp:
    """One operator: an input queue, running tasks, and an output buffer released downstream
    (in order or as completed)."""

    def __init__(self, name: str, ordered: bool, rm=None, rm_op=None):
        self.name = name
        self.ordered = ordered
        self.rm = rm
        self.rm_op = rm_op
        self.inq: collections.deque = collections.deque()
        self.running: Dict[Any, Tuple[int, Any, Any]] = {}  # meta ref -> (seq, block ref, extra)
        self.finished: Dict[int, _Bundle] = {}               # seq -> bundle (ordered mode)
        self.ready_out: collections.deque = collections.deque()
        self.next_seq = 0
        self.upstream_done = False
        self.downstream: Optional["PhysicalOp"] = None
        self.out_limit = 8
        self.stats: Dict[str, Any] = {"name": name, "tasks": 0}

    # -------------------------------------------------------------- queues
    def add_input(self, b: _Bundle):
        self.inq.append(b)

    def pending_outputs(self) -> int:
        return len(self.ready_out) + len(self.finished)

    def _emit(self, b: _Bundle):
        if not self.ordered:
            self.ready_out.append(b)
            return
        self.finished[b.seq] = b
        while self.next_seq in self.finished:
            self.ready_out.append(self.finished.pop(self.next_seq))
            self.next_seq += 1

    def take_outputs(self) -> List[_Bundle]:
        out = list(self.ready_out)
        self.ready_out.clear()
        return out

    def on_task_done(self, meta_ref):
        seq, block, _ = self.running.pop(meta_ref)
        if self.rm is not None:
            self.rm.on_finish(self.rm_op, meta_ref)
        self._emit(_Bundle(seq, block, meta_ref))

    # -------------------------------------------------------------- scheduling
    def can_dispatch(self) -> bool:
        return bool(self.inq)

    def dispatch_one(self):
        raise NotImplementedError

    def done(self) -> bool:
        return self.upstream_done and not self.inq and not self.running and not self.finished and not self.ready_out

    def autoscale(self, now: float):
        pass

    def shutdown(self):
        pass


class InputOp(PhysicalOp):
    """Read tasks (one per input) or already-materialised block refs."""

    def __init__(self, inputs, ordered, rm, rm_op):
        super().__init__("Input", ordered, rm, rm_op)
        from .execution import _read_task, _remote_fn

        self._rf = None
        self._read = _read_task
        self._mk = _remote_fn
        for i, x in enumerate(inputs):
            if x[0] == "ref":
                self._emit(_Bundle(i, x[1], x[2]))
            else:
                self.inq.append(_Bundle(i, x[1], None))
        self.upstream_done = True

    def dispatch_one(self):
        b = self.inq.popleft()
        if self._rf is None:
            self._rf = self._mk(self._read, {"num_cpus": 1})
        blk, meta = self._rf.remote(b.block)
        self.running[meta] = (b.seq, blk, None)
        self.stats["tasks"] += 1
        if self.rm is not None:
            self.rm.on_submit(self.rm_op, meta)


class TaskMapOp(PhysicalOp):
    def __init__(self, name, ops, remote_opts, ordered, rm, rm_op):
        super().__init__(name, ordered, rm, rm_op)
        from .execution import _remote_fn, _run_chain

        self._rf = _remote_fn(_run_chain, remote_opts)
        self._ops = ops

    def dispatch_one(self):
        b = self.inq.popleft()
        blk, meta = self._rf.remote(b.block, self._ops)
        self.running[meta] = (b.seq, blk, None)
        self.stats["tasks"] += 1
        if self.rm is not None:
            self.rm.on_submit(self.rm_op, meta)


class ActorPoolMapOp(PhysicalOp):
    def __init__(self, name, op, actor_opts, min_size, max_size, max_in_flight, idle_timeout_s, ordered, rm,
                 rm_op, pre_ops=None):
        super().__init__(name, ordered, rm, rm_op)
        self._pre = list(pre_ops or [])  # fused upstream task-compute maps, run in the actor first
        from ...actor import ActorClass
        from .execution import _MapActor

        self._cls = ActorClass(_MapActor, actor_opts)
        self._op = op
        self.min_size = max(1, int(min_size))
        self.max_size = max(self.min_size, int(max_size))
        self.max_in_flight = max(1, int(max_in_flight))
        self.idle_timeout_s = idle_timeout_s
        self.actors: Dict[int, Dict[str, Any]] = {}
        self._next_id = 0
        self.stats.update({"pool_size_history": [], "peak_pool_size": 0, "scale_ups": 0, "scale_downs": 0})
        for _ in range(self.min_size):
            self._add_actor()

    def _add_actor(self):
        op = self._op
        h = self._cls.remote(op["fn"], op.get("fn_constructor_args", ()), op.get("fn_constructor_kwargs", {}),
                             self._pre, [], {k: v for k, v in op.items() if k != "fn"})
        self.actors[self._next_id] = {"h": h, "load": 0, "ready": h.ready.remote(), "is_ready": False,
                                      "idle_since": time.monotonic()}
        self._next_id += 1
        self._record_size()

    def _record_size(self):
        n = len(self.actors)
        self.stats["pool_size_history"].append((time.monotonic(), n))
        self.stats["peak_pool_size"] = max(self.stats["peak_pool_size"], n)

    def _pick(self):
        best = None
        for aid, a in self.actors.items():
            if a["load"] >= self.max_in_flight:
                continue
            key = (not a["is_ready"], a["load"])
            if best is None or key < best[0]:
                best = (key, aid)
        return None if best is None else best[1]

    def can_dispatch(self) -> bool:
        return bool(self.inq) and self._pick() is not None

    def dispatch_one(self):
        aid = self._pick()
        a = self.actors[aid]
        b = self.inq.popleft()
        blk, meta = a["h"].process.options(num_returns=2).remote(b.block)
        a["load"] += 1
        self.running[meta] = (b.seq, blk, aid)
        self.stats["tasks"] += 1
        if self.rm is not None:
            self.rm.on_submit(self.rm_op, meta)

    def on_task_done(self, meta_ref):
        aid = self.running[meta_ref][2]
        a = self.actors.get(aid)
        if a is not None:
            a["load"] -= 1
            if a["load"] == 0:
                a["idle_since"] = time.monotonic()
        super().on_task_done(meta_ref)

    def autoscale(self, now: float):
        from ..._private.worker import kill, wait

        pend = [a["ready"] for a in self.actors.values() if not a["is_ready"]]
        if pend:
            ready, _ = wait(pend, num_returns=len(pend), timeout=0)
            rs = set(id(r) for r in ready)
            for a in self.actors.values():
                if not a["is_ready"] and id(a["ready"]) in rs:
                    a["is_ready"] = True
        # up: queued work, every actor saturated, no actor still starting, below max
        if (self.inq and len(self.actors) < self.max_size and all(a["is_ready"] for a in self.actors.values())
                and all(a["load"] >= self.max_in_flight for a in self.actors.values())):
            self._add_actor()
            self.stats["scale_ups"] += 1
        # down: idle actors beyond min_size while nothing is queued
        if not self.inq and len(self.actors) > self.min_size:
            for aid, a in sorted(self.actors.items(), key=lambda kv: -kv[0]):
                if len(self.actors) <= self.min_size:
                    break
                if a["load"] == 0 and a["is_ready"] and now - a["idle_since"] >= self.idle_timeout_s:
                    try:
                        kill(a["h"])
                    except Exception:
                        pass
                    del self.actors[aid]
                    self.stats["scale_downs"] += 1
                    self._record_size()

    def done(self) -> bool:
        return super().done()

    def shutdown(self):
        from ..._private.worker import kill

        for a in self.actors.values():
            try:
                kill(a["h"])
            except Exception:
                pass
        self.actors.clear()
        self._record_size()


class LimitOp(PhysicalOp):
    """Passes the first ``n`` rows through (truncating one block), then tells every upstream
    operator to stop launching work."""

    def __init__(self, n, ordered, executor):
        super().__init__(f"Limit[{n}]", ordered)
        self.n = n
        self.seen = 0
        self.executor = executor
        self._trunc = None

    def can_dispatch(self) -> bool:
        return bool(self.inq)

    def dispatch_one(self):
        from ..._private.worker import get
        from .execution import _remote_fn, _truncate

        b = self.inq.popleft()
        if self.seen >= self.n:
            return
        rows = get(b.meta)["num_rows"]
        if self.seen + rows <= self.n:
            self.seen += rows
            self.ready_out.append(b)
        else:
            if self._trunc is None:
                self._trunc = _remote_fn(_truncate, {"num_cpus": 0.5})
            blk, meta = self._trunc.remote(b.block, self.n - self.seen)
            self.seen = self.n
            self.ready_out.append(_Bundle(b.seq, blk, meta))
        if self.seen >= self.n:
            self.inq.clear()
            self.executor.stop_upstream_of(self)


    def done(self) -> bool:
        return (self.seen >= self.n and not self.ready_out) or super().done()


class AllToAllOp(PhysicalOp):
    """Barrier: collects every input (in sequence order), then runs the exchange function."""

    def __init__(self, name, fn, ordered):
        super().__init__(name, ordered)
        self.fn = fn
        self._fired = False

    def can_dispatch(self) -> bool:
        return self.upstream_done and not self._fired

    def dispatch_one(self):
        self._fired = True
        ins = sorted(self.inq, key=lambda b: b.seq)
        self.inq.clear()
        outs = self.fn([(b.block, b.meta) for b in ins])
        for i, (blk, meta) in enumerate(outs):
            self.ready_out.append(_Bundle(i, blk, meta))

    def done(self) -> bool:
        return self._fired and not self.ready_out


class _SideInput:
    """Another dataset streamed into an n-ary operator: a pump thread pulls ``(block, meta)``
    pairs from that dataset's own streaming execution into a queue of at most ``window`` items,
    so the side input runs concurrently with this pipeline and is backpressured by it."""

    def __init__(self, ds, window: int):
        self.ds = ds
        self.items: collections.deque = collections.deque()
        self.room = threading.Semaphore(max(1, window))
        self.exhausted = False
        self.error: Optional[BaseException] = None
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def start(self):
        if self._t is None:
            self._t = threading.Thread(target=self._pump, name="rca-data-side-input", daemon=True)
            self._t.start()

    def _pump(self):
        gen = None
        try:
            gen = self.ds._iter_refs()
            while not self._stop.is_set():
                self.room.acquire()
                if self._stop.is_set():
                    break
                try:
                    item = next(gen)
                except StopIteration:
                    break
                self.items.append(item)
        except BaseException as e:  # noqa  (re-raised by the operator in the executor loop)
            self.error = e
        finally:
            self.exhausted = True
            if gen is not None and hasattr(gen, "close"):
                try:
                    gen.close()
                except Exception:
                    pass

    def poll(self):
        if self.error is not None:
            raise self.error
        if self.items:
            item = self.items.popleft()
            self.room.release()
            return item
        return None

    def drained(self) -> bool:
        return self.exhausted and not self.items

    def close(self):
        self._stop.set()
        self.room.release()
        ex = getattr(self.ds, "_executor", None)
        if ex is not None and not self.exhausted:
            ex._stop.set()
        t = self._t
        if t is not None and t is not threading.current_thread():
            t.join(timeout=10.0)  # the pump must not outlive the pipeline (nor the session)


class UnionOp(PhysicalOp):
    """Streaming union (reference ``operators/union_operator.py``): this pipeline's blocks and
    the other datasets' blocks, each other dataset executing concurrently through its own
    streaming execution. Ordered mode emits the inputs one after another (this dataset's
    blocks first); otherwise blocks flow out as they become available."""

    def __init__(self, others, ordered, window):
        super().__init__("Union", ordered)
        self.sides = [_SideInput(o, 2) for o in others]  # each other dataset's executor window sits behind it
        self._out = 0

    def _start(self):
        for sd in self.sides:
            sd.start()

    def _pass(self, block, meta):
        self.ready_out.append(_Bundle(self._out, block, meta))
        self._out += 1

    def _side(self) -> Optional[_SideInput]:
        """The side input the next block may come from (None: nothing available now)."""
        for sd in self.sides:
            if sd.error is not None:
                raise sd.error
        if self.ordered:
            if not self.upstream_done or self.inq:
                return None
            for sd in self.sides:
                if sd.items:
                    return sd
                if not sd.drained():
                    return None  # keep the order: wait for this input before the next one
            return None
        return next((sd for sd in self.sides if sd.items), None)

    def can_dispatch(self) -> bool:
        self._start()
        return bool(self.inq) or self._side() is not None

    def dispatch_one(self):
        if self.inq:
            b = self.inq.popleft()
            self._pass(b.block, b.meta)
            return
        self._pass(*self._side().poll())

    def done(self) -> bool:
        self._start()
        return (self.upstream_done and not self.inq and not self.ready_out
                and all(sd.drained() for sd in self.sides))

    def shutdown(self):
        for sd in self.sides:
            sd.close()


class ZipOp(PhysicalOp):
    """Streaming zip: row-aligns this pipeline's blocks with another dataset's (executing
    concurrently) and launches one zip task per aligned run of rows as soon as both sides have
    it -- no barrier (the reference's ``operators/zip_operator.py`` materialises both inputs
    first). Row counts come from the block metadata; a row-count mismatch raises at the end."""

    def __init__(self, other, ordered, window):
        super().__init__("Zip", ordered)
        self.side = _SideInput(other, 2)  # the other dataset's own executor window sits behind it
        self.left: collections.deque = collections.deque()   # [block, rows, offset]
        self.right: collections.deque = collections.deque()
        self._out = 0
        self._zip = None
        self._zip_pending = None  # a side-input item polled but whose metadata is not ready yet

    @staticmethod
    def _rows(meta):
        from ..._private.worker import get

        return int(get(meta)["num_rows"])

    @staticmethod
    def _meta_ready(meta) -> bool:
        """Non-blocking: is the block's metadata computed? (The executor loop never waits on an
        object fetch here; a block whose metadata is pending is taken on a later pass.)"""
        from ..._private.worker import wait

        ready, _ = wait([meta], num_returns=1, timeout=0)
        return bool(ready)

    def _refill(self):
        """Hold at most two blocks of each side here: the rest stays upstream (this op's input
        queue, the side input's bounded queue), where the executor's windows bound it."""
        self.side.start()
        for q in (self.left, self.right):
            while q and q[0][1] - q[0][2] <= 0:
                q.popleft()
        while self.inq and len(self.left) < 2 and self._meta_ready(self.inq[0].meta):
            b = self.inq.popleft()
            self.left.append([b.block, self._rows(b.meta), 0])
        while len(self.right) < 2:
            if self._zip_pending is None:
                self._zip_pending = self.side.poll()
            it = self._zip_pending
            if it is None or not self._meta_ready(it[1]):
                break
            self._zip_pending = None
            self.right.append([it[0], self._rows(it[1]), 0])
        for q in (self.left, self.right):
            while q and q[0][1] - q[0][2] <= 0:
                q.popleft()

    def can_dispatch(self) -> bool:
        self._refill()
        return bool(self.left and self.right)

    def dispatch_one(self):
        from .execution import _remote_fn, _zip_slices

        if self._zip is None:
            self._zip = _remote_fn(_zip_slices, {"num_cpus": 0.5})
        lb, rb = self.left[0], self.right[0]
        k = min(lb[1] - lb[2], rb[1] - rb[2])
        blk, meta = self._zip.remote(lb[0], lb[2], rb[0], rb[2], k)
        self.running[meta] = (self._out, blk, None)
        self._out += 1
        self.stats["tasks"] += 1
        lb[2] += k
        rb[2] += k
        for q in (self.left, self.right):
            if q[0][2] >= q[0][1]:
                q.popleft()

    def done(self) -> bool:
        self._refill()
        if not (self.upstream_done and self.side.drained() and not self.inq) or self._zip_pending is not None:
            return False
        self._refill()
        if self.left and self.right:
            return False  # more aligned rows to dispatch (waiting for downstream room)
        if self.left or self.right:
            if not self.running:
                n_l = sum(x[1] - x[2] for x in self.left)
                n_r = sum(x[1] - x[2] for x in self.right)
                raise ValueError(f"Cannot zip datasets of different number of rows: {n_l} left over on "
                                 f"one side, {n_r} on the other")
            return False
        return not self.running and not self.finished and not self.ready_out

    def shutdown(self):
        self.side.close()


class StreamingExecutor:
    def __init__(self, ops: List[PhysicalOp], rm, out_window: int):
        self.ops = ops
        for a, b in zip(ops, ops[1:]):
            a.downstream = b
        self.rm = rm
        self.out_window = max(1, out_window)
        for o in ops:
            o.out_limit = self.out_window
        self.outq: "queue.Queue" = queue.Queue()
        self._out_count = 0
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.stats: Dict[str, Any] = {}

    # -------------------------------------------------------------- control
    def start(self):
        self._thread = threading.Thread(target=self._run, name="rca-data-executor", daemon=True)
        self._thread.start()
        return self

    def stop_upstream_of(self, op: PhysicalOp):
        for o in self.ops:
            if o is op:
                break
            o.inq.clear()
            o.upstream_done = True
            if isinstance(o, InputOp):
                o.inq.clear()

    def shutdown(self):
        self._stop.set()
        t = self._thread
        if t is not None and t is not threading.current_thread():
            t.join(timeout=30)
        for o in self.ops:
            try:
                o.shutdown()
            except Exception:
                pass

    def consumed(self):
        with self._lock:
            self._out_count -= 1

    # -------------------------------------------------------------- loop
    def _downstream_room(self, op: PhysicalOp) -> bool:
        if op.downstream is None:
            with self._lock:
                return self._out_count + op.pending_outputs() + len(op.running) < self.out_window
        d = op.downstream
        if isinstance(d, AllToAllOp):
            # a barrier consumes its whole input before it emits anything: bounding its input
            # queue would stall the producer short of the barrier forever (more input blocks than
            # the window)
            return True
        return len(d.inq) + op.pending_outputs() + len(op.running) < op.out_limit

    def _can_run(self, op: PhysicalOp) -> bool:
        if not op.can_dispatch() or not self._downstream_room(op):
            return False
        if self.rm is not None and op.rm_op is not None and not self.rm.can_submit(op.rm_op, poll=False):
            return False
        return True

    def _step(self) -> bool:
        from ..._private.worker import wait

        progressed = False
        refs = [r for o in self.ops for r in o.running]
        if refs:
            ready, _ = wait(refs, num_returns=len(refs), timeout=0)
            if not ready and not any(self._can_run(o) for o in self.ops):
                ready, _ = wait(refs, num_returns=1, timeout=0.05)
            if ready:
                rs = set(ready)
                for o in self.ops:
                    for r in [r for r in o.running if r in rs]:
                        o.on_task_done(r)
                progressed = True
        # release outputs downstream (and to the consumer)
        for o in self.ops:
            outs = o.take_outputs()
            if not outs:
                continue
            progressed = True
            if o.downstream is None:
                with self._lock:
                    self._out_count += len(outs)
                for b in outs:
                    self.outq.put(b)
            else:
                for b in outs:
                    o.downstream.add_input(b)
        # completion propagates forward
        for a, b in zip(self.ops, self.ops[1:]):
            if a.done() and not b.upstream_done:
                b.upstream_done = True
                progressed = True
        now = time.monotonic()
        for o in self.ops:
            o.autoscale(now)
        # dispatch, downstream first (drain before filling)
        for o in reversed(self.ops):
            while self._can_run(o):
                o.dispatch_one()
                progressed = True
        return progressed

    def _run(self):
        try:
            while not self._stop.is_set():
                progressed = self._step()
                if self.ops[-1].done():
                    break
                if not progressed:
                    time.sleep(0.002)
        except BaseException as e:  # noqa  (surface in the consumer)
            self.outq.put(e)
        finally:
            for o in self.ops:
                try:
                    o.shutdown()
                except Exception:
                    pass
            self.stats = {o.name: dict(o.stats) for o in self.ops}
            self.outq.put(_DONE)

    def iter_outputs(self):
        """Yields (block ref, meta ref) as the final operator releases them."""
        try:
            while True:
                item = self.outq.get()
                if item is _DONE:
                    return
                if isinstance(item, BaseException):
                    raise item
                self.consumed()
                yield item.block, item.meta
        finally:
            self.shutdown()
