"""Compiled (accelerated) DAG execution (reference: ``python/ray/dag/compiled_dag_node.py``).

``dag.experimental_compile()`` turns a graph of actor-method nodes into a static pipeline:
every actor runs ONE resident loop (a thread started through ``__ray_call__``) that reads its
inputs from shared-memory channels (``experimental/channel.py``), calls the bound methods in
topological order and writes each result to a channel read by the downstream actors and/or the
driver. ``execute(x)`` is then a single shared-memory write; no task submission, scheduling or
object-store traffic per call. Edges between two methods of the SAME actor are passed in-process.
Exceptions travel through the channels as values and are re-raised on ``begin_read``.
"""
from __future__ import annotations

import asyncio
import threading
import time
import traceback
from typing import Any, Dict, List, Optional, Tuple

from ..experimental.channel import Channel, _Closed
from .dag_node import (ClassMethodNode, ClassNode, DAGInputData, DAGNode, InputAttributeNode, InputNode,
                       MultiOutputNode, _scan_nodes)


class _DAGTaskError:
    def __init__(self, exc: BaseException, tb: str):
        self.exc = exc
        self.tb = tb


def _spec_of(x):
    """Turn a bound argument into a loop-side spec."""
    if isinstance(x, (InputNode, InputAttributeNode)):
        spec = ("input",) if isinstance(x, InputNode) else ("input_attr", x.key, x._accessor)
        return spec
    if isinstance(x, ClassMethodNode):
        return ("node", id(x))
    if isinstance(x, DAGNode):
        raise TypeError(f"compiled DAGs support only actor method nodes and InputNode arguments, got {x}")
    return ("const", x)


def _on_device(node) -> bool:
    h = getattr(node, "type_hint", None)
    return bool(h is not None and getattr(h, "on_device", False))


def _actor_loop_main(actor, plan):
    """Runs inside the actor process (thread). ``plan``: channels + this actor's ordered tasks."""
    in_ch: Optional[Channel] = plan["input"]
    in_reader = plan["input_reader"]
    reads: Dict[int, Tuple[Channel, int]] = plan["reads"]  # node id -> (channel, reader index)
    tasks = plan["tasks"]
    from .torch_tensor import DeviceSender, receiver

    senders = {t["nid"]: DeviceSender() for t in tasks if t.get("device")}
    recv = receiver() if plan.get("device_reads") else None
    while True:
        local: Dict[int, Any] = {}
        fetched: Dict[int, Any] = {}
        inp = None
        closed = False
        if in_ch is not None:
            inp = in_ch.begin_read(in_reader)
            closed = isinstance(inp, _Closed)
        for nid, (ch, r) in reads.items():
            if closed:
                break
            v = ch.begin_read(r)
            if isinstance(v, _Closed):
                closed = True
                break
            fetched[nid] = recv.unpack(v) if recv is not None else v
        if closed:
            for t in tasks:
                if t["out"] is not None:
                    t["out"].close()
            if in_ch is not None:
                in_ch.end_read(in_reader)
            for ch, r in reads.values():
                ch.end_read(r)
            return

        def resolve(spec):
            kind = spec[0]
            if kind == "const":
                return spec[1]
            if kind == "input":
                return inp
            if kind == "input_attr":
                if isinstance(inp, DAGInputData):
                    return inp[spec[1]]
                return inp[spec[1]] if spec[2] == "__getitem__" else getattr(inp, spec[1])
            nid = spec[1]
            return local[nid] if nid in local else fetched[nid]

        for t in tasks:
            args = [resolve(s) for s in t["args"]]
            kwargs = {k: resolve(s) for k, s in t["kwargs"].items()}
            err = next((a for a in list(args) + list(kwargs.values()) if isinstance(a, _DAGTaskError)), None)
            if err is not None:
                out = err
            else:
                try:
                    out = getattr(actor, t["method"])(*args, **kwargs)
                    if asyncio.iscoroutine(out):
                        out = asyncio.run(out)
                except Exception as e:  # noqa
                    out = _DAGTaskError(e, traceback.format_exc())
            local[t["nid"]] = out
            if t["out"] is not None:
                snd = senders.get(t["nid"])
                if snd is not None and not isinstance(out, _DAGTaskError):
                    try:
                        out = snd.pack(out)
                    except Exception as e:  # noqa
                        out = _DAGTaskError(e, traceback.format_exc())
                t["out"].write(out)
        if in_ch is not None:
            in_ch.end_read(in_reader)
        for ch, r in reads.values():
            ch.end_read(r)


def _start_loop(actor, plan):
    th = threading.Thread(target=_actor_loop_main, args=(actor, plan), daemon=True, name="rca-compiled-dag")
    th.start()
    return True


class CompiledDAGRef:
    """Result handle of one ``CompiledDAG.execute`` (``begin_read``/``end_read`` or ``get``).

    Results leave the output channels in execution order; a ref read out of order, or an execute
    that finds the input channel full, moves earlier results into the DAG's result buffer first
    (reference: CompiledDAG._result_buffer / max_buffered_results,
    /root/reference/python/ray/dag/compiled_dag_node.py), so any number of executions may be in
    flight and refs may be read in any order."""

    def __init__(self, dag: "CompiledDAG", seq: int):
        self._dag = dag
        self._seq = seq
        self._read = False

    def begin_read(self, timeout: Optional[float] = None):
        vals = self._dag._result_of(self._seq, timeout)
        self._read = True
        for v in vals:
            if isinstance(v, _DAGTaskError):
                raise v.exc
        return vals if self._dag._multi else vals[0]

    def end_read(self):
        self._read = False  # values were copied out of the channels when they were fetched

    def get(self, timeout: Optional[float] = None):
        try:
            return self.begin_read(timeout)
        finally:
            self.end_read()


class CompiledDAG:
    def __init__(self, root: DAGNode, buffer_size_bytes: Optional[int] = None, enable_asyncio: bool = False,
                 max_buffered_results: int = 1000):
        from .._private.worker import get

        self._enable_asyncio = enable_asyncio
        self._buffer = buffer_size_bytes
        nodes = root._topo()
        self._multi = isinstance(root, MultiOutputNode)
        out_nodes = list(root.get_args()) if self._multi else [root]
        for o in out_nodes:
            if not isinstance(o, ClassMethodNode):
                raise TypeError("compiled DAG outputs must be actor method nodes")
        # actors: ClassNodes are instantiated now
        handles: Dict[int, Any] = {}
        for n in nodes:
            if isinstance(n, ClassNode):
                if n._children():
                    raise TypeError("ClassNode constructor arguments must be constants in a compiled DAG")
                handles[id(n)] = n._execute_impl(list(n.get_args()), n.get_kwargs(), {}, (), {})
        methods = [n for n in nodes if isinstance(n, ClassMethodNode)]
        if not methods:
            raise ValueError("nothing to compile: the DAG has no actor method nodes")

        def actor_of(m: ClassMethodNode):
            a = m._actor
            return handles[id(a)] if isinstance(a, ClassNode) else a

        akey = {id(m): actor_of(m)._actor_id for m in methods}
        by_actor: Dict[bytes, List[ClassMethodNode]] = {}
        handle_of: Dict[bytes, Any] = {}
        for m in methods:
            by_actor.setdefault(akey[id(m)], []).append(m)
            handle_of[akey[id(m)]] = actor_of(m)
        # consumers of each method node / of the input, by actor
        consumers: Dict[int, set] = {id(m): set() for m in methods}
        input_consumers: set = set()
        for m in methods:
            deps: List[DAGNode] = []
            _scan_nodes(list(m.get_args()), deps)
            _scan_nodes(m.get_kwargs(), deps)
            for d in deps:
                if isinstance(d, ClassMethodNode):
                    if akey[id(d)] != akey[id(m)]:
                        consumers[id(d)].add(akey[id(m)])
                elif isinstance(d, (InputNode, InputAttributeNode)):
                    input_consumers.add(akey[id(m)])
                else:
                    raise TypeError(f"unsupported node {d} in a compiled DAG")
        out_ids = [id(o) for o in out_nodes]
        self._channels: List[Channel] = []
        out_chan: Dict[int, Channel] = {}
        reader_idx: Dict[Tuple[int, Any], int] = {}
        for m in methods:
            readers = sorted(consumers[id(m)])
            n_driver = 1 if id(m) in out_ids else 0
            if not readers and not n_driver:
                continue
            ch = Channel(buffer_size_bytes, len(readers) + n_driver)
            self._channels.append(ch)
            out_chan[id(m)] = ch
            for i, ak in enumerate(readers):
                reader_idx[(id(m), ak)] = i
            if n_driver:
                reader_idx[(id(m), "driver")] = len(readers)
        in_readers = sorted(input_consumers)
        self._input = Channel(buffer_size_bytes, max(1, len(in_readers))) if in_readers else None
        if self._input is not None:
            self._channels.append(self._input)
        # per-actor plans
        loops = []
        for ak, ms in by_actor.items():
            reads = {}
            tasks = []
            for m in ms:
                deps: List[DAGNode] = []
                _scan_nodes(list(m.get_args()), deps)
                _scan_nodes(m.get_kwargs(), deps)
                for d in deps:
                    if isinstance(d, ClassMethodNode) and akey[id(d)] != ak:
                        reads[id(d)] = (out_chan[id(d)], reader_idx[(id(d), ak)])
                args = [_spec_of(a) for a in m.get_args()]
                kwargs = {k: _spec_of(v) for k, v in m.get_kwargs().items()}
                tasks.append({"nid": id(m), "method": m.get_method_name(), "args": args, "kwargs": kwargs,
                              "out": out_chan.get(id(m)), "device": _on_device(m)})
            plan = {"input": self._input if ak in input_consumers else None,
                    "input_reader": in_readers.index(ak) if ak in input_consumers else 0,
                    "reads": reads, "tasks": tasks,
                    "device_reads": any(_on_device(d) for d in methods if id(d) in reads)}
            loops.append(handle_of[ak].__ray_call__.remote(_start_loop, plan))
        get(loops)
        self._outputs = [(out_chan[i], reader_idx[(i, "driver")]) for i in out_ids]
        self._device_outputs = any(_on_device(o) for o in out_nodes)
        self._handles = handle_of
        self._seq = 0
        self._next_read = 1          # seq of the next result waiting in the output channels
        self._partial: list = []     # outputs of execution ``_next_read`` read before a timeout
        self._results: Dict[int, list] = {}
        self._max_buffered = int(max_buffered_results)
        self._torn_down = False

    def _fetch_next(self, timeout: Optional[float] = None):
        """Moves the oldest unread execution's outputs from the channels into the result buffer."""
        if len(self._results) >= self._max_buffered:
            raise RuntimeError(f"compiled DAG holds {len(self._results)} unread results "
                               f"(max_buffered_results={self._max_buffered}); read earlier refs first")
        # channel by channel: each value is copied out and its channel released before the next
        # read, and the values already read are kept in ``_partial``, so a timeout on a later
        # output leaves no channel half-read and the retry resumes at the output that timed out
        vals = self._partial
        for ch, r in self._outputs[len(vals):]:
            v = ch.begin_read(r, timeout)
            try:
                if self._device_outputs:
                    from .torch_tensor import receiver

                    v = receiver().unpack(v)  # copied out before the channel is released
            finally:
                ch.end_read(r)
            vals.append(v)
        self._partial = []
        self._results[self._next_read] = vals
        self._next_read += 1

    def _result_of(self, seq: int, timeout: Optional[float] = None) -> list:
        if seq not in self._results and seq < self._next_read:
            raise ValueError("this compiled DAG result was already read")
        while seq >= self._next_read:
            self._fetch_next(timeout)
        return self._results.pop(seq)

    def execute(self, *args, **kwargs) -> CompiledDAGRef:
        if self._torn_down:
            raise RuntimeError("compiled DAG was torn down")
        if self._enable_asyncio:
            raise ValueError("Use execute_async if enable_asyncio=True")
        value = args[0] if len(args) == 1 and not kwargs else DAGInputData(*args, **kwargs)
        if self._input is not None:
            # a full input channel with results still unread means the pipeline is backed up behind
            # the driver: drain results into the buffer until the input can take the value
            while not self._input.can_write():
                if self._next_read <= self._seq:
                    self._fetch_next()
                else:
                    time.sleep(20e-6)
            self._input.write(value)
        self._seq += 1
        return CompiledDAGRef(self, self._seq)

    async def execute_async(self, *args, **kwargs):
        loop = asyncio.get_running_loop()
        self._enable_asyncio, was = False, self._enable_asyncio
        try:
            ref = await loop.run_in_executor(None, lambda: self.execute(*args, **kwargs))
        finally:
            self._enable_asyncio = was
        fut = loop.run_in_executor(None, ref.get)
        return await fut

    def teardown(self, timeout: float = 10.0):
        if self._torn_down:
            return
        self._torn_down = True
        try:
            if self._input is not None:
                self._input.close()
            for ch, r in self._outputs:
                try:
                    while not isinstance(ch.begin_read(r, timeout), _Closed):
                        ch.end_read(r)
                    ch.end_read(r)
                except Exception:
                    pass
        finally:
            for ch in self._channels:
                ch.destroy()

    def __del__(self):
        try:
            self.teardown(timeout=1.0)
        except Exception:
            pass


def build_compiled_dag(root: DAGNode, buffer_size_bytes=None, enable_asyncio=False,
                       max_buffered_results=None) -> CompiledDAG:
    return CompiledDAG(root, buffer_size_bytes, enable_asyncio,
                       1000 if max_buffered_results is None else max_buffered_results)
