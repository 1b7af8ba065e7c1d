"""Resource budget and backpressure for the streaming executor.

Reference behaviour: ``python/ray/data/_internal/execution/resource_manager.py:32`` (global
limits from the cluster, a reserved share of them per operator plus a shared pool) and
``execution/backpressure_policy/`` (per-operator concurrency caps). Consulted by the streaming
executor's scheduling loop (``streaming_executor.py``) before every dispatch:

  * every stage registers an :class:`OpState`; a stage asks :meth:`ResourceManager.can_submit`
    before launching a task and, when it has nothing to hand downstream and may not launch,
    blocks in :meth:`wait_for_capacity` on the outstanding tasks of ALL operators until one
    finishes (progress: tasks never depend on downstream operators, so every outstanding task
    eventually frees its CPUs; an idle operator is exempt from memory budgets and caps);
  * **CPU / GPU**: the sum over operators of running tasks x per-task resources stays within the
    limits (default: the cluster's CPUs / GPUs; actor-pool operators hold theirs in actors);
  * **object-store memory**: an operator's usage is its outstanding tasks x the running mean of
    its observed output size; its budget is ``reservation_ratio * limit / #ops`` (reserved) plus
    whatever the shared remainder is not used by the other operators' excess over their own
    reservations -- a slow downstream operator keeps its reserved share even when an upstream
    producer is flooding the store;
  * **concurrency caps**: ``map_batches(concurrency=N)`` on task-pool operators.
Per-operator counters (tasks, peak concurrency, times backpressured, output bytes) feed
``Dataset.stats()``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional


@dataclass
class ExecutionResources:
    cpu: Optional[float] = None
    gpu: Optional[float] = None
    object_store_memory: Optional[float] = None

    @classmethod
    def for_limits(cls, cpu=None, gpu=None, object_store_memory=None) -> "ExecutionResources":
        return cls(cpu, gpu, object_store_memory)

    def add(self, o: "ExecutionResources") -> "ExecutionResources":
        f = lambda a, b: (a or 0.0) + (b or 0.0)  # noqa: E731
        return ExecutionResources(f(self.cpu, o.cpu), f(self.gpu, o.gpu),
                                  f(self.object_store_memory, o.object_store_memory))

    def _map2(self, o: "ExecutionResources", f) -> "ExecutionResources":
        return ExecutionResources(f(self.cpu, o.cpu), f(self.gpu, o.gpu),
                                  f(self.object_store_memory, o.object_store_memory))

    def subtract(self, o: "ExecutionResources") -> "ExecutionResources":
        return self._map2(o, lambda a, b: (a or 0.0) - (b or 0.0))

    def min(self, o: "ExecutionResources") -> "ExecutionResources":
        """Per resource the smaller value (None = unlimited on that side)."""
        return self._map2(o, lambda a, b: b if a is None else a if b is None else min(a, b))

    def max(self, o: "ExecutionResources") -> "ExecutionResources":
        return self._map2(o, lambda a, b: None if a is None or b is None else max(a, b))

    @classmethod
    def zero(cls) -> "ExecutionResources":
        return cls(0.0, 0.0, 0.0)

    def is_zero(self) -> bool:
        return not (self.cpu or self.gpu or self.object_store_memory)

    def is_non_negative(self) -> bool:
        return all((v or 0.0) >= 0 for v in (self.cpu, self.gpu, self.object_store_memory))

    def copy(self) -> "ExecutionResources":
        return ExecutionResources(self.cpu, self.gpu, self.object_store_memory)

    def satisfies_limit(self, limit: "ExecutionResources") -> bool:
        for mine, lim in ((self.cpu, limit.cpu), (self.gpu, limit.gpu),
                          (self.object_store_memory, limit.object_store_memory)):
            if lim is not None and (mine or 0.0) > lim + 1e-9:
                return False
        return True


class OpState:
    def __init__(self, name: str, cpu: float = 0.0, gpu: float = 0.0, concurrency_cap: Optional[int] = None):
        self.name = name
        self.cpu, self.gpu = float(cpu), float(gpu)
        self.concurrency_cap = concurrency_cap
        self.outstanding: List = []  # metadata refs of submitted, not yet finished tasks
        self.tasks = 0
        self.finished = 0
        self.out_bytes = 0
        self.out_rows = 0
        self.peak_running = 0
        self.backpressured = 0

    @property
    def running(self) -> int:
        return len(self.outstanding)

    def est_output_bytes(self) -> float:
        return self.out_bytes / self.finished if self.finished else 0.0

    def memory_usage(self) -> float:
        return self.running * self.est_output_bytes()

    def stats(self) -> Dict:
        return {"name": self.name, "tasks": self.tasks, "peak_running": self.peak_running,
                "backpressured": self.backpressured, "output_bytes": self.out_bytes, "output_rows": self.out_rows}


class BackpressurePolicy:
    def can_submit(self, rm: "ResourceManager", op: OpState) -> bool:  # pragma: no cover - interface
        raise NotImplementedError


class ConcurrencyCapBackpressurePolicy(BackpressurePolicy):
    def can_submit(self, rm, op):
        return op.concurrency_cap is None or op.running < op.concurrency_cap


class ResourceBudgetBackpressurePolicy(BackpressurePolicy):
    def can_submit(self, rm, op):
        lim = rm.limits
        if not rm._compute_fits(op):
            return False
        if lim.object_store_memory is not None:
            est = op.est_output_bytes()
            if est and op.memory_usage() + est > rm.op_memory_budget(op):
                return False
        return True


class ResourceManager:
    def __init__(self, limits: ExecutionResources, reservation_ratio: float = 0.5,
                 policies: Optional[List[BackpressurePolicy]] = None):
        self.limits = limits
        self.reservation_ratio = reservation_ratio
        self.ops: List[OpState] = []
        self.policies = policies if policies is not None else [ConcurrencyCapBackpressurePolicy(),
                                                                ResourceBudgetBackpressurePolicy()]
        self.peak_cpu = 0.0
        self.peak_gpu = 0.0

    @classmethod
    def from_context(cls, ctx) -> "ResourceManager":
        from ..._private.worker import cluster_resources, is_initialized

        opts = ctx.execution_options
        user = opts.resource_limits
        cr = cluster_resources() if is_initialized() else {}
        cpu = user.cpu if user.cpu is not None else cr.get("CPU")
        gpu = user.gpu if user.gpu is not None else cr.get("GPU", 0.0)
        mem = user.object_store_memory
        if mem is None and cr.get("object_store_memory"):
            mem = cr["object_store_memory"] * ctx.object_store_memory_limit_fraction
        return cls(ExecutionResources(cpu, gpu, mem), ctx.op_resource_reservation_ratio)

    # ------------------------------------------------------------------ registry
    def register(self, name: str, cpu: float = 0.0, gpu: float = 0.0, concurrency_cap: Optional[int] = None) -> OpState:
        op = OpState(name, cpu, gpu, concurrency_cap)
        self.ops.append(op)
        return op

    def on_submit(self, op: OpState, meta_ref):
        op.outstanding.append(meta_ref)
        op.tasks += 1
        op.peak_running = max(op.peak_running, op.running)
        u = self.global_usage()
        self.peak_cpu = max(self.peak_cpu, u.cpu or 0.0)
        self.peak_gpu = max(self.peak_gpu, u.gpu or 0.0)

    def on_finish(self, op: OpState, meta_ref):
        """The streaming executor saw ``meta_ref`` complete: retire it without another wait."""
        from ..._private.worker import get

        try:
            op.outstanding.remove(meta_ref)
        except ValueError:
            return
        try:
            m = get(meta_ref)
            op.out_bytes += int(m.get("size_bytes", 0))
            op.out_rows += int(m.get("num_rows", 0))
        except Exception:  # a failed task: its error surfaces where the block is consumed
            pass
        op.finished += 1

    # ------------------------------------------------------------------ accounting
    def poll(self):
        """Retire finished tasks (non-blocking) and fold their output sizes into the estimates."""
        from ..._private.worker import get, wait

        for op in self.ops:
            if not op.outstanding:
                continue
            ready, rest = wait(op.outstanding, num_returns=len(op.outstanding), timeout=0)
            if ready:
                for m in get(ready):
                    op.out_bytes += int(m.get("size_bytes", 0))
                    op.out_rows += int(m.get("num_rows", 0))
                    op.finished += 1
                op.outstanding = list(rest)

    def global_usage(self) -> ExecutionResources:
        cpu = sum(op.running * op.cpu for op in self.ops)
        gpu = sum(op.running * op.gpu for op in self.ops)
        mem = sum(op.memory_usage() for op in self.ops)
        return ExecutionResources(cpu, gpu, mem)

    def op_memory_budget(self, op: OpState) -> float:
        lim = self.limits.object_store_memory
        if lim is None:
            return float("inf")
        n = max(1, len(self.ops))
        reserved = lim * self.reservation_ratio / n
        shared = lim * (1.0 - self.reservation_ratio)
        for o in self.ops:
            if o is not op:
                shared -= max(0.0, o.memory_usage() - reserved)
        return reserved + max(0.0, shared)

    def _compute_fits(self, op: OpState) -> bool:
        lim, u = self.limits, self.global_usage()
        if lim.cpu is not None and op.cpu and u.cpu + op.cpu > lim.cpu + 1e-9:
            return False
        if lim.gpu is not None and op.gpu and u.gpu + op.gpu > lim.gpu + 1e-9:
            return False
        return True

    def can_submit(self, op: OpState, poll: bool = True) -> bool:
        """``poll=False``: the caller (the streaming executor) retires finished tasks itself."""
        if poll:
            self.poll()
        if op.running == 0:
            # liveness: an idle operator may always run one task when the CPUs/GPUs allow it (or
            # when nothing at all is running); memory budgets and caps never block it
            ok = self._compute_fits(op) or not any(o.outstanding for o in self.ops)
            if not ok:
                op.backpressured += 1
            return ok
        ok = all(p.can_submit(self, op) for p in self.policies)
        if not ok:
            op.backpressured += 1
        return ok

    def wait_for_capacity(self, op: OpState):
        """Block until ``op`` may submit: waits on the outstanding tasks of every operator."""
        from ..._private.worker import wait

        while not self.can_submit(op):
            refs = [r for o in self.ops for r in o.outstanding]
            if not refs:
                return
            wait(refs, num_returns=1)

    def stats(self) -> Dict:
        return {"limits": {"cpu": self.limits.cpu, "gpu": self.limits.gpu,
                           "object_store_memory": self.limits.object_store_memory},
                "peak_cpu": self.peak_cpu, "peak_gpu": self.peak_gpu, "ops": [op.stats() for op in self.ops]}
