"""Deployment handles + router (reference: ``serve/handle.py``, ``_private/router.py``,
``_private/replica_scheduler/pow_2_scheduler.py``).

Replica scheduling (reference ``pow_2_scheduler.py:49,92-103,294,445``): power of two choices over
replica queue lengths that the router PROBES (``get_num_ongoing`` RPCs, answers cached for a short
TTL, probe deadline backed off while replicas answer slowly), so N callers in N processes see the
load the others put on a replica instead of each believing it idle; a replica is never sent more
than ``max_ongoing_requests`` (requests wait on the caller when every replica is full).
Candidates come in locality tiers: for a request that carries a GPU tensor, replicas on the SAME
physical GPU of the caller's node first (the tensor needs no xGMI copy), then replicas on the
caller's node, then all.
"""
from __future__ import annotations

import asyncio
import collections
import concurrent.futures
import random
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

from .._private.core_worker import ObjectRef, ObjectRefGenerator


class _HandleSpec:
    """Placeholder for a bound deployment inside another deployment's init args."""

    def __init__(self, app_name, deployment_name):
        self.app_name = app_name
        self.deployment_name = deployment_name


def _resolve_handle_args(args, kwargs):
    def conv(x):
        if isinstance(x, _HandleSpec):
            return DeploymentHandle(x.deployment_name, x.app_name)
        if isinstance(x, DeploymentResponse):
            return x._to_object_ref_sync()
        return x

    return tuple(conv(a) for a in args), {k: conv(v) for k, v in kwargs.items()}


def physical_gpu_ids(indices) -> List[int]:
    """Physical device ids (the node's full GPU list) of this process's HIP device indices: ROCm
    applies ``ROCR_VISIBLE_DEVICES`` first and ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``
    indexes into what it left (``_private/head.py::worker_hip_visible_devices``)."""
    import os

    def parse(var):
        v = os.environ.get(var)
        return [int(x) for x in v.split(",") if x.strip()] if v else None

    rocr = parse("ROCR_VISIBLE_DEVICES")
    hip = parse("HIP_VISIBLE_DEVICES") or parse("CUDA_VISIBLE_DEVICES")
    out = []
    for i in indices:
        j = hip[i] if hip is not None and i < len(hip) else i
        out.append(rocr[j] if rocr is not None and j < len(rocr) else j)
    return out


def _request_gpu(args, kwargs) -> Optional[int]:
    """Physical GPU of the first device tensor among the request's top-level arguments."""
    for v in list(args) + list(kwargs.values()):
        dev = getattr(v, "device", None)
        if dev is not None and getattr(dev, "type", None) == "cuda":
            idx = dev.index
            if idx is None:
                try:
                    import torch

                    idx = torch.cuda.current_device()
                except Exception:
                    idx = 0
            return physical_gpu_ids([idx])[0]
    return None


_NODE_ID: List[Optional[str]] = []


def _caller_node() -> Optional[str]:
    if not _NODE_ID:
        try:
            from .._private.worker import get_runtime_context

            _NODE_ID.append(get_runtime_context().get_node_id())
        except Exception:
            return None
    return _NODE_ID[0]


class _Router:
    """Per-(app, deployment) request router living in the caller's process.

    ``submit`` never blocks: a request goes straight to a replica chosen by power-of-two-choices
    when one has spare capacity, otherwise it waits in a local FIFO that is drained as replies
    come back (or new replicas appear). The queue length is reported to the controller so the
    autoscaler sees demand that has not reached any replica yet."""

    _routers: Dict[Tuple[str, str], "_Router"] = {}
    _lock = threading.Lock()

    def __init__(self, app, dep):
        self.app = app
        self.dep = dep
        self.id = f"{id(self):x}-{random.getrandbits(32):08x}"
        self.replicas: List[Tuple[str, Any]] = []
        self.inflight: Dict[str, int] = {}
        self.max_ongoing = 5
        self.max_queued = -1  # max_queued_requests (-1: unbounded)
        self.last_refresh = 0.0
        self.cv = threading.Condition()
        self.queue: "collections.deque" = collections.deque()
        self._reported = 0
        self._drainer: Optional[threading.Thread] = None
        self.locations: Dict[str, Dict] = {}
        # probed load of OTHER callers: tag -> (requests not from this router, probe time). A
        # probe's answer counts this router's own requests too; they are known exactly
        # (``inflight``) and taken out at the upper bound of what the replica could have counted,
        # so the estimate is own in-flight + others. Entries older than queue_len_ttl_s fall
        # back to the own view alone.
        self.qlen: Dict[str, Tuple[int, float]] = {}
        self.sent: Dict[str, int] = {}
        self.probing: Dict[str, float] = {}
        self.queue_len_ttl_s = 0.5
        self.probe_deadline_s = 0.05
        self.stats = {"probes": 0, "probe_timeouts": 0, "picks": 0, "local_gpu_picks": 0, "local_node_picks": 0}

    @classmethod
    def get(cls, app, dep):
        with cls._lock:
            r = cls._routers.get((app, dep))
            if r is None:
                r = _Router(app, dep)
                cls._routers[(app, dep)] = r
            return r

    def _refresh(self, force=False, period=2.0):
        now = time.time()
        if not force and self.replicas and now - self.last_refresh < period:
            return
        from .api import _get_controller
        from .._private.worker import get

        info = get(_get_controller().get_replicas.remote(self.app, self.dep))
        self.last_refresh = now
        if info is None:
            raise RuntimeError(f"Deployment {self.dep} of app {self.app} does not exist")
        self._apply(info)
        self._ensure_listener()

    def _ensure_listener(self):
        """One daemon thread per router long-polls the controller for replica-set changes, so
        scale-ups, replacements and removals reach routing right away instead of at the next
        periodic refresh (reference: the router's LongPollClient on the deployment's targets)."""
        if getattr(self, "_listener", None) is not None and self._listener.is_alive():
            return
        self._listener = threading.Thread(target=self._listen_loop, name=f"serve-router-{self.dep}", daemon=True)
        self._listener.start()

    def _listen_loop(self):
        from .._private import worker as w
        from .api import _get_controller

        known = getattr(self, "_members", -1)
        # exits with the session, with the deployment, or when serve.shutdown() dropped this router
        while w.is_initialized() and _Router._routers.get((self.app, self.dep)) is self:
            try:
                info = w.get(_get_controller().listen_replicas.remote(self.app, self.dep, known, 10.0),
                             timeout=30)
            except Exception:  # controller restarting / shutting down
                if not w.is_initialized():
                    return
                time.sleep(1.0)
                continue
            if info is None:  # deployment deleted
                return
            if info.get("unchanged"):
                continue
            known = info.get("members", known)
            self._apply(info)
            self.last_refresh = time.time()

    def _apply(self, info):
        self._members = info.get("members", -1)
        with self.cv:
            self.replicas = info["replicas"]
            self.max_ongoing = info["max_ongoing_requests"]
            self.max_queued = int(info.get("max_queued_requests", -1))
            self.locations = dict(info.get("locations") or {})
            live = {t for t, _ in self.replicas}
            for d in (self.qlen, self.sent, self.probing):
                for tag in list(d):
                    if tag not in live:
                        d.pop(tag)
            for tag in live:
                self.inflight.setdefault(tag, 0)
            for tag in list(self.inflight):
                if tag not in live:
                    self.inflight.pop(tag)

    # ------------------------------------------------------------------ scheduling
    def _load_locked(self, tag: str, now: float) -> int:
        """Best estimate of ``tag``'s queue length: its last probe (fresh) plus what this router
        sent it since, never below this router's own in-flight requests to it."""
        own = self.inflight.get(tag, 0)
        c = self.qlen.get(tag)
        if c is None or now - c[1] > self.queue_len_ttl_s:
            self._probe_locked(tag, now)
            return own
        return own + c[0]

    def _probe_locked(self, tag: str, now: float):
        t0 = self.probing.get(tag)
        if t0 is not None:
            if now - t0 < self.probe_deadline_s:
                return
            # no answer within the deadline: back off (reference: queue_len_response_deadline_s)
            self.stats["probe_timeouts"] += 1
            self.probe_deadline_s = min(1.0, self.probe_deadline_s * 2)
        actor = next((a for t, a in self.replicas if t == tag), None)
        if actor is None:
            return
        self.probing[tag] = now
        sent_at = self.sent.get(tag, 0)
        own_at = self.inflight.get(tag, 0)
        self.stats["probes"] += 1
        try:
            ref = actor.get_num_ongoing.remote()
        except Exception:  # noqa  (dead handle: routing drops it at the next refresh)
            self.probing.pop(tag, None)
            return

        def on_done(f, tag=tag, sent_at=sent_at, own_at=own_at, t_issue=now):
            try:
                n = int(f.result())
            except Exception:  # noqa
                with self.cv:
                    self.probing.pop(tag, None)
                return
            with self.cv:
                self.probing.pop(tag, None)
                mine = own_at + self.sent.get(tag, 0) - sent_at  # most of ours it could have seen
                self.qlen[tag] = (max(0, n - mine), time.time())
                if time.time() - t_issue < self.probe_deadline_s / 2:
                    self.probe_deadline_s = max(0.05, self.probe_deadline_s / 2)
                self._drain_locked()
                self.cv.notify_all()

        ref.future().add_done_callback(on_done)

    def _ensure_fresh(self, limit: int = 4):
        """Before scheduling: probe (up to ``limit`` random) replicas whose queue length is stale and
        wait for the answers up to the probe deadline -- a cold router would otherwise place its
        first requests blind (reference: the scheduler awaits its probes with a deadline)."""
        now = time.time()
        with self.cv:
            stale = [t for t, _ in self.replicas
                     if t not in self.qlen or now - self.qlen[t][1] > self.queue_len_ttl_s]
            if not stale:
                return
            if len(stale) > limit:
                stale = random.sample(stale, limit)
            for t in stale:
                self._probe_locked(t, now)
            deadline = now + self.probe_deadline_s
            while any(t in self.probing for t in stale):
                rem = deadline - time.time()
                if rem <= 0:
                    return
                self.cv.wait(rem)

    def _tiers_locked(self, gpu: Optional[int]):
        live = self.replicas
        if not self.locations:
            return [live]
        node = _caller_node()
        tiers = []
        if node is not None:
            same_node = [r for r in live if (self.locations.get(r[0]) or {}).get("node_id") == node]
            if gpu is not None:
                same_gpu = [r for r in same_node if gpu in ((self.locations.get(r[0]) or {}).get("gpus") or ())]
                if same_gpu:
                    tiers.append(same_gpu)
            if same_node:
                tiers.append(same_node)
        tiers.append(live)
        return tiers

    def _pick_locked(self, gpu: Optional[int] = None):
        now = time.time()
        for ti, tier in enumerate(self._tiers_locked(gpu)):
            cands = [r for r in tier if self.inflight.get(r[0], 0) < self.max_ongoing]
            if not cands:
                continue
            pick = random.sample(cands, min(2, len(cands)))
            loads = [(self._load_locked(t, now), random.random(), t, a) for t, a in pick]
            load, _, tag, actor = min(loads)
            if load >= self.max_ongoing:
                # both candidates full by their probed queues: re-probe them (an answer drains the
                # queue again) and try the next tier
                for _, _, t, _ in loads:
                    c = self.qlen.get(t)
                    if c is not None and now - c[1] > 0.01:
                        self._probe_locked(t, now)
                continue
            self.inflight[tag] = self.inflight.get(tag, 0) + 1
            self.sent[tag] = self.sent.get(tag, 0) + 1
            self.stats["picks"] += 1
            if self.locations and len(self._tiers_locked(gpu)) > 1 and ti == 0:
                self.stats["local_gpu_picks" if gpu is not None else "local_node_picks"] += 1
            return tag, actor
        return None

    def choose(self, timeout_s=60.0):
        """Blocking pick (used by callers that manage the call themselves)."""
        deadline = time.time() + timeout_s
        while True:
            self._refresh()
            with self.cv:
                got = self._pick_locked()
                if got is not None:
                    return got
                self.cv.wait(0.05)
            if not self.replicas:
                self._refresh(force=True)
            if time.time() > deadline:
                raise TimeoutError(f"no replica of {self.dep} available")

    def submit(self, method: str, args, kwargs, meta, actor_method: str = "handle_request"):
        fut: concurrent.futures.Future = concurrent.futures.Future()
        self._refresh()
        self._ensure_fresh()
        gpu = _request_gpu(args, kwargs) if self.locations else None
        with self.cv:
            item = (actor_method, method, args, kwargs, meta, fut, gpu)
            self.queue.append(item)
            self._drain_locked()
            # backpressure (reference router.py wrap_request_assignment): a request no replica
            # can take right now is dropped once max_queued_requests others are already waiting
            if self.max_queued >= 0 and self.queue and self.queue[-1] is item and len(self.queue) > self.max_queued:
                self.queue.pop()
                from .exceptions import BackPressureError

                fut.set_exception(BackPressureError(num_queued_requests=len(self.queue),
                                                    max_queued_requests=self.max_queued))
            pending = bool(self.queue)
        if pending:
            self._ensure_drainer()
        self._report()
        return fut

    def _drain_locked(self):
        while self.queue:
            got = self._pick_locked(self.queue[0][6])
            if got is None:
                return
            tag, actor = got
            actor_method, method, args, kwargs, meta, fut, _ = self.queue.popleft()
            try:
                if actor_method in ("handle_request", "handle_request_stream"):
                    ref = getattr(actor, actor_method).remote(method, args, kwargs, meta)
                else:
                    ref = getattr(actor, actor_method).remote(*args)
            except Exception as e:  # noqa
                self.inflight[tag] = max(0, self.inflight.get(tag, 0) - 1)
                fut.set_exception(e)
                continue
            done_ref = ref.completed() if isinstance(ref, ObjectRefGenerator) else ref
            done_ref.future().add_done_callback(lambda f, tag=tag: self.done(tag))
            fut.set_result((ref, tag))

    def _ensure_drainer(self):
        with self.cv:
            if self._drainer is not None and self._drainer.is_alive():
                return
            self._drainer = threading.Thread(target=self._drain_loop, daemon=True, name=f"serve-router-{self.dep}")
            self._drainer.start()

    def _drain_loop(self):
        while True:
            with self.cv:
                if not self.queue:
                    self._drainer = None
                    break
                self.cv.wait(0.1)
            try:
                self._refresh(period=0.5)
            except Exception:  # noqa
                pass
            with self.cv:
                self._drain_locked()
            self._report()
        self._report()

    def _report(self):
        n = len(self.queue)
        if n == self._reported:
            return
        self._reported = n
        try:
            from .api import _get_controller

            _get_controller().record_handle_queue.remote(self.app, self.dep, self.id, n)
        except Exception:  # noqa
            pass

    def done(self, tag):
        with self.cv:
            self.inflight[tag] = max(0, self.inflight.get(tag, 0) - 1)
            self._drain_locked()
            self.cv.notify_all()

    def replica_died(self, tag):
        with self.cv:
            self.replicas = [(t, a) for t, a in self.replicas if t != tag]
            self.inflight.pop(tag, None)
        self.last_refresh = 0.0


class DeploymentResponse:
    """Future for one request; the underlying ObjectRef exists once the router assigned a replica."""

    def __init__(self, fut: concurrent.futures.Future):
        self._fut = fut

    @property
    def _ref(self) -> ObjectRef:
        return self._fut.result()[0]

    def result(self, *, timeout_s: Optional[float] = None):
        from .._private.worker import get

        t0 = time.time()
        ref = self._fut.result(timeout=timeout_s)[0]
        rem = None if timeout_s is None else max(0.0, timeout_s - (time.time() - t0))
        return get(ref, timeout=rem)

    async def _await(self):
        ref, _ = await asyncio.wrap_future(self._fut)
        return await ref

    def __await__(self):
        return self._await().__await__()

    async def _to_object_ref(self):
        return (await asyncio.wrap_future(self._fut))[0]

    def _to_object_ref_sync(self):
        return self._ref

    def cancel(self):
        from .._private.worker import cancel

        if not self._fut.done():
            self._fut.cancel()
            return
        cancel(self._ref)


class DeploymentResponseGenerator:
    """Streaming response of ``handle.options(stream=True)``: items arrive one by one as the
    replica's generator yields them (an ObjectRefGenerator underneath)."""

    def __init__(self, fut: concurrent.futures.Future):
        self._fut = fut

    def _gen(self):
        return self._fut.result()[0]

    def __iter__(self):
        from .._private.worker import get

        for ref in self._gen():
            yield get(ref)

    def __aiter__(self):
        async def gen():
            g = (await asyncio.wrap_future(self._fut))[0]
            async for ref in g:
                yield await ref

        return gen()

    def cancel(self):
        from .._private.worker import cancel

        if self._fut.done():
            cancel(self._gen()._main)


class DeploymentHandle:
    def __init__(self, deployment_name: str, app_name: str = "default", *, method_name: str = "__call__",
                 multiplexed_model_id: str = "", stream: bool = False, _grpc_context=None):
        self.deployment_name = deployment_name
        self.app_name = app_name
        self._method = method_name
        self._model_id = multiplexed_model_id
        self._stream = stream
        self._grpc_context = _grpc_context  # set by the gRPC proxy (serve.grpc_util)

    def options(self, *, method_name: Optional[str] = None, multiplexed_model_id: Optional[str] = None,
                stream: Optional[bool] = None, use_new_handle_api=None, _grpc_context=None,
                **kw) -> "DeploymentHandle":
        return DeploymentHandle(self.deployment_name, self.app_name,
                                method_name=method_name or self._method,
                                multiplexed_model_id=self._model_id if multiplexed_model_id is None else
                                multiplexed_model_id,
                                stream=self._stream if stream is None else stream,
                                _grpc_context=self._grpc_context if _grpc_context is None else _grpc_context)

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return self.options(method_name=name)

    def remote(self, *args, **kwargs):
        router = _Router.get(self.app_name, self.deployment_name)
        args = tuple(a._ref if isinstance(a, DeploymentResponse) else a for a in args)
        kwargs = {k: (v._ref if isinstance(v, DeploymentResponse) else v) for k, v in kwargs.items()}
        meta = {"multiplexed_model_id": self._model_id} if self._model_id else {}
        if self._grpc_context is not None:
            meta["grpc_context"] = self._grpc_context
        if self._stream:
            return DeploymentResponseGenerator(router.submit(self._method, args, kwargs, meta,
                                                             actor_method="handle_request_stream"))
        return DeploymentResponse(router.submit(self._method, args, kwargs, meta))

    def __reduce__(self):
        return (DeploymentHandle, (self.deployment_name, self.app_name), {"_method": self._method,
                                                                          "_model_id": self._model_id,
                                                                          "_stream": self._stream})

    def __setstate__(self, st):
        self.__dict__.update(st)

    def __repr__(self):
        return f"DeploymentHandle(deployment='{self.deployment_name}', app='{self.app_name}')"


RayServeHandle = DeploymentHandle
RayServeSyncHandle = DeploymentHandle
