"""Fault-tolerant management of a set of remote actors (reference:
``rllib/utils/actor_manager.py`` -- ``FaultTolerantActorManager:193``, ``foreach_actor:563``,
``probe_unhealthy_actors:792``).

Every call fans out to the HEALTHY actors only; an actor whose call fails with an actor-death
error (or, when ``mark_unhealthy_on_error``, any error) is marked unhealthy instead of failing
the whole call, and ``probe_unhealthy_actors`` pings those later: the ones that answer (restarted
by the runtime, or replaced through ``replace_actor``) become healthy again.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterator, List, Optional, Union


class ResultOrError:
    def __init__(self, result: Any = None, error: Optional[BaseException] = None):
        self._result = result
        self._error = error

    @property
    def ok(self) -> bool:
        return self._error is None

    def get(self):
        return self._result if self.ok else self._error


@dataclass
class CallResult:
    actor_id: int
    result_or_error: ResultOrError
    tag: Optional[str] = None

    @property
    def ok(self) -> bool:
        return self.result_or_error.ok

    def get(self):
        return self.result_or_error.get()


class RemoteCallResults:
    """Results of one fan-out, one ``CallResult`` per actor called."""

    def __init__(self):
        self.result_or_errors: List[CallResult] = []

    def add_result(self, actor_id: int, result_or_error: ResultOrError, tag: Optional[str] = None):
        self.result_or_errors.append(CallResult(actor_id, result_or_error, tag))

    def __iter__(self) -> Iterator[CallResult]:
        return iter(list(self.result_or_errors))

    def __len__(self):
        return len(self.result_or_errors)

    def ignore_errors(self) -> Iterator[CallResult]:
        return iter([r for r in self.result_or_errors if r.ok])

    def ignore_ray_errors(self) -> Iterator[CallResult]:
        return iter([r for r in self.result_or_errors if r.ok or not is_actor_failure(r.get())])


def is_actor_failure(err: BaseException) -> bool:
    """True for the errors that mean the actor (process) is gone or unreachable, as opposed to an
    exception raised by the method itself."""
    from ... import exceptions as exc

    kinds = tuple(k for k in (getattr(exc, "RayActorError", None), getattr(exc, "ActorDiedError", None),
                              getattr(exc, "ActorUnavailableError", None), getattr(exc, "OwnerDiedError", None),
                              getattr(exc, "WorkerCrashedError", None)) if k is not None)
    return isinstance(err, kinds)


class FaultTolerantActorManager:
    """A set of actors addressed by integer ids, each with a health flag.

    ``foreach_actor(func, ...)``: ``func`` is a method name, or a callable applied to the actor
    (through its ``apply`` method: ``FaultAwareApply``), or a list with one per actor.
    """

    def __init__(self, actors: Optional[List[Any]] = None, max_remote_requests_in_flight_per_actor: int = 2,
                 init_id: int = 0, mark_unhealthy_on_error: bool = False):
        self._next_id = init_id
        self._actors: Dict[int, Any] = {}
        self._healthy: Dict[int, bool] = {}
        self._restarts: Dict[int, int] = {}
        self.max_in_flight = max_remote_requests_in_flight_per_actor
        self.mark_unhealthy_on_error = mark_unhealthy_on_error
        self.add_actors(actors or [])

    # ------------------------------------------------------------------ membership
    def add_actors(self, actors: List[Any]) -> List[int]:
        ids = []
        for a in actors:
            i = self._next_id
            self._next_id += 1
            self._actors[i] = a
            self._healthy[i] = True
            self._restarts[i] = 0
            ids.append(i)
        return ids

    def remove_actor(self, actor_id: int):
        self._healthy.pop(actor_id, None)
        self._restarts.pop(actor_id, None)
        return self._actors.pop(actor_id, None)

    def replace_actor(self, actor_id: int, actor) -> None:
        """A recreated actor takes the failed one's id (and stays unhealthy until probed)."""
        self._actors[actor_id] = actor
        self._restarts[actor_id] = self._restarts.get(actor_id, 0) + 1

    def actor_ids(self) -> List[int]:
        return list(self._actors)

    def healthy_actor_ids(self) -> List[int]:
        return [i for i in self._actors if self._healthy.get(i)]

    def unhealthy_actor_ids(self) -> List[int]:
        return [i for i in self._actors if not self._healthy.get(i)]

    def num_actors(self) -> int:
        return len(self._actors)

    def num_healthy_actors(self) -> int:
        return len(self.healthy_actor_ids())

    def total_num_restarts(self) -> int:
        return sum(self._restarts.values())

    def num_restarts(self, actor_id: int) -> int:
        return self._restarts.get(actor_id, 0)

    def is_actor_healthy(self, actor_id: int) -> bool:
        return bool(self._healthy.get(actor_id))

    def set_actor_state(self, actor_id: int, healthy: bool) -> None:
        if actor_id in self._actors:
            self._healthy[actor_id] = bool(healthy)

    def actors(self) -> Dict[int, Any]:
        return dict(self._actors)

    def healthy_actors(self) -> List[Any]:
        return [self._actors[i] for i in self.healthy_actor_ids()]

    def clear(self):
        from ..._private.worker import kill

        for a in self._actors.values():
            try:
                kill(a)
            except Exception:
                pass
        self._actors.clear()
        self._healthy.clear()
        self._restarts.clear()

    # ------------------------------------------------------------------ calls
    def _submit(self, actor, func, args, kwargs):
        if isinstance(func, str):
            return getattr(actor, func).remote(*args, **kwargs)
        return actor.apply.remote(func, *args, **kwargs)

    def foreach_actor(self, func: Union[str, Callable, List], *args, healthy_only: bool = True,
                      remote_actor_ids: Optional[List[int]] = None, timeout_seconds: Optional[float] = None,
                      return_obj_refs: bool = False, mark_healthy: bool = False, **kwargs) -> RemoteCallResults:
        from ..._private.worker import get, wait

        ids = list(remote_actor_ids) if remote_actor_ids is not None else self.actor_ids()
        if isinstance(func, list):
            # one callable per actor id: filter the (id, func) pairs together, so a skipped
            # unhealthy actor does not shift the remaining actors onto each other's functions
            if len(func) != len(ids):
                raise ValueError(f"foreach_actor got {len(func)} functions for {len(ids)} actors")
            pairs = list(zip(ids, func))
        else:
            pairs = [(i, func) for i in ids]
        if healthy_only:
            pairs = [(i, f) for i, f in pairs if self._healthy.get(i)]
        ids = [i for i, _ in pairs]
        funcs = [f for _, f in pairs]
        refs = {}
        out = RemoteCallResults()
        for i, f in zip(ids, funcs):
            try:
                refs[self._submit(self._actors[i], f, args, kwargs)] = i
            except Exception as e:  # noqa  (a handle that cannot even submit is a dead actor)
                self._on_error(i, e)
                out.add_result(i, ResultOrError(error=e))
        if return_obj_refs:
            for ref, i in refs.items():
                out.add_result(i, ResultOrError(result=ref))
            return out
        pending = list(refs)
        ready = pending
        if timeout_seconds is not None and pending:
            ready, not_ready = wait(pending, num_returns=len(pending), timeout=timeout_seconds)
            for ref in not_ready:
                i = refs[ref]
                err = TimeoutError(f"actor {i} did not answer within {timeout_seconds}s")
                self._on_error(i, err, force=True)
                out.add_result(i, ResultOrError(error=err))
        for ref in ready:
            i = refs[ref]
            try:
                res = get(ref)
            except Exception as e:  # noqa
                self._on_error(i, e)
                out.add_result(i, ResultOrError(error=e))
                continue
            if mark_healthy:
                self._healthy[i] = True
            out.add_result(i, ResultOrError(result=res))
        return out

    def _on_error(self, actor_id: int, err: BaseException, force: bool = False):
        if force or self.mark_unhealthy_on_error or is_actor_failure(err):
            self._healthy[actor_id] = False

    def probe_unhealthy_actors(self, timeout_seconds: Optional[float] = None,
                               mark_healthy: bool = False) -> List[int]:
        """Ping every unhealthy actor; return the ids that answered (marked healthy when
        ``mark_healthy``: the caller may want to restore their state first)."""
        ids = self.unhealthy_actor_ids()
        if not ids:
            return []
        res = self.foreach_actor("ping", healthy_only=False, remote_actor_ids=ids, timeout_seconds=timeout_seconds,
                                 mark_healthy=mark_healthy)
        return [r.actor_id for r in res if r.ok]


class FaultAwareApply:
    """Mixin for managed actors: ``ping`` for health probes, ``apply(fn)`` for callables."""

    def ping(self) -> str:
        return "pong"

    def apply(self, func, *args, **kwargs):
        return func(self, *args, **kwargs)
