"""ActorPool: spread work over a fixed set of actors (API of ``python/ray/util/actor_pool.py``).

Bookkeeping here is a ticket scheme: every submitted item takes the next ticket number; an
item waits in ``_backlog`` until an actor is idle; ``_running`` maps the object ref that signals
an item's completion to its ticket. Results are handed out either in ticket order (``get_next``)
or in completion order (``get_next_unordered``); a ticket consumed out of order is remembered in
``_taken`` so ordered retrieval skips it.
"""
from __future__ import annotations

import collections
from dataclasses import dataclass, field
from typing import Any, Callable, Deque, Dict, Iterable, List, Optional, Set, Tuple


@dataclass
class _Ticket:
    number: int
    actor: Any
    result: Any                       # what ``fn`` returned (an ObjectRef or a list of them)

    @property
    def signal(self):
        """The ref whose readiness marks this item done."""
        return self.result[0] if isinstance(self.result, list) else self.result


@dataclass
class _State:
    idle: Deque[Any] = field(default_factory=collections.deque)
    backlog: Deque[Tuple[Callable, Any]] = field(default_factory=collections.deque)
    running: Dict[Any, _Ticket] = field(default_factory=dict)      # signal ref -> ticket
    by_number: Dict[int, _Ticket] = field(default_factory=dict)
    taken: Set[int] = field(default_factory=set)
    issued: int = 0
    next_ordered: int = 0


class ActorPool:
    def __init__(self, actors: list):
        self._s = _State(idle=collections.deque(actors))

    # ------------------------------------------------------------------ submission
    def submit(self, fn: Callable[[Any, Any], Any], value):
        """Schedule ``fn(actor, value)`` on an idle actor, or queue it until one frees up."""
        s = self._s
        if not s.idle:
            s.backlog.append((fn, value))
            return
        actor = s.idle.popleft()
        t = _Ticket(s.issued, actor, fn(actor, value))
        s.issued += 1
        s.running[t.signal] = t
        s.by_number[t.number] = t

    def _release(self, actor):
        s = self._s
        s.idle.append(actor)
        if s.backlog:
            fn, value = s.backlog.popleft()
            self.submit(fn, value)

    def _drain_ready(self):
        """Discard already-finished results before a new map() so it starts from a clean slate."""
        while self.has_next():
            try:
                self.get_next_unordered(timeout=0)
            except TimeoutError:
                return

    # ------------------------------------------------------------------ map
    def map(self, fn: Callable[[Any, Any], Any], values: Iterable):
        self._drain_ready()
        for v in values:
            self.submit(fn, v)
        return (self.get_next() for _ in iter(self.has_next, False))

    def map_unordered(self, fn: Callable[[Any, Any], Any], values: Iterable):
        self._drain_ready()
        for v in values:
            self.submit(fn, v)
        return (self.get_next_unordered() for _ in iter(self.has_next, False))

    # ------------------------------------------------------------------ retrieval
    def has_next(self) -> bool:
        return bool(self._s.running)

    def _finish(self, t: _Ticket):
        from .._private.worker import get

        s = self._s
        s.running.pop(t.signal, None)
        s.by_number.pop(t.number, None)
        self._release(t.actor)
        return get(t.result)

    def get_next(self, timeout: Optional[float] = None, ignore_if_timedout: bool = False):
        """The result of the oldest outstanding item (submission order)."""
        from .._private.worker import wait

        s = self._s
        if not self.has_next():
            raise StopIteration("No more results to get")
        while s.next_ordered in s.taken:
            s.taken.discard(s.next_ordered)
            s.next_ordered += 1
        t = s.by_number.get(s.next_ordered)
        if t is None:
            raise ValueError("It is not allowed to call get_next() after get_next_unordered().")
        if timeout is not None:
            ready, _ = wait([t.signal], timeout=timeout)
            if not ready:
                if ignore_if_timedout:  # give up on this item: ordered retrieval moves past it
                    s.next_ordered += 1
                raise TimeoutError("Timed out waiting for result")
        s.next_ordered += 1
        return self._finish(t)

    def get_next_unordered(self, timeout: Optional[float] = None, ignore_if_timedout: bool = False):
        """The result of whichever outstanding item finishes first."""
        from .._private.worker import wait

        s = self._s
        if not self.has_next():
            raise StopIteration("No more results to get")
        ready, _ = wait(list(s.running), num_returns=1, timeout=timeout)
        if not ready:
            raise TimeoutError("Timed out waiting for result")
        t = s.running[ready[0]]
        if t.number >= s.next_ordered:
            s.taken.add(t.number)
        return self._finish(t)

    # ------------------------------------------------------------------ pool membership
    def has_free(self) -> bool:
        return bool(self._s.idle) and not self._s.backlog

    def pop_idle(self):
        return self._s.idle.popleft() if self.has_free() else None

    def push(self, actor):
        s = self._s
        if actor in s.idle or any(t.actor is actor or t.actor == actor for t in s.running.values()):
            raise ValueError("Actor already belongs to current ActorPool")
        self._release(actor)
