"""The algorithm's env runners: one local runner plus N remote runner actors, fault tolerant
(reference: ``rllib/env/env_runner_group.py`` / ``rllib/evaluation/worker_set.py`` WorkerSet over
``FaultTolerantActorManager``, and ``Algorithm.restore_workers``, ``algorithm.py:1429``).

Failure policy (``AlgorithmConfig.fault_tolerance`` / ``env_runners``):
  * default: a failing remote runner fails the call (and ``train()``), as in the reference;
  * ``ignore_env_runner_failures``: the failed runner is marked unhealthy and the iteration goes on
    with the healthy ones (the local runner samples when none is left);
  * ``recreate_failed_env_runners`` (implies ignoring): the failed runner is also replaced by a
    fresh actor with the same ``worker_index`` -- at most ``max_num_env_runner_restarts`` times,
    ``delay_between_env_runner_restarts_s`` after the failure -- and, once it answers a health
    probe, gets the current weights and connector state before it samples again.
More than ``num_consecutive_env_runner_failures_tolerance`` failing calls in a row fail anyway.
"""
from __future__ import annotations

import time
from typing import Any, Dict, List, Optional

from ..utils.actor_manager import FaultTolerantActorManager


class EnvRunnerGroup:
    def __init__(self, runner_cls, runner_config: Dict, algo_config, local_runner, num_remote: int,
                 actor_options: Optional[Dict] = None):
        from ...actor import ActorClass

        self._runner_config = runner_config
        self._cls = ActorClass(runner_cls, dict(actor_options or {})) if num_remote > 0 else None
        self.local = local_runner
        c = algo_config
        self.recreate = bool(getattr(c, "recreate_failed_env_runners", False))
        self.ignore = self.recreate or bool(getattr(c, "ignore_env_runner_failures", False))
        self.max_restarts = int(getattr(c, "max_num_env_runner_restarts", 1000))
        self.delay = float(getattr(c, "delay_between_env_runner_restarts_s", 60.0))
        self.tolerance = int(getattr(c, "num_consecutive_env_runner_failures_tolerance", 100))
        self.probe_timeout = float(getattr(c, "env_runner_health_probe_timeout_s", 30.0))
        self.restore_timeout = float(getattr(c, "env_runner_restore_timeout_s", 1800.0))
        actors = [self._create(i + 1) for i in range(num_remote)]
        self.manager = FaultTolerantActorManager(actors, init_id=1, mark_unhealthy_on_error=self.ignore)
        self._failed_at: Dict[int, float] = {}
        self._consecutive_failures = 0
        self.failures: List[str] = []  # "runner <id>: <error>" of every failure seen

    def _create(self, worker_index: int):
        return self._cls.remote(self._runner_config, worker_index)

    # ------------------------------------------------------------------ views
    def local_env_runner(self):
        return self.local

    local_worker = local_env_runner

    def healthy_env_runners(self) -> List[Any]:
        return self.manager.healthy_actors()

    def healthy_env_runner_ids(self) -> List[int]:
        return self.manager.healthy_actor_ids()

    def num_remote_env_runners(self) -> int:
        return self.manager.num_actors()

    num_remote_workers = num_remote_env_runners

    def num_healthy_remote_env_runners(self) -> int:
        return self.manager.num_healthy_actors()

    num_healthy_remote_workers = num_healthy_remote_env_runners

    def num_remote_env_runner_restarts(self) -> int:
        return self.manager.total_num_restarts()

    # ------------------------------------------------------------------ calls
    def foreach_env_runner(self, func, *args, local_env_runner: bool = False, healthy_only: bool = True,
                           remote_env_runner_ids: Optional[List[int]] = None,
                           timeout_seconds: Optional[float] = None, **kwargs) -> List[Any]:
        """Results of ``func`` (a method name or ``fn(runner)``) on the local runner (if asked)
        and on every healthy remote runner that did not fail; failures follow the group's policy."""
        out = []
        if local_env_runner:
            out.append(getattr(self.local, func)(*args, **kwargs) if isinstance(func, str)
                       else func(self.local, *args, **kwargs))
        if self.manager.num_actors() == 0:
            return out
        res = self.manager.foreach_actor(func, *args, healthy_only=healthy_only,
                                         remote_actor_ids=remote_env_runner_ids, timeout_seconds=timeout_seconds,
                                         **kwargs)
        errors = [r for r in res if not r.ok]
        if errors:
            self._on_failures(errors)
        else:
            self._consecutive_failures = 0
        out += [r.get() for r in res if r.ok]
        return out

    foreach_worker = foreach_env_runner

    def _on_failures(self, errors):
        now = time.time()
        for r in errors:
            self.failures.append(f"runner {r.actor_id}: {type(r.get()).__name__}: {r.get()}")
        if not self.ignore:
            raise errors[0].get()
        self._consecutive_failures += 1
        if self._consecutive_failures > self.tolerance:
            raise RuntimeError(f"{self._consecutive_failures} consecutive env-runner failures (> "
                               f"num_consecutive_env_runner_failures_tolerance={self.tolerance}); last: "
                               f"{self.failures[-1]}") from errors[-1].get()
        for r in errors:
            self.manager.set_actor_state(r.actor_id, False)
            self._failed_at.setdefault(r.actor_id, now)

    def mark_failed(self, actor_id: int, err: BaseException):
        """An async caller (IMPALA) saw ``actor_id`` fail outside ``foreach_env_runner``."""
        from ..utils.actor_manager import CallResult, ResultOrError

        self._on_failures([CallResult(actor_id, ResultOrError(error=err))])

    def actor_id_of(self, actor) -> Optional[int]:
        for i, a in self.manager.actors().items():
            if a is actor:
                return i
        return None

    def probe_unhealthy_env_runners(self) -> List[int]:
        """Replace (``recreate``) failed runners whose restart delay has passed, ping every unhealthy
        one, and return the ids that answered -- still marked unhealthy: the algorithm restores
        their state and then marks them healthy."""
        if not self.manager.unhealthy_actor_ids():
            return []
        from ..._private.worker import kill

        now = time.time()
        if self.recreate:
            for i in self.manager.unhealthy_actor_ids():
                if now - self._failed_at.get(i, 0.0) < self.delay or self.manager.num_restarts(i) >= self.max_restarts:
                    continue
                old = self.manager.actors()[i]
                try:
                    kill(old)
                except Exception:
                    pass
                self.manager.replace_actor(i, self._create(i))
                self._failed_at[i] = now
        return self.manager.probe_unhealthy_actors(timeout_seconds=self.probe_timeout, mark_healthy=False)

    probe_unhealthy_workers = probe_unhealthy_env_runners

    def mark_healthy(self, ids: List[int]):
        for i in ids:
            self.manager.set_actor_state(i, True)
            self._failed_at.pop(i, None)

    def stop(self):
        self.manager.clear()
