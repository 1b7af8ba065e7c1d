"""Node memory monitor + worker-killing policy (the OOM killer).

Reference: ``src/ray/common/memory_monitor.cc`` (periodic usage sampling against
``memory_usage_threshold``) and ``src/ray/raylet/worker_killing_policy*.cc`` (pick a victim when
above it). Here the head's event loop calls :meth:`MemoryMonitor.poll` every
``memory_monitor_refresh_ms``; above the threshold ONE worker is killed and no further kill
happens until that worker is gone and a cool-down has passed (so a burst of samples does not
empty the node). Victim order: retriable normal tasks before non-retriable ones before actors,
newest first within a class (LIFO — the most recently started work has made the least progress).
The killed task fails with ``OutOfMemoryError`` once its retries are used up.

Usage source: cgroup v2 ``memory.current/memory.max`` when the process is limited by one, else
``psutil.virtual_memory()``; ``memory_monitor_usage_file`` (system config) overrides it with a
fraction read from a file (test hook, like the reference's fake-memory tests).
"""
from __future__ import annotations

import os
import time
from typing import Optional


def _cgroup_fraction() -> Optional[float]:
    try:
        with open("/sys/fs/cgroup/memory.max") as f:
            mx = f.read().strip()
        if mx == "max":
            return None
        with open("/sys/fs/cgroup/memory.current") as f:
            cur = int(f.read().strip())
        inactive = 0
        with open("/sys/fs/cgroup/memory.stat") as f:  # reclaimable page cache is not pressure
            for line in f:
                if line.startswith("inactive_file "):
                    inactive = int(line.split()[1])
                    break
        return max(0, cur - inactive) / max(1, int(mx))
    except (OSError, ValueError):
        return None


def system_memory_fraction() -> float:
    frac = _cgroup_fraction()
    if frac is not None:
        return frac
    import psutil

    vm = psutil.virtual_memory()
    return (vm.total - vm.available) / max(1, vm.total)


class MemoryMonitor:
    def __init__(self, config: dict):
        env_thr = os.environ.get("RAY_memory_usage_threshold")
        self.threshold = float(config.get("memory_usage_threshold", env_thr if env_thr else 0.95))
        env_ms = os.environ.get("RAY_memory_monitor_refresh_ms")
        self.refresh_s = float(config.get("memory_monitor_refresh_ms", env_ms if env_ms else 250)) / 1000.0
        self.usage_file = config.get("memory_monitor_usage_file")
        self.enabled = self.refresh_s > 0 and 0 < self.threshold < 1
        self._next = 0.0
        self._victim = None
        self._cooldown_until = 0.0
        self.num_killed = 0
        self.last_usage = 0.0

    def usage(self) -> float:
        if self.usage_file:
            try:
                with open(self.usage_file) as f:
                    return float(f.read().strip() or 0.0)
            except (OSError, ValueError):
                return 0.0
        return system_memory_fraction()

    @staticmethod
    def _rank(w):
        ts = w.task
        started = (ts.times.get("start", 0.0) if ts is not None else 0.0) or 0.0
        if w.actor is not None:
            cls = 2
        elif ts is not None and ts.retries_left != 0:
            cls = 0
        else:
            cls = 1
        return (cls, -started)

    def poll(self, head) -> None:
        """Called from the head loop (head lock NOT held); kills at most one worker."""
        if not self.enabled:
            return
        now = time.time()
        if now < self._next:
            return
        self._next = now + self.refresh_s
        if self._victim is not None:
            if not self._victim.dead:
                return
            self._victim = None
            self._cooldown_until = now + 2 * self.refresh_s
        if now < self._cooldown_until:
            return
        self.last_usage = u = self.usage()
        if u < self.threshold:
            return
        with head.lock:
            cands = [w for w in head.workers.values()
                     if not w.dead and (w.task is not None or w.actor is not None) and w.state != "starting"]
            if not cands:
                return
            victim = min(cands, key=self._rank)
            victim.oom_killed = (u, self.threshold)
            self._victim = victim
            self.num_killed += 1
            what = (f"actor {victim.actor.aid.hex()[:12]}" if victim.actor is not None
                    else f"task {victim.task.spec.get('name')}")
            head._oom_log.append((now, victim.pid, what, u))
            head._kill_worker(victim)
