"""Memory monitor / OOM killer (reference: python/ray/tests/test_memory_pressure.py), driven by
the ``memory_monitor_usage_file`` hook instead of really exhausting host memory."""
import time

import pytest

import ray_community_amd as ray
from ray_community_amd.exceptions import OutOfMemoryError


def _init(tmp_path, usage="0.1"):
    f = tmp_path / "usage"
    f.write_text(usage)
    ray.init(num_cpus=2, _system_config={"memory_usage_threshold": 0.9, "memory_monitor_refresh_ms": 20,
                                         "memory_monitor_usage_file": str(f)})
    return f


def test_task_killed_raises_oom(shutdown_only, tmp_path):
    f = _init(tmp_path)

    @ray.remote(max_retries=0)
    def hog(marker):
        import pathlib

        pathlib.Path(marker).write_text("started")
        time.sleep(60)

    marker = tmp_path / "m"
    ref = hog.remote(str(marker))
    deadline = time.time() + 30
    while not marker.exists() and time.time() < deadline:
        time.sleep(0.02)
    f.write_text("0.97")
    with pytest.raises(OutOfMemoryError) as ei:
        ray.get(ref, timeout=30)
    assert "memory monitor" in str(ei.value)


def test_oom_killed_task_is_retried(shutdown_only, tmp_path):
    f = _init(tmp_path)

    @ray.remote(max_retries=2)
    def attempt(marker):
        import pathlib

        p = pathlib.Path(marker)
        n = int(p.read_text()) if p.exists() else 0
        p.write_text(str(n + 1))
        if n == 0:
            time.sleep(60)  # first attempt: killed under pressure
        return n

    marker = tmp_path / "n"
    ref = attempt.remote(str(marker))
    deadline = time.time() + 30
    while not marker.exists() and time.time() < deadline:
        time.sleep(0.02)
    f.write_text("0.97")
    while (marker.read_text() if marker.exists() else "0") == "1" and time.time() < deadline:
        time.sleep(0.02)
    f.write_text("0.1")  # pressure relieved: the retry runs to completion
    assert ray.get(ref, timeout=30) >= 1


def test_victim_is_newest_retriable_task(shutdown_only, tmp_path):
    from ray_community_amd._private.memory_monitor import MemoryMonitor

    class TS:
        def __init__(self, start, retries):
            self.times = {"start": start}
            self.retries_left = retries

    class W:
        def __init__(self, ts=None, actor=None):
            self.task, self.actor = ts, actor

    old_retriable, new_retriable = W(TS(1.0, 3)), W(TS(2.0, 3))
    non_retriable, actor = W(TS(3.0, 0)), W(None, actor=object())
    ws = [actor, non_retriable, old_retriable, new_retriable]
    assert min(ws, key=MemoryMonitor._rank) is new_retriable
    assert min([actor, non_retriable], key=MemoryMonitor._rank) is non_retriable
