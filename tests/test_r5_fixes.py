"""Regression tests for round-5 correctness fixes: wait() remainder cache keeps no strong refs,
per-actor function lists stay paired with their actors, duplicate placement-group names are
rejected, the GPU worker device mask under ROCR_VISIBLE_DEVICES, the atomic session file."""
import gc
import json
import os

import pytest

import ray_community_amd as ray
from ray_community_amd._private.head import worker_hip_visible_devices


def test_wait_remainder_is_released_after_del(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    import numpy as np

    @ray.remote
    def quick():
        return np.zeros(10)

    @ray.remote
    def slow():
        import time

        time.sleep(1.0)
        return np.ones(200_000)

    a, b = quick.remote(), slow.remote()  # task returns: owned by this worker
    ray.get(a)
    ready, rest = ray.wait([a, b], num_returns=1)
    assert len(ready) == 1 and len(rest) == 1
    from ray_community_amd._private.worker import _core

    core = _core()
    assert core._wait_rest is not None and core._wait_rest[0]() is rest
    del rest, b
    gc.collect()
    # the wait() fast-path cache holds the remainder only weakly: dropping it releases the refs
    assert core._wait_rest[0]() is None
    # polling fast path still works on a live remainder
    refs = [ray.put(i) for i in range(5)]
    got = []
    rest = refs
    while rest:
        r, rest = ray.wait(rest)
        got.extend(ray.get(r))
    assert sorted(got) == list(range(5))


def test_foreach_actor_function_list_skips_unhealthy_in_pairs(shutdown_only):
    ray.init(num_cpus=3, include_dashboard=False, log_to_driver=False)
    from ray_community_amd.rllib.utils.actor_manager import FaultAwareApply, FaultTolerantActorManager

    @ray.remote
    class A(FaultAwareApply):
        def __init__(self, name):
            self.name = name

        def who(self):
            return self.name

    mgr = FaultTolerantActorManager([A.remote(n) for n in ("a", "b", "c")])
    ids = mgr.actor_ids()
    mgr.set_actor_state(ids[1], False)
    funcs = [lambda x, t=t: (t, x.who()) for t in ("for-a", "for-b", "for-c")]
    res = mgr.foreach_actor(funcs)
    got = sorted(r.get() for r in res if r.ok)
    assert got == [("for-a", "a"), ("for-c", "c")]
    with pytest.raises(ValueError):
        mgr.foreach_actor(funcs[:2])


def test_duplicate_live_placement_group_name_rejected(shutdown_only):
    ray.init(num_cpus=2, include_dashboard=False, log_to_driver=False)
    from ray_community_amd.util.placement_group import (get_placement_group, placement_group,
                                                        remove_placement_group)

    pg1 = placement_group([{"CPU": 1}], name="dup")
    ray.get(pg1.ready(), timeout=30)
    with pytest.raises(Exception, match="already exists"):
        placement_group([{"CPU": 1}], name="dup")
    assert get_placement_group("dup").id == pg1.id
    remove_placement_group(pg1)
    pg2 = placement_group([{"CPU": 1}], name="dup")  # the name is free again once removed
    ray.get(pg2.ready(), timeout=30)
    assert get_placement_group("dup").id == pg2.id


def test_worker_hip_mask_indexes_into_rocr_set():
    # ROCR filters the runtime's agents; HIP ids index into the filtered set
    assert worker_hip_visible_devices([0], {"ROCR_VISIBLE_DEVICES": "4,5"}) == "0"
    assert worker_hip_visible_devices([1], {"ROCR_VISIBLE_DEVICES": "4,5"}) == "1"
    # a parent HIP mask is translated entry by entry (ROCR underneath stays inherited)
    assert worker_hip_visible_devices([1], {"ROCR_VISIBLE_DEVICES": "2,3,4,5", "HIP_VISIBLE_DEVICES": "1,3"}) == "3"
    assert worker_hip_visible_devices([0, 1], {"CUDA_VISIBLE_DEVICES": "6,7"}) == "6,7"
    assert worker_hip_visible_devices([2, 3], {}) == "2,3"


def test_session_file_written_atomically(shutdown_only, tmp_path, monkeypatch):
    monkeypatch.setenv("RCA_TEMP_DIR", str(tmp_path))
    ray.init(num_cpus=1, include_dashboard=False, log_to_driver=False)
    path = tmp_path / "latest_session.json"
    assert path.exists()
    rec = json.loads(path.read_text())
    assert rec["pid"] == os.getpid() and rec["sock"]
    assert not [p for p in os.listdir(tmp_path) if p.endswith(".tmp")]


def test_async_puts_are_registered_before_their_refs_escape(shutdown_only):
    """Worker-side ray.put returns before the head acknowledges it; a ref passed on (nested in an
    actor argument, as a top-level argument, inside a returned value) still resolves everywhere,
    and a process's own puts are read back locally."""
    ray.init(num_cpus=3, include_dashboard=False, log_to_driver=False)

    @ray.remote
    class Sink:
        def take(self, refs):
            return sum(ray.get(refs))

        def take_one(self, v):
            return v

    @ray.remote
    def producer(sink):
        from ray_community_amd._private.worker import _core

        core = _core()
        out = []
        for i in range(100):
            out.append(ray.get(sink.take.remote([ray.put(i), ray.put(2 * i)])))
            out.append(ray.get(sink.take_one.remote(ray.put(i))))
            r = ray.put({"k": i})
            assert ray.get(r) == {"k": i} and r._id in core._put_cache  # local read of an own put
        return out, [ray.put(i) for i in range(50)]

    sink = Sink.remote()
    out, refs = ray.get(producer.remote(sink))
    assert out[0::2] == [3 * i for i in range(100)] and out[1::2] == list(range(100))
    assert ray.get(refs) == list(range(50))


def test_core_microbenchmark_separate_driver_mode():
    """bench_core --mode separate: the head runs in its own process (CLI), the driver connects with
    address='auto' and the put/get rows work across the socket."""
    from ray_community_amd._private import ray_perf

    with ray_perf._session("separate", 2):
        from ray_community_amd._private.worker import _core

        core = _core()
        assert type(core.client).__name__ == "SocketClient"
        refs = [ray.put(i) for i in range(200)]
        assert ray.get(refs) == list(range(200))

        @ray.remote
        def add(xs):
            return sum(ray.get(xs))

        assert ray.get(add.remote(refs)) == sum(range(200))
    assert not ray.is_initialized()


def test_direct_call_pins_released_when_caller_dies(shutdown_only):
    """Nested refs of a direct actor call are pinned at the head for the caller; when the caller
    process dies before its unpin, the head drops those pins itself."""
    import time

    ray.init(num_cpus=3, include_dashboard=False, log_to_driver=False)
    from ray_community_amd._private.worker import _core

    head = _core().client.head

    @ray.remote
    class Slow:
        def hold(self, refs):
            time.sleep(3)
            return len(refs)

    @ray.remote(max_retries=0)
    def caller(a):
        import numpy as np

        r = ray.put(np.zeros(200_000))
        a.hold.remote([r])
        time.sleep(1.0)
        os._exit(1)

    a = Slow.remote()
    with pytest.raises(Exception):
        ray.get(caller.remote(a))
    deadline = time.time() + 10
    while time.time() < deadline:
        with head.lock:
            left = {k: dict(v) for k, v in head.call_pins.items() if k.startswith("w:")}
        if not left:
            break
        time.sleep(0.1)
    assert not left, left


def test_remaining_top_level_api_names(shutdown_only):
    """ray.internal (free / memory_summary), ray.widgets, ray._config, ray.util.ray_debugpy,
    ray.job_submission.DriverInfo: the last names of the reference's public __all__ lists."""
    ray.init(num_cpus=1, include_dashboard=False, log_to_driver=False)
    import numpy as np

    big = ray.put(np.zeros(200_000))
    s = ray.internal.memory_summary()
    assert "Objects:" in s and big.hex()[:16] in s.replace("-", "")
    ray.internal.free([big])
    assert "<table>" in ray.widgets.make_table_html_repr({"a": 1}, title="t")
    assert ray.widgets.Template("{{ x }}!").render(x=3) == "3!"
    assert callable(ray.util.ray_debugpy.set_trace)
    from ray_community_amd.job_submission import DriverInfo

    assert DriverInfo(id="j", node_ip_address="127.0.0.1", pid="1").pid == "1"
    with pytest.raises(AttributeError):
        ray._config.not_a_config_entry()
