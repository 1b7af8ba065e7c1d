"""Serve replica scheduler (reference: serve/_private/replica_scheduler/pow_2_scheduler.py): replica
queue lengths are probed (short-TTL cache, deadline backoff), so routers in different processes
see each other's load; node / GPU locality tiers."""
import time

import pytest

import ray_community_amd as ray
from ray_community_amd import serve
from ray_community_amd.serve.handle import _Router, physical_gpu_ids


@pytest.fixture
def serve_instance():
    ray.init(num_cpus=12, include_dashboard=False, log_to_driver=False)
    yield
    serve.shutdown()
    ray.shutdown()


def test_eight_callers_in_eight_processes_balance_two_replicas(serve_instance):
    @serve.deployment(num_replicas=2, max_ongoing_requests=4)
    class Work:
        def __init__(self):
            self.active = 0
            self.peak = 0

        async def __call__(self, s):
            import asyncio

            from ray_community_amd.serve import get_replica_context

            self.active += 1
            self.peak = max(self.peak, self.active)
            await asyncio.sleep(s)
            self.active -= 1
            return get_replica_context().replica_tag

        async def peak_active(self):
            return self.peak

    serve.run(Work.bind(), name="bal", route_prefix="/bal")

    @ray.remote(num_cpus=1)
    class Caller:
        def __init__(self):
            self.h = serve.get_deployment_handle("Work", app_name="bal")
            self.h.remote(0).result()  # warm this process's router (replica set + locations)

        def call(self, delay, s):
            time.sleep(delay)
            return self.h.remote(s).result()

    callers = [Caller.remote() for _ in range(8)]
    ray.get([c.call.remote(0, 0) for c in callers])
    time.sleep(0.6)  # every router's cached queue lengths expire: the next picks probe fresh
    # staggered: each caller's request arrives while the earlier ones are still running
    tags = ray.get([c.call.remote(0.15 * i, 3.0) for i, c in enumerate(callers)])
    counts = {t: tags.count(t) for t in set(tags)}
    assert sorted(counts.values()) == [4, 4], counts
    h = serve.get_deployment_handle("Work", app_name="bal")
    peaks = [h.peak_active.remote().result() for _ in range(8)]
    assert max(peaks) <= 4


def test_router_records_replica_locations_and_probes(serve_instance):
    @serve.deployment(num_replicas=2)
    class Echo:
        def __call__(self, x):
            return x

    h = serve.run(Echo.bind(), name="loc", route_prefix="/loc")
    for _ in range(5):
        assert h.remote(1).result() == 1
    r = _Router.get("loc", "Echo")
    deadline = time.time() + 10
    while len(r.locations) < 2 and time.time() < deadline:
        time.sleep(0.1)
    node = ray.get_runtime_context().get_node_id()
    assert len(r.locations) == 2 and all(loc["node_id"] == node for loc in r.locations.values())
    assert r.stats["probes"] >= 1 and r.stats["picks"] >= 5


def test_physical_gpu_id_layering(monkeypatch):
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "4,5,6")
    assert physical_gpu_ids([0, 2]) == [4, 6]
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,1")
    assert physical_gpu_ids([0, 1]) == [6, 5]
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES")
    assert physical_gpu_ids([0]) == [2]


def test_gpu_tensor_request_prefers_replica_on_same_gpu(monkeypatch):
    """Tier order without a cluster: a request whose tensor sits on physical GPU 3 of this node goes
    to the replica that owns GPU 3 (no xGMI copy), a CPU request to any replica of this node."""
    r = _Router("app", "dep")
    r.replicas = [("a", object()), ("b", object()), ("c", object())]
    r.locations = {"a": {"node_id": "n0", "gpus": [2]}, "b": {"node_id": "n0", "gpus": [3]},
                   "c": {"node_id": "n1", "gpus": [3]}}
    r.max_ongoing = 4
    r.qlen = {t: (0, time.time() + 60) for t in "abc"}
    monkeypatch.setattr("ray_community_amd.serve.handle._caller_node", lambda: "n0")
    with r.cv:
        picks = {r._pick_locked(3)[0] for _ in range(3)}
    assert picks == {"b"}
    r.inflight = {}
    with r.cv:
        picks = [r._pick_locked(None)[0] for _ in range(8)]
    assert set(picks) == {"a", "b"}  # this node's replicas first, until both are full (4 + 4)
    with r.cv:
        assert r._pick_locked(None)[0] == "c"  # then the other node


def test_replica_enforces_max_ongoing_requests_against_overcommitting_routers(serve_instance):
    """Routers in different processes decide on cached queue lengths and can send a replica more
    than ``max_ongoing_requests`` at once; the replica runs at most that many and queues the rest."""

    @serve.deployment(num_replicas=1, max_ongoing_requests=2)
    class Slow:
        def __init__(self):
            self.active = 0
            self.peak = 0

        async def __call__(self, s):
            import asyncio

            self.active += 1
            self.peak = max(self.peak, self.active)
            await asyncio.sleep(s)
            self.active -= 1
            return True

        async def peak_active(self):
            return self.peak

    serve.run(Slow.bind(), name="cap", route_prefix="/cap")

    @ray.remote(num_cpus=0)
    class Caller:
        def __init__(self):
            self.h = serve.get_deployment_handle("Slow", app_name="cap")

        def burst(self, n, s):
            return [r.result() for r in [self.h.remote(s) for _ in range(n)]]

    callers = [Caller.remote() for _ in range(5)]
    t0 = time.time()
    out = ray.get([c.burst.remote(2, 0.5) for c in callers])
    assert all(all(x) for x in out)
    h = serve.get_deployment_handle("Slow", app_name="cap")
    assert h.peak_active.remote().result() <= 2
    assert time.time() - t0 >= 0.5 * 10 / 2 * 0.9  # 10 requests, 2 at a time
