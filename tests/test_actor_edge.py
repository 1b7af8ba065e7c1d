"""Actor edge cases (reference test models: python/ray/tests/test_actor.py, test_actor_failures.py,
test_asyncio.py (async actors overlap awaits), test_actor_advanced.py (named actors, get_if_exists,
ray.kill(no_restart=False) restarts))."""
import os
import time

import pytest

import ray_community_amd as ray


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_async_actor_overlaps_awaits(session):
    @ray.remote
    class A:
        async def nap(self, t):
            import asyncio

            await asyncio.sleep(t)
            return t

    a = A.options(max_concurrency=8).remote()
    ray.get(a.nap.remote(0))
    t0 = time.time()
    assert ray.get([a.nap.remote(0.5) for _ in range(8)]) == [0.5] * 8
    assert time.time() - t0 < 2.5


def test_get_if_exists_returns_the_same_actor(session):
    @ray.remote
    class Named:
        def pid(self):
            return os.getpid()

    a = Named.options(name="edge_named", get_if_exists=True).remote()
    b = Named.options(name="edge_named", get_if_exists=True).remote()
    assert ray.get(a.pid.remote()) == ray.get(b.pid.remote())
    assert ray.get(ray.get_actor("edge_named").pid.remote()) == ray.get(a.pid.remote())
    ray.kill(a)
    deadline = time.time() + 10
    while time.time() < deadline:
        try:
            ray.get_actor("edge_named")
        except ValueError:
            break
        time.sleep(0.1)
    with pytest.raises(ValueError):
        ray.get_actor("edge_named")


def test_kill_with_restart_brings_a_fresh_instance(session):
    @ray.remote(max_restarts=1)
    class Stateful:
        def __init__(self):
            self.n = 0

        def inc(self):
            self.n += 1
            return self.n, os.getpid()

    s = Stateful.remote()
    n1, pid1 = ray.get(s.inc.remote())
    ray.get(s.inc.remote())
    ray.kill(s, no_restart=False)
    deadline = time.time() + 30
    while True:
        try:
            n, pid = ray.get(s.inc.remote(), timeout=10)
            break
        except Exception:
            if time.time() > deadline:
                raise
            time.sleep(0.2)
    assert pid != pid1 and n == 1                          # constructor re-ran in a new process


def test_actor_method_num_returns_and_ordering(session):
    @ray.remote
    class Seq:
        def __init__(self):
            self.log = []

        def push(self, x):
            self.log.append(x)

        @ray.method(num_returns=2)
        def split(self):
            return self.log[: len(self.log) // 2], self.log[len(self.log) // 2:]

    s = Seq.remote()
    for i in range(50):
        s.push.remote(i)
    lo, hi = s.split.remote()
    assert ray.get(lo) + ray.get(hi) == list(range(50))   # per-caller submission order kept
