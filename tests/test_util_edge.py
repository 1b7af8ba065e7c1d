"""ray.util edge cases (reference test models: python/ray/tests/test_multiprocessing.py (imap keeps
order, imap_unordered covers all, starmap, apply_async callbacks), test_queue.py (Empty/Full with
timeouts, batch put/get), test_actor_pool.py (map_unordered covers all inputs))."""
import time

import pytest

import ray_community_amd as ray
from ray_community_amd.util.actor_pool import ActorPool
from ray_community_amd.util.multiprocessing import Pool
from ray_community_amd.util.queue import Empty, Full, Queue


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _sq(x):
    return x * x


def _add(a, b):
    return a + b


def test_pool_orderings_and_async(session):
    with Pool(processes=2) as p:
        assert list(p.imap(_sq, range(20), chunksize=3)) == [i * i for i in range(20)]
        assert sorted(p.imap_unordered(_sq, range(20))) == [i * i for i in range(20)]
        assert p.starmap(_add, [(1, 2), (3, 4)]) == [3, 7]
        got = []
        r = p.apply_async(_sq, (7,), callback=got.append)
        assert r.get(timeout=30) == 49
        deadline = time.time() + 5
        while not got and time.time() < deadline:
            time.sleep(0.01)
        assert got == [49]


def test_queue_timeouts_and_batches(session):
    q = Queue(maxsize=2)
    q.put_nowait_batch([1, 2])
    with pytest.raises(Full):
        q.put(3, timeout=0.2)
    assert q.get_nowait_batch(2) == [1, 2]
    with pytest.raises(Empty):
        q.get(timeout=0.2)
    assert q.empty() and q.size() == 0


def test_actor_pool_map_unordered_covers_inputs(session):
    @ray.remote
    class W:
        def f(self, x):
            return 2 * x

    pool = ActorPool([W.remote() for _ in range(3)])
    out = list(pool.map_unordered(lambda a, v: a.f.remote(v), range(30)))
    assert sorted(out) == [2 * i for i in range(30)]
