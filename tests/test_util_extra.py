"""util.iter / joblib backend / check_serialize / annotations / custom serializers
(reference tests: python/ray/tests/test_iter.py, test_joblib.py, test_serialization.py)."""
import threading

import pytest

import ray_community_amd as ray


def test_parallel_iterator(ray_start_regular):
    from ray_community_amd.util import iter as it

    p = it.from_range(20, num_shards=3).for_each(lambda x: x * 2).filter(lambda x: x % 3 == 0)
    assert sorted(p.gather_sync()) == [0, 6, 12, 18, 24, 30, 36]
    q = it.from_items(list(range(10)), num_shards=2).batch(3)
    assert sorted(x for b in q.gather_async() for x in b) == list(range(10))
    assert p.num_shards() == 3
    assert sorted(x for s in p.shards() for x in s) == [0, 6, 12, 18, 24, 30, 36]
    loc = it.from_items([1, 2, 3], num_shards=1).gather_sync().for_each(lambda x: x + 1)
    assert loc.take(2) == [2, 3]
    with pytest.raises(TypeError):
        iter(p)


def test_joblib_backend(ray_start_regular):
    import joblib

    from ray_community_amd.util.joblib import register_ray

    register_ray()
    with joblib.parallel_backend("ray"):
        out = joblib.Parallel(n_jobs=4)(joblib.delayed(pow)(i, 2) for i in range(16))
    assert out == [i * i for i in range(16)]


def test_pool_callbacks_fire_without_get(ray_start_regular):
    from ray_community_amd.util.multiprocessing import Pool

    ev = threading.Event()
    got = []
    pool = Pool(2)
    pool.apply_async(pow, (3, 2), callback=lambda v: (got.append(v), ev.set()))
    assert ev.wait(30) and got == [9]
    pool.terminate()


def test_inspect_serializability():
    from ray_community_amd.util import inspect_serializability

    lock = threading.Lock()

    def uses_lock():
        return lock

    ok, fails = inspect_serializability(uses_lock, name="uses_lock")
    assert not ok and {f.name for f in fails} == {"lock"}
    assert inspect_serializability(lambda: 1)[0]


def test_annotations_and_custom_serializer(ray_start_regular):
    from ray_community_amd.util.annotations import Deprecated, DeveloperAPI, PublicAPI
    from ray_community_amd.util.serialization import deregister_serializer, register_serializer

    @PublicAPI(stability="beta")
    def f():
        """doc"""
        return 1

    @DeveloperAPI
    class C:
        pass

    @Deprecated(message="use g")
    def old():
        return 2

    assert f() == 1 and "PublicAPI" in f.__doc__
    with pytest.warns(DeprecationWarning):
        assert old() == 2

    class Point:
        def __init__(self, x):
            self.x = x
            self.lock = threading.Lock()  # not picklable by default

    register_serializer(Point, serializer=lambda p: p.x, deserializer=lambda x: Point(x))
    try:
        @ray.remote
        def get_x(p):
            return p.x

        assert ray.get(get_x.remote(Point(7))) == 7
    finally:
        deregister_serializer(Point)
