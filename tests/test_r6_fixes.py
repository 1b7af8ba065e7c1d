"""Round-6 fixes: put-cache correctness under rejected puts and ray.internal.free."""
import concurrent.futures
import threading

import pytest

import ray_community_amd as ray
from ray_community_amd import exceptions as rexc


def test_free_then_get_is_not_answered_from_local_put_cache(shutdown_only):
    ray.init(num_cpus=1)
    ref = ray.put({"v": 1})
    assert ray.get(ref) == {"v": 1}  # served locally
    from ray_community_amd._private.worker import free

    free([ref])
    with pytest.raises((rexc.RayError, TimeoutError)):
        ray.get(ref, timeout=2)


def test_rejected_async_put_raises_on_get_and_wait(shutdown_only):
    ray.init(num_cpus=1)
    from ray_community_amd._private.worker import _core

    core = _core()
    orig = core.client.call_async
    pending = []

    def fake(method, *args):
        if method == "put":
            f = concurrent.futures.Future()
            pending.append(f)
            return f
        return orig(method, *args)

    core.client.call_async = fake
    try:
        ref = ray.put([1, 2, 3])
    finally:
        core.client.call_async = orig
    assert pending
    threading.Thread(target=lambda: pending[0].set_exception(ValueError("store rejected the put"))).start()
    for _ in range(200):
        if ref._id in core._put_errors:
            break
        import time
        time.sleep(0.01)
    with pytest.raises(ValueError, match="rejected"):
        ray.get(ref)
    with pytest.raises(ValueError, match="rejected"):
        ray.wait([ref], timeout=0.1)


def test_repeated_shm_get_is_local_and_survives_spill(shutdown_only):
    """A ref's shm descriptor is cached after the first get: repeated gets map the object with no
    head round trip. When the object is spilled meanwhile, the native pin fails and the head is
    asked again (it restores the object); freed objects are never answered from the cache."""
    import numpy as np

    ray.init(num_cpus=1, object_store_memory=40 << 20)
    from ray_community_amd._private.worker import _core, free

    core = _core()
    big = np.arange(2_000_000, dtype=np.float64)  # 16 MB: the shm store
    ref = ray.put(big)
    assert np.array_equal(ray.get(ref), big)
    calls = []
    orig = core.client.call

    def counting(method, *a, **k):
        calls.append(method)
        return orig(method, *a, **k)

    core.client.call = counting
    try:
        for _ in range(5):
            assert ray.get(ref)[123] == 123.0
        assert "get" not in calls
        # push it out of shared memory, then read it again
        others = [ray.put(np.full(2_000_000, i, dtype=np.float64)) for i in range(6)]
        assert orig("store_stats")["num_spilled"] > 0
        assert np.array_equal(ray.get(ref), big)
        del others
    finally:
        core.client.call = orig
    free([ref])
    with pytest.raises((rexc.RayError, TimeoutError)):
        ray.get(ref, timeout=2)
