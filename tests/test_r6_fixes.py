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
