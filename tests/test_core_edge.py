"""Core API edge cases (reference test models: python/ray/tests/test_basic.py (num_returns, nested
tasks, options), test_get_or_put / test_object_store (zero-copy read-only numpy), test_wait.py
(num_returns / timeout ordering), test_failure.py (retry_exceptions, GetTimeoutError),
test_actor.py (actor handles passed to tasks))."""
import time

import numpy as np
import pytest

import ray_community_amd as ray
from ray_community_amd import exceptions as rexc


@pytest.fixture(scope="module")
def session():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_num_returns_and_nested_tasks(session):
    @ray.remote(num_returns=3)
    def three(x):
        return x, x + 1, x + 2

    @ray.remote
    def outer(n):
        return sum(ray.get(list(three.remote(n))))

    a, b, c = three.remote(1)
    assert ray.get([a, b, c]) == [1, 2, 3]
    assert ray.get(outer.remote(10)) == 33
    refs = three.options(num_returns=3).remote(5)
    assert ray.get(refs[2]) == 7


def test_numpy_put_is_read_only_zero_copy(session):
    arr = np.arange(1 << 20, dtype=np.float32)
    ref = ray.put(arr)
    got = ray.get(ref)
    assert np.array_equal(got, arr)
    assert not got.flags.writeable                       # a view of the shared store, not a copy
    with pytest.raises(ValueError):
        got[0] = 1.0

    @ray.remote
    def total(x):
        return float(x.sum())

    assert ray.get(total.remote(ref)) == pytest.approx(float(arr.sum()))


def test_wait_returns_ready_first_and_respects_timeout(session):
    @ray.remote
    def sleepy(t):
        time.sleep(t)
        return t

    fast, slow = sleepy.remote(0.0), sleepy.remote(3.0)
    ready, rest = ray.wait([slow, fast], num_returns=1, timeout=2.0)
    assert ready == [fast] and rest == [slow]
    t0 = time.time()
    ready, rest = ray.wait([slow], num_returns=1, timeout=0.2)
    assert ready == [] and rest == [slow] and time.time() - t0 < 1.5
    with pytest.raises(rexc.GetTimeoutError):
        ray.get(slow, timeout=0.1)
    assert ray.get(slow) == 3.0


def test_retry_exceptions_reruns_application_errors(session, tmp_path):
    marker = tmp_path / "attempts"

    @ray.remote(max_retries=3, retry_exceptions=True)
    def flaky(path):
        import os

        n = int(open(path).read()) if os.path.exists(path) else 0
        open(path, "w").write(str(n + 1))
        if n < 2:
            raise RuntimeError("transient")
        return n

    assert ray.get(flaky.remote(str(marker))) == 2
    assert marker.read_text() == "3"

    @ray.remote(max_retries=3)  # application errors are not retried without retry_exceptions
    def always(path):
        import os

        n = int(open(path).read()) if os.path.exists(path) else 0
        open(path, "w").write(str(n + 1))
        raise RuntimeError("boom")

    m2 = tmp_path / "once"
    with pytest.raises(Exception, match="boom"):
        ray.get(always.remote(str(m2)))
    assert m2.read_text() == "1"


def test_actor_handle_passed_to_tasks(session):
    @ray.remote
    class Counter:
        def __init__(self):
            self.n = 0

        def inc(self, k=1):
            self.n += k
            return self.n

        def get(self):
            return self.n

    @ray.remote
    def bump(c, k):
        return ray.get(c.inc.remote(k))

    c = Counter.remote()
    ray.get([bump.remote(c, k) for k in range(1, 6)])
    assert ray.get(c.get.remote()) == 15


def test_options_override_resources(session):
    @ray.remote(num_cpus=1)
    def cpus():
        return ray.get_runtime_context().get_assigned_resources().get("CPU")

    assert ray.get(cpus.remote()) == 1
    assert ray.get(cpus.options(num_cpus=2).remote()) == 2
