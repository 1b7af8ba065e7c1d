"""Serve fault handling and handle options (reference: serve/tests/test_failure.py,
test_healthcheck.py, test_handle_api.py, test_max_queued_requests.py)."""
import os
import signal
import time

import pytest

import ray_community_amd as ray
from ray_community_amd import serve


@pytest.fixture
def serve_instance():
    ray.init(num_cpus=8, log_to_driver=False)
    serve.start(http_options={"port": 18124})
    yield
    serve.shutdown()
    ray.shutdown()


def _wait(pred, timeout=60.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            if pred():
                return True
        except Exception:  # noqa
            pass
        time.sleep(0.2)
    return False


def test_killed_replica_is_replaced(serve_instance):
    @serve.deployment(num_replicas=1, health_check_period_s=0.5)
    class P:
        def __call__(self):
            return os.getpid()

    h = serve.run(P.bind(), name="kill", route_prefix=None)
    pid = h.remote().result()
    os.kill(pid, signal.SIGKILL)
    assert _wait(lambda: h.remote().result(timeout_s=5) != pid), "no replacement replica served"
    assert _wait(lambda: serve.status().applications["kill"].status == "RUNNING")


def test_failing_health_check_restarts_replica(serve_instance):
    @serve.deployment(health_check_period_s=0.3, health_check_timeout_s=2)
    class H:
        def __init__(self):
            self.bad = False

        def check_health(self):
            if self.bad:
                raise RuntimeError("unhealthy")

        def poison(self):
            self.bad = True
            return os.getpid()

        def __call__(self):
            return os.getpid()

    h = serve.run(H.bind(), name="hc", route_prefix=None)
    pid = h.poison.remote().result()
    assert _wait(lambda: h.remote().result(timeout_s=5) != pid), "unhealthy replica kept serving"


def test_handle_options_method_and_errors(serve_instance):
    @serve.deployment
    class M:
        def a(self, x):
            return ("a", x)

        def b(self, x):
            return ("b", x)

        def boom(self):
            raise ValueError("kaboom")

    h = serve.run(M.bind(), name="opts", route_prefix=None)
    assert h.options(method_name="b").remote(3).result() == ("b", 3)
    assert h.a.remote(4).result() == ("a", 4)
    with pytest.raises(Exception) as ei:
        h.boom.remote().result()
    assert "kaboom" in str(ei.value)
    # the handle keeps working after a user exception
    assert h.b.remote(5).result() == ("b", 5)


def test_two_apps_and_get_app_handle(serve_instance):
    @serve.deployment
    def one():
        return 1

    @serve.deployment
    def two():
        return 2

    serve.run(one.bind(), name="app1", route_prefix="/one")
    serve.run(two.bind(), name="app2", route_prefix="/two")
    assert serve.get_app_handle("app1").remote().result() == 1
    assert serve.get_app_handle("app2").remote().result() == 2
    st = serve.status()
    assert {"app1", "app2"} <= set(st.applications)
    serve.delete("app1")
    assert "app1" not in serve.status().applications
    assert serve.get_app_handle("app2").remote().result() == 2
