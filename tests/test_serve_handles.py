"""Serve handle behaviour (reference test models: python/ray/serve/tests/test_handle_api.py
(method calls, options(method_name=...), streaming), test_api.py (multiple applications,
get_app_handle / get_deployment_handle, user_config + reconfigure), test_deploy.py (delete),
test_standalone / test_http_routes (HTTP ingress on a route prefix, replica exceptions))."""
import json
import time
import urllib.request

import pytest

import ray_community_amd as ray
from ray_community_amd import serve

PORT = 18131


@pytest.fixture(scope="module")
def serve_instance():
    ray.init(num_cpus=8, log_to_driver=False)
    serve.start(http_options={"port": PORT})
    yield
    serve.shutdown()
    ray.shutdown()


def test_method_calls_and_options(serve_instance):
    @serve.deployment
    class Calc:
        def __init__(self, base):
            self.base = base

        def add(self, x):
            return self.base + x

        def mul(self, x):
            return self.base * x

        def __call__(self, x):
            return -x

    h = serve.run(Calc.bind(10), name="calc", route_prefix=None)
    assert h.remote(3).result() == -3
    assert h.add.remote(3).result() == 13
    assert h.options(method_name="mul").remote(3).result() == 30
    # handles from the registry reach the same application
    assert serve.get_app_handle("calc").add.remote(1).result() == 11
    assert serve.get_deployment_handle("Calc", app_name="calc").mul.remote(2).result() == 20


def test_streaming_handle_yields_in_order(serve_instance):
    @serve.deployment
    class Gen:
        def __call__(self, n):
            for i in range(n):
                yield i * i

    h = serve.run(Gen.bind(), name="gen", route_prefix=None)
    assert list(h.options(stream=True).remote(6)) == [i * i for i in range(6)]


def test_replica_exception_reaches_caller_and_replica_survives(serve_instance):
    @serve.deployment
    class Picky:
        def __call__(self, x):
            if x < 0:
                raise ValueError("negative input")
            return x

    h = serve.run(Picky.bind(), name="picky", route_prefix=None)
    with pytest.raises(Exception, match="negative input"):
        h.remote(-1).result()
    assert h.remote(5).result() == 5                    # the replica kept serving


def test_user_config_reconfigure_in_place(serve_instance):
    @serve.deployment(user_config={"scale": 2})
    class Scaled:
        def __init__(self):
            self.scale = None

        def reconfigure(self, cfg):
            self.scale = cfg["scale"]

        def __call__(self, x):
            import os

            return self.scale * x, os.getpid()

    h = serve.run(Scaled.bind(), name="scaled", route_prefix=None)
    v, pid = h.remote(3).result()
    assert v == 6
    serve.run(Scaled.options(user_config={"scale": 5}).bind(), name="scaled", route_prefix=None)
    deadline = time.time() + 30
    while time.time() < deadline:
        v, pid2 = h.remote(3).result()
        if v == 15:
            break
        time.sleep(0.2)
    assert v == 15 and pid2 == pid                       # same replica, new config


def test_multiple_apps_and_delete(serve_instance):
    @serve.deployment
    class Echo:
        def __init__(self, tag):
            self.tag = tag

        def __call__(self):
            return self.tag

    ha = serve.run(Echo.bind("a"), name="app_a", route_prefix=None)
    hb = serve.run(Echo.bind("b"), name="app_b", route_prefix=None)
    assert ha.remote().result() == "a" and hb.remote().result() == "b"
    apps = serve.status().applications
    assert "app_a" in apps and "app_b" in apps
    serve.delete("app_a")
    deadline = time.time() + 30
    while time.time() < deadline and "app_a" in serve.status().applications:
        time.sleep(0.2)
    assert "app_a" not in serve.status().applications
    assert hb.remote().result() == "b"                   # the other app is untouched


def test_http_ingress_on_route_prefix(serve_instance):
    @serve.deployment
    class Api:
        async def __call__(self, request):
            body = await request.json()
            return {"sum": sum(body["xs"])}

    serve.run(Api.bind(), name="http_api", route_prefix="/sum")
    req = urllib.request.Request(f"http://127.0.0.1:{PORT}/sum", data=json.dumps({"xs": [1, 2, 3]}).encode(),
                                 headers={"Content-Type": "application/json"}, method="POST")
    deadline = time.time() + 30
    while True:
        try:
            with urllib.request.urlopen(req, timeout=10) as r:
                out = json.loads(r.read())
            break
        except Exception:
            if time.time() > deadline:
                raise
            time.sleep(0.3)
    assert out == {"sum": 6}
