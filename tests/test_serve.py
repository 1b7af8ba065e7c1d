"""Serve tests (modelled on reference serve/tests/test_api.py, test_handle*.py, test_batching.py,
test_autoscaling_policy.py, test_fastapi.py)."""
import asyncio
import time

import pytest
import requests

import ray_community_amd as ray
from ray_community_amd import serve


@pytest.fixture
def serve_instance():
    ray.init(num_cpus=8)
    serve.start(http_options={"port": 18123})
    yield
    serve.shutdown()
    ray.shutdown()


def test_function_and_class_deployments(serve_instance):
    @serve.deployment
    def hello(name):
        return f"hello {name}"

    h = serve.run(hello.bind(), name="f", route_prefix=None)
    assert h.remote("x").result() == "hello x"

    @serve.deployment(num_replicas=2)
    class Counter:
        def __init__(self, start):
            self.n = start

        def __call__(self, k):
            self.n += k
            return self.n

        def pid(self):
            import os

            return os.getpid()

    h2 = serve.run(Counter.bind(10), name="c", route_prefix=None)
    assert h2.remote(1).result() >= 11
    pids = {h2.pid.remote().result() for _ in range(30)}
    assert len(pids) == 2
    st = serve.status()
    assert st.applications["c"].status == "RUNNING"


def test_composition_and_chaining(serve_instance):
    @serve.deployment
    class Adder:
        def __init__(self, k):
            self.k = k

        def __call__(self, x):
            return x + self.k

    @serve.deployment
    class Pipeline:
        def __init__(self, a, b):
            self.a = a
            self.b = b

        async def __call__(self, x):
            r = self.a.remote(x)
            return await self.b.remote(r)  # chained response resolved in the replica

    h = serve.run(Pipeline.bind(Adder.bind(1), Adder.options(name="Adder2").bind(10)), name="p", route_prefix=None)
    assert h.remote(5).result() == 16


def test_batching(serve_instance):
    @serve.deployment(max_ongoing_requests=32)
    class B:
        @serve.batch(max_batch_size=8, batch_wait_timeout_s=0.2)
        async def __call__(self, xs):
            return [(x, len(xs)) for x in xs]

    h = serve.run(B.bind(), name="b", route_prefix=None)
    rs = [h.remote(i) for i in range(8)]
    out = [r.result() for r in rs]
    assert [o[0] for o in out] == list(range(8))
    assert max(o[1] for o in out) > 1


def test_http_ingress_fastapi(serve_instance):
    from fastapi import FastAPI

    app = FastAPI()

    @serve.deployment
    @serve.ingress(app)
    class Api:
        def __init__(self):
            self.msg = "hi"

        @app.get("/hello")
        def hello(self, name: str = "x"):
            return {"msg": f"{self.msg} {name}"}

        @app.post("/echo")
        async def echo(self, payload: dict):
            return payload

    serve.run(Api.bind(), name="api", route_prefix="/api")
    r = requests.get("http://127.0.0.1:18123/api/hello", params={"name": "bob"}, timeout=30)
    assert r.status_code == 200 and r.json() == {"msg": "hi bob"}
    r = requests.post("http://127.0.0.1:18123/api/echo", json={"a": 1}, timeout=30)
    assert r.json() == {"a": 1}
    assert requests.get("http://127.0.0.1:18123/nope", timeout=30).status_code == 404


def test_http_plain_call(serve_instance):
    @serve.deployment
    class Plain:
        async def __call__(self, request):
            body = await request.json()
            return {"sum": sum(body["xs"])}

    serve.run(Plain.bind(), name="plain", route_prefix="/plain")
    r = requests.post("http://127.0.0.1:18123/plain", json={"xs": [1, 2, 3]}, timeout=30)
    assert r.json() == {"sum": 6}


def test_user_config_and_delete(serve_instance):
    @serve.deployment(user_config={"v": 1})
    class C:
        def reconfigure(self, cfg):
            self.v = cfg["v"]

        def __call__(self):
            return self.v

    h = serve.run(C.bind(), name="uc", route_prefix=None)
    assert h.remote().result() == 1
    h = serve.run(C.options(user_config={"v": 2}).bind(), name="uc", route_prefix=None)
    assert h.remote().result() == 2
    serve.delete("uc")
    assert "uc" not in serve.status()


def test_autoscaling(serve_instance):
    @serve.deployment(max_ongoing_requests=2,
                      autoscaling_config={"min_replicas": 1, "max_replicas": 3, "target_ongoing_requests": 1,
                                          "upscale_delay_s": 0, "downscale_delay_s": 1})
    class Slow:
        async def __call__(self):
            await asyncio.sleep(1.0)
            return 1

    h = serve.run(Slow.bind(), name="as", route_prefix=None)
    rs = [h.remote() for _ in range(12)]
    time.sleep(2.0)
    n = serve.status()["as"]["deployments"]["Slow"]["replicas"]
    [r.result() for r in rs]
    assert n > 1


def test_multiplexing(serve_instance):
    @serve.deployment
    class M:
        def __init__(self):
            self.loads = 0

        @serve.multiplexed(max_num_models_per_replica=2)
        async def get_model(self, mid):
            self.loads += 1
            return f"model-{mid}"

        async def __call__(self):
            mid = serve.get_multiplexed_model_id()
            m = await self.get_model(mid)
            return m, self.loads

    h = serve.run(M.bind(), name="mux", route_prefix=None)
    assert h.options(multiplexed_model_id="a").remote().result() == ("model-a", 1)
    assert h.options(multiplexed_model_id="a").remote().result() == ("model-a", 1)
    assert h.options(multiplexed_model_id="b").remote().result() == ("model-b", 2)


def test_streaming_http_and_handle(serve_instance):
    """Responses stream chunk by chunk: a generator __call__ over HTTP (the first chunk arrives
    before the generator finishes), a FastAPI StreamingResponse, and handle.options(stream=True)."""
    import time as _time

    from fastapi import FastAPI
    from fastapi.responses import StreamingResponse

    @serve.deployment
    class Ticker:
        def __call__(self, request):
            def gen():
                for i in range(3):
                    yield f"tick{i}\n"
                    _time.sleep(0.4)
            return gen()

        def count(self, n):
            for i in range(n):
                yield i

    h = serve.run(Ticker.bind(), name="ticker", route_prefix="/ticker")
    t0 = _time.time()
    with requests.get("http://127.0.0.1:18123/ticker", stream=True, timeout=30) as r:
        it = r.iter_lines()
        first = next(it)
        t_first = _time.time() - t0
        rest = list(it)
    assert first == b"tick0" and rest == [b"tick1", b"tick2"]
    assert t_first < 0.7  # the whole response takes >= 0.8 s
    assert list(h.options(method_name="count", stream=True).remote(4)) == [0, 1, 2, 3]

    app = FastAPI()

    @serve.deployment
    @serve.ingress(app)
    class Api:
        @app.get("/s")
        def s(self):
            return StreamingResponse(iter([b"a", b"b", b"c"]), media_type="text/plain")

    serve.run(Api.bind(), name="sapi", route_prefix="/sapi")
    assert requests.get("http://127.0.0.1:18123/sapi/s", timeout=30).content == b"abc"
