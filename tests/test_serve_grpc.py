"""Serve gRPC proxy (serve/_private/grpc_proxy.py; reference serve/_private/proxy.py:632,
serve/tests/test_grpc.py): generated-style servicer registration with real protobuf messages
(google.protobuf Struct), unary and server-streaming methods, application routing by metadata,
the built-in RayServeAPIService."""
import json
import socket
import sys

import cloudpickle
import grpc
import pytest
from google.protobuf.struct_pb2 import Struct

import ray_community_amd as ray
from ray_community_amd import serve
from ray_community_amd.serve.config import gRPCOptions

cloudpickle.register_pickle_by_value(sys.modules[__name__])


def add_EchoServicer_to_server(servicer, server):
    """What protoc's grpc plugin generates for ``service Echo {rpc Echo; rpc Count (stream)}``."""
    handlers = {
        "Echo": grpc.unary_unary_rpc_method_handler(servicer.Echo, request_deserializer=Struct.FromString,
                                                    response_serializer=Struct.SerializeToString),
        "Count": grpc.unary_stream_rpc_method_handler(servicer.Count, request_deserializer=Struct.FromString,
                                                      response_serializer=Struct.SerializeToString),
    }
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler("test.Echo", handlers),))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def grpc_serve():
    port = _port()
    ray.init(num_cpus=6)
    serve.start(http_options={"port": _port()},
                grpc_options=gRPCOptions(port=port, grpc_servicer_functions=[add_EchoServicer_to_server]))
    yield port
    serve.shutdown()
    ray.shutdown()


def _s(**kw):
    m = Struct()
    m.update(kw)
    return m


def test_grpc_unary_stream_and_routing(grpc_serve):
    @serve.deployment
    class EchoDep:
        def __init__(self, tag):
            self.tag = tag

        def Echo(self, req):
            return _s(msg=req["msg"] + "!", app=self.tag)

        def Count(self, req):
            for i in range(int(req["n"])):
                yield _s(i=i, app=self.tag)

    serve.run(EchoDep.bind("a"), name="a", route_prefix=None)
    ch = grpc.insecure_channel(f"127.0.0.1:{grpc_serve}")
    echo = ch.unary_unary("/test.Echo/Echo", request_serializer=Struct.SerializeToString,
                          response_deserializer=Struct.FromString)
    count = ch.unary_stream("/test.Echo/Count", request_serializer=Struct.SerializeToString,
                            response_deserializer=Struct.FromString)
    # single application: no metadata needed
    r = echo(_s(msg="hi"), timeout=60)
    assert r["msg"] == "hi!" and r["app"] == "a"
    out = list(count(_s(n=4), timeout=60))
    assert [int(m["i"]) for m in out] == [0, 1, 2, 3]
    # two applications: routed by the 'application' metadata key
    serve.run(EchoDep.bind("b"), name="b", route_prefix=None)
    assert echo(_s(msg="x"), metadata=(("application", "b"),), timeout=60)["app"] == "b"
    assert echo(_s(msg="x"), metadata=(("application", "a"),), timeout=60)["app"] == "a"
    with pytest.raises(grpc.RpcError) as ei:
        echo(_s(msg="x"), timeout=60)  # ambiguous
    assert ei.value.code() == grpc.StatusCode.NOT_FOUND
    with pytest.raises(grpc.RpcError) as ei:
        echo(_s(msg="x"), metadata=(("application", "nope"),), timeout=60)
    assert ei.value.code() == grpc.StatusCode.NOT_FOUND
    # built-in API service
    apps = ch.unary_unary("/ray.serve.RayServeAPIService/ListApplications")(b"", timeout=60)
    assert json.loads(apps) == ["a", "b"]
    assert ch.unary_unary("/ray.serve.RayServeAPIService/Healthz")(b"", timeout=60) == b"success"
    ch.close()


def test_grpc_user_errors_are_internal(grpc_serve):
    @serve.deployment
    class Bad:
        def Echo(self, req):
            raise RuntimeError("model exploded")

    serve.run(Bad.bind(), name="bad", route_prefix=None)
    ch = grpc.insecure_channel(f"127.0.0.1:{grpc_serve}")
    echo = ch.unary_unary("/test.Echo/Echo", request_serializer=Struct.SerializeToString,
                          response_deserializer=Struct.FromString)
    with pytest.raises(grpc.RpcError) as ei:
        echo(_s(msg="x"), timeout=60)
    assert ei.value.code() == grpc.StatusCode.INTERNAL and "model exploded" in ei.value.details()
    ch.close()


def test_grpc_context_reaches_the_deployment_and_its_settings_come_back(grpc_serve):
    """reference serve/grpc_util.py RayServegRPCContext: a method declaring ``grpc_context`` gets
    the request's metadata and can set the status code, details and trailing metadata."""

    @serve.deployment
    class Ctx:
        def Echo(self, req, grpc_context):
            md = dict(grpc_context.invocation_metadata())
            if req["msg"] == "missing":
                grpc_context.set_code(grpc.StatusCode.NOT_FOUND)
                grpc_context.set_details("no such item")
                return _s()
            grpc_context.set_trailing_metadata([("x-served-by", "ctx"), ("x-user", md.get("user", ""))])
            return _s(msg=req["msg"], peer=grpc_context.peer())

        def Count(self, req, grpc_context):
            for i in range(2):
                yield _s(i=i)
            grpc_context.set_trailing_metadata([("x-count", "2")])

    serve.run(Ctx.bind(), name="c", route_prefix=None)
    ch = grpc.insecure_channel(f"127.0.0.1:{grpc_serve}")
    echo = ch.unary_unary("/test.Echo/Echo", request_serializer=Struct.SerializeToString,
                          response_deserializer=Struct.FromString)
    resp, call = echo.with_call(_s(msg="hi"), metadata=(("user", "ann"),), timeout=60)
    assert resp["msg"] == "hi" and resp["peer"]
    assert dict(call.trailing_metadata())["x-served-by"] == "ctx"
    assert dict(call.trailing_metadata())["x-user"] == "ann"
    with pytest.raises(grpc.RpcError) as e:
        echo(_s(msg="missing"), timeout=60)
    assert e.value.code() == grpc.StatusCode.NOT_FOUND and e.value.details() == "no such item"
    count = ch.unary_stream("/test.Echo/Count", request_serializer=Struct.SerializeToString,
                            response_deserializer=Struct.FromString)
    it = count(_s(), timeout=60)
    assert [int(m["i"]) for m in it] == [0, 1]
    assert dict(it.trailing_metadata())["x-count"] == "2"

    # a plain handle call (no gRPC request) never sees a context
    @serve.deployment
    class Plain:
        def __call__(self, x):
            return x + 1

    h = serve.run(Plain.bind(), name="p", route_prefix=None)
    assert h.remote(1).result() == 2
