"""gRPC proxy actor (reference: ``serve/_private/proxy.py:632`` ``gRPCProxy`` and
``serve/config.py`` ``gRPCOptions``).

Users register their generated ``add_<Service>Servicer_to_server`` functions through
``serve.start(grpc_options={"port": ..., "grpc_servicer_functions": [...]})``. The proxy calls
each one against a capturing stand-in server to learn the service's methods together with their
protobuf (de)serializers, then serves those methods itself: a call is routed to the ingress
deployment of the application named by the ``application`` metadata key (or the only running
application), and the deployment method with the gRPC method's name receives the decoded request
message and returns the response message (unary) or yields messages (server streaming, over
``handle.options(stream=True)``). ``multiplexed_model_id`` metadata selects a multiplexed model.
Built-in ``/ray.serve.RayServeAPIService/{ListApplications,Healthz}`` answer with JSON bytes;
methods of unregistered services are served with raw bytes in and out.
"""
from __future__ import annotations

import importlib
import json
import threading
import time

from ..exceptions import BackPressureError
from concurrent import futures
from typing import Dict, List, Optional


def _resolve(fn):
    if callable(fn):
        return fn
    mod, _, name = str(fn).rpartition(".")
    return getattr(importlib.import_module(mod), name)


class _Capture:
    """Stand-in ``grpc.Server`` that records the generic handlers a servicer function adds."""

    def __init__(self):
        self.handlers = []

    def add_generic_rpc_handlers(self, handlers):
        self.handlers.extend(handlers)

    def add_registered_method_handlers(self, service, handlers):  # grpcio >= 1.62 generated code
        import grpc

        self.handlers.append(grpc.method_handlers_generic_handler(service, handlers))


class _AnyServicer:
    def __getattr__(self, name):
        def _placeholder(*a, **k):  # pragma: no cover - replaced by the proxy's own handlers
            raise NotImplementedError(name)

        return _placeholder


class gRPCProxy:
    def __init__(self, host: str = "127.0.0.1", port: int = 9000, servicer_functions: Optional[List] = None,
                 max_workers: int = 32):
        import grpc

        self.host, self.port = host, port
        self._apps: Dict[str, str] = {}
        self._apps_t = 0.0
        self._lock = threading.Lock()
        self.methods: Dict[str, tuple] = {}  # "/pkg.Service/Method" -> (kind, req_deser, resp_ser)
        for fn in servicer_functions or []:
            cap = _Capture()
            _resolve(fn)(_AnyServicer(), cap)
            for h in cap.handlers:
                # method_handlers_generic_handler keeps {full method path: RpcMethodHandler}
                table = getattr(h, "_method_handlers", None) or {}
                for path, mh in table.items():
                    kind = "unary_stream" if mh.unary_stream is not None else "unary_unary"
                    if mh.stream_unary is not None or mh.stream_stream is not None:
                        continue  # client streaming is not supported by Serve (as in the reference)
                    self.methods[path] = (kind, mh.request_deserializer, mh.response_serializer)
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
        self._server.add_generic_rpc_handlers((_Router(self),))
        bound = self._server.add_insecure_port(f"{host}:{port}")
        if bound == 0:
            raise RuntimeError(f"gRPC proxy could not bind {host}:{port}")
        self.port = bound
        self._server.start()

    def ready(self):
        return {"host": self.host, "port": self.port, "methods": sorted(self.methods)}

    # ------------------------------------------------------------------ routing
    def _app_table(self, force=False) -> Dict[str, str]:
        from ..api import _get_controller
        from ..._private import worker as w

        with self._lock:
            if force or time.time() - self._apps_t > 1.0:
                self._apps = w.get(_get_controller().list_applications.remote())
                self._apps_t = time.time()
            return dict(self._apps)

    def handle_for(self, context, method: str):
        import grpc

        from ..handle import DeploymentHandle

        md = dict(context.invocation_metadata() or ())
        app = md.get("application")
        apps = self._app_table()
        if app is None:
            if len(apps) != 1:
                apps = self._app_table(force=True)
            if len(apps) != 1:
                context.abort(grpc.StatusCode.NOT_FOUND,
                              f"set the 'application' metadata key; running applications: {sorted(apps)}")
            app = next(iter(apps))
        if app not in apps:
            apps = self._app_table(force=True)
            if app not in apps:
                context.abort(grpc.StatusCode.NOT_FOUND, f"application '{app}' not found")
        h = DeploymentHandle(apps[app], app).options(method_name=method)
        mid = md.get("multiplexed_model_id")
        if mid:
            h = h.options(multiplexed_model_id=mid)
        return h

    def shutdown(self):
        self._server.stop(grace=1.0)
        return True


class _Router:
    """``grpc.GenericRpcHandler``: maps every incoming method path to a handler."""

    def __init__(self, proxy: gRPCProxy):
        self.proxy = proxy

    def service(self, details):
        import grpc

        path = details.method
        if path == "/ray.serve.RayServeAPIService/ListApplications":
            return grpc.unary_unary_rpc_method_handler(
                lambda req, ctx: json.dumps(sorted(self.proxy._app_table(force=True))).encode())
        if path == "/ray.serve.RayServeAPIService/Healthz":
            return grpc.unary_unary_rpc_method_handler(lambda req, ctx: b"success")
        method = path.rsplit("/", 1)[-1]
        kind, deser, ser = self.proxy.methods.get(path, ("unary_unary", None, None))
        from ..grpc_util import RayServegRPCContext, _GrpcReply

        if kind == "unary_stream":
            def stream(req, ctx, method=method):
                h = self.proxy.handle_for(ctx, method).options(stream=True, _grpc_context=RayServegRPCContext(ctx))
                try:
                    for item in h.remote(req):
                        if isinstance(item, _GrpcReply):  # the stream's final context
                            item.context._apply(ctx)
                            continue
                        yield item
                except BackPressureError as e:
                    ctx.abort(grpc.StatusCode.UNAVAILABLE, e.message)
                except Exception as e:  # noqa
                    ctx.abort(grpc.StatusCode.INTERNAL, f"{type(e).__name__}: {e}")

            return grpc.unary_stream_rpc_method_handler(stream, request_deserializer=deser, response_serializer=ser)

        def unary(req, ctx, method=method):
            h = self.proxy.handle_for(ctx, method).options(_grpc_context=RayServegRPCContext(ctx))
            try:
                out = h.remote(req).result()
                if isinstance(out, _GrpcReply):
                    out.context._apply(ctx)
                    out = out.value
                return out
            except BackPressureError as e:
                ctx.abort(grpc.StatusCode.UNAVAILABLE, e.message)
            except Exception as e:  # noqa
                ctx.abort(grpc.StatusCode.INTERNAL, f"{type(e).__name__}: {e}")

        return grpc.unary_unary_rpc_method_handler(unary, request_deserializer=deser, response_serializer=ser)
