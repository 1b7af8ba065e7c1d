"""Serve public API (reference: ``python/ray/serve/api.py``, ``deployment.py``)."""
from __future__ import annotations

import copy
import hashlib
import inspect
import time
from typing import Any, Callable, Dict, List, Optional, Union

from .._private import serialization as ser
from ._private.controller import CONTROLLER_NAME, NAMESPACE, ServeController
from .handle import DeploymentHandle, _HandleSpec

_STATE = {"controller": None, "proxy": None, "http": {"host": "127.0.0.1", "port": 8000}, "grpc": None,
          "grpc_proxy": None}

_DEP_OPTS = {"name", "num_replicas", "ray_actor_options", "max_ongoing_requests", "max_concurrent_queries",
             "autoscaling_config", "user_config", "health_check_period_s", "health_check_timeout_s",
             "graceful_shutdown_wait_loop_s", "graceful_shutdown_timeout_s", "route_prefix", "version",
             "max_queued_requests", "placement_group_bundles", "placement_group_strategy", "logging_config",
             "max_replicas_per_node"}


class Deployment:
    def __init__(self, body, name: str, config: Dict):
        self._body = body
        self.name = name
        self._config = config

    @property
    def func_or_class(self):
        return self._body

    @property
    def num_replicas(self):
        return self._config.get("num_replicas", 1)

    @property
    def user_config(self):
        return self._config.get("user_config")

    @property
    def max_ongoing_requests(self):
        return self._config.get("max_ongoing_requests", 5)

    @property
    def max_concurrent_queries(self):  # the pre-2.10 name of max_ongoing_requests
        return self.max_ongoing_requests

    @property
    def max_queued_requests(self):
        return self._config.get("max_queued_requests", -1)

    @property
    def version(self):
        return self._config.get("version")

    @property
    def ray_actor_options(self):
        return self._config.get("ray_actor_options")

    @property
    def route_prefix(self):
        return self._config.get("route_prefix")

    @property
    def url(self):
        """HTTP URL of an ingress deployment, None without a route prefix (reference ``url``)."""
        rp = self.route_prefix
        if rp is None:
            return None
        from ._private import proxy

        host, port = getattr(proxy, "DEFAULT_HTTP_HOST", "127.0.0.1"), getattr(proxy, "DEFAULT_HTTP_PORT", 8000)
        return f"http://{host}:{port}{rp}"

    @property
    def init_args(self):
        return tuple(self._config.get("init_args") or ())

    @property
    def init_kwargs(self):
        return dict(self._config.get("init_kwargs") or {})

    @property
    def logging_config(self):
        return self._config.get("logging_config")

    def set_logging_config(self, logging_config) -> None:
        self._config["logging_config"] = logging_config

    def options(self, **kw) -> "Deployment":
        bad = set(kw) - _DEP_OPTS
        if bad:
            raise ValueError(f"invalid deployment options {bad}")
        cfg = dict(self._config)
        cfg.update(kw)
        return Deployment(self._body, kw.get("name", self.name), cfg)

    def bind(self, *args, **kwargs) -> "Application":
        return Application(self, args, kwargs)

    def __call__(self, *a, **k):
        raise RuntimeError("Deployments cannot be constructed directly. Use `deployment.bind()` instead.")


class Application:
    def __init__(self, deployment: Deployment, args, kwargs):
        self._deployment = deployment
        self._args = args
        self._kwargs = kwargs

    def _collect(self, app_name, out: Dict[str, Dict]):
        """Flatten the bound graph into deployment specs (children first)."""

        def conv(x):
            if isinstance(x, Application):
                n = x._collect(app_name, out)
                return _HandleSpec(app_name, n)
            return x

        args = tuple(conv(a) for a in self._args)
        kwargs = {k: conv(v) for k, v in self._kwargs.items()}
        d = self._deployment
        name = d.name
        if name in out and out[name]["_app"] is not self:
            i = 1
            while f"{name}_{i}" in out:
                i += 1
            name = f"{name}_{i}"
        blob = ser.dumps_function(d._body)
        cfg = d._config
        init_blob = ser.serialize((args, kwargs)).to_bytes()
        ac = cfg.get("autoscaling_config")
        if ac is not None and not isinstance(ac, dict):
            ac = dict(ac.__dict__)
        out[name] = {"name": name, "body": blob, "body_hash": hashlib.sha1(blob).hexdigest(),
                     "init_args": args, "init_kwargs": kwargs, "init_args_blob": hashlib.sha1(init_blob).hexdigest(),
                     "is_function": not inspect.isclass(d._body),
                     "num_replicas": 1 if cfg.get("num_replicas") in (None, "auto") else int(cfg["num_replicas"]),
                     "actor_options": dict(cfg.get("ray_actor_options") or {}),
                     "max_ongoing_requests": cfg.get("max_ongoing_requests") or cfg.get("max_concurrent_queries") or 5,
                     "autoscaling_config": ac if ac else ({"min_replicas": 1, "max_replicas": 100,
                                                           "target_ongoing_requests": 2}
                                                          if cfg.get("num_replicas") == "auto" else None),
                     "user_config": cfg.get("user_config"), "_app": self,
                     **_lifecycle_options(cfg), **_placement_options(cfg)}
        return name


def _logging_dict(lc) -> Optional[Dict]:
    """``LoggingConfig`` (model or dict) -> plain dict with the reference defaults filled in."""
    if lc is None:
        return None
    if not isinstance(lc, dict):
        lc = lc.model_dump() if hasattr(lc, "model_dump") else dict(lc.__dict__)
    from .schema import LoggingConfig

    return LoggingConfig(**lc).model_dump()


def _placement_options(cfg: Dict) -> Dict:
    """Replica placement (reference: serve/_private/deployment_scheduler.py): every replica gets a
    placement group of ``placement_group_bundles`` (the replica actor in bundle 0) with
    ``placement_group_strategy``; ``max_replicas_per_node`` caps replicas per node."""
    bundles = cfg.get("placement_group_bundles")
    strategy = cfg.get("placement_group_strategy")
    mrpn = cfg.get("max_replicas_per_node")
    if strategy is not None and bundles is None:
        raise ValueError("placement_group_strategy is set but placement_group_bundles is not")
    if bundles is not None:
        if not isinstance(bundles, (list, tuple)) or not bundles or not all(isinstance(b, dict) for b in bundles):
            raise ValueError("placement_group_bundles must be a non-empty list of resource dicts")
        bundles = [{k: float(v) for k, v in b.items()} for b in bundles]
        strategy = strategy or "PACK"
        if strategy not in ("PACK", "SPREAD", "STRICT_PACK", "STRICT_SPREAD"):
            raise ValueError(f"invalid placement_group_strategy {strategy!r}")
        opts = cfg.get("ray_actor_options") or {}
        need = {"CPU": float(opts.get("num_cpus", 0) or 0), "GPU": float(opts.get("num_gpus", 0) or 0)}
        need.update({k: float(v) for k, v in (opts.get("resources") or {}).items()})
        for k, v in need.items():
            if v > 0 and bundles[0].get(k, 0.0) < v:
                raise ValueError(f"the replica actor needs {k}={v} but placement_group_bundles[0] has "
                                 f"{bundles[0].get(k, 0.0)}: the actor runs in the first bundle")
    if mrpn is not None:
        mrpn = int(mrpn)
        if mrpn < 1:
            raise ValueError("max_replicas_per_node must be >= 1")
        if bundles is not None:
            raise ValueError("max_replicas_per_node cannot be combined with placement_group_bundles")
    return {"placement_group_bundles": bundles, "placement_group_strategy": strategy,
            "max_replicas_per_node": mrpn, "logging_config": _logging_dict(cfg.get("logging_config"))}


# replica lifecycle options and their reference defaults (serve/config.py DeploymentConfig)
_LIFECYCLE_DEFAULTS = {"max_queued_requests": -1, "health_check_period_s": 10.0, "health_check_timeout_s": 30.0,
                       "graceful_shutdown_wait_loop_s": 2.0, "graceful_shutdown_timeout_s": 20.0}


def _lifecycle_options(cfg: Dict) -> Dict:
    out = {}
    for k, d in _LIFECYCLE_DEFAULTS.items():
        v = cfg.get(k)
        out[k] = d if v is None else (int(v) if k == "max_queued_requests" else float(v))
    return out


def deployment(_func_or_class=None, *, name: Optional[str] = None, num_replicas: Union[int, str, None] = None,
               ray_actor_options: Optional[Dict] = None, max_ongoing_requests: Optional[int] = None,
               max_concurrent_queries: Optional[int] = None, autoscaling_config=None, user_config=None,
               health_check_period_s=None, health_check_timeout_s=None, graceful_shutdown_wait_loop_s=None,
               graceful_shutdown_timeout_s=None, route_prefix=None, version=None, max_queued_requests=None,
               placement_group_bundles=None, placement_group_strategy=None, logging_config=None,
               max_replicas_per_node=None):
    cfg = {k: v for k, v in dict(num_replicas=num_replicas, ray_actor_options=ray_actor_options,
                                 max_ongoing_requests=max_ongoing_requests or max_concurrent_queries,
                                 autoscaling_config=autoscaling_config, user_config=user_config,
                                 max_queued_requests=max_queued_requests,
                                 health_check_period_s=health_check_period_s,
                                 health_check_timeout_s=health_check_timeout_s,
                                 graceful_shutdown_wait_loop_s=graceful_shutdown_wait_loop_s,
                                 graceful_shutdown_timeout_s=graceful_shutdown_timeout_s,
                                 placement_group_bundles=placement_group_bundles,
                                 placement_group_strategy=placement_group_strategy,
                                 max_replicas_per_node=max_replicas_per_node,
                                 logging_config=logging_config, version=version,
                                 route_prefix=route_prefix).items()
           if v is not None}
    _placement_options(cfg)  # validate at decoration time, as the reference does
    if num_replicas is not None and autoscaling_config is not None and num_replicas != "auto":
        raise ValueError("Manually setting num_replicas is not allowed when autoscaling_config is provided.")

    def deco(body):
        return Deployment(body, name or body.__name__, cfg)

    return deco(_func_or_class) if _func_or_class is not None else deco


# ------------------------------------------------------------------------------ controller
def _get_controller():
    from .._private import worker as w
    from ..actor import ActorClass

    if not w.is_initialized():
        w.init()
    c = _STATE["controller"]
    if c is not None:
        return c
    try:
        c = w.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
    except ValueError:
        c = ActorClass(ServeController, {"name": CONTROLLER_NAME, "namespace": NAMESPACE, "lifetime": "detached",
                                         "num_cpus": 0, "max_concurrency": 1000}).options(get_if_exists=True).remote()
    _STATE["controller"] = c
    return c


def start(http_options: Optional[Dict] = None, detached: bool = True, proxy_location=None, grpc_options=None, **kw):
    """``grpc_options``: ``serve.config.gRPCOptions`` or a dict with ``port`` (and ``host``) and
    ``grpc_servicer_functions`` (``add_<Service>Servicer_to_server`` callables or import paths)."""
    if http_options:
        if not isinstance(http_options, dict):
            http_options = {k: getattr(http_options, k, None)
                            for k in ("host", "port", "request_timeout_s", "keep_alive_timeout_s", "root_path")}
        _STATE["http"].update({k: v for k, v in http_options.items()
                               if k in ("host", "port", "request_timeout_s", "keep_alive_timeout_s", "root_path")
                               and v is not None})
    if grpc_options is not None:
        if not isinstance(grpc_options, dict):
            grpc_options = {"host": getattr(grpc_options, "host", "127.0.0.1"), "port": grpc_options.port,
                            "grpc_servicer_functions": list(grpc_options.grpc_servicer_functions)}
        _STATE["grpc"] = {"host": grpc_options.get("host", "127.0.0.1"), "port": int(grpc_options.get("port", 9000)),
                          "grpc_servicer_functions": list(grpc_options.get("grpc_servicer_functions", []))}
    _get_controller()
    if _STATE["grpc"] is not None:
        _ensure_grpc_proxy()


def _ensure_grpc_proxy():
    from .._private import worker as w
    from ..actor import ActorClass
    from ._private.grpc_proxy import gRPCProxy

    if _STATE["grpc_proxy"] is not None or _STATE["grpc"] is None:
        return
    g = _STATE["grpc"]
    try:
        p = w.get_actor("SERVE_GRPC_PROXY_ACTOR", namespace=NAMESPACE)
    except ValueError:
        p = ActorClass(gRPCProxy, {"name": "SERVE_GRPC_PROXY_ACTOR", "namespace": NAMESPACE, "lifetime": "detached",
                                   "num_cpus": 0, "max_concurrency": 100}).remote(
            g["host"], g["port"], g["grpc_servicer_functions"])
    _STATE["grpc_info"] = w.get(p.ready.remote())
    _STATE["grpc_proxy"] = p


def _ensure_proxy():
    from .._private import worker as w
    from ..actor import ActorClass
    from ._private.proxy import HTTPProxy

    if _STATE["proxy"] is not None:
        return
    h = _STATE["http"]
    try:
        p = w.get_actor("SERVE_PROXY_ACTOR", namespace=NAMESPACE)
    except ValueError:
        p = ActorClass(HTTPProxy, {"name": "SERVE_PROXY_ACTOR", "namespace": NAMESPACE, "lifetime": "detached",
                                   "num_cpus": 0, "max_concurrency": 100}).remote(
            h["host"], h["port"], h.get("request_timeout_s"), h.get("keep_alive_timeout_s", 5), h.get("root_path", ""))
    w.get(p.ready.remote())
    _STATE["proxy"] = p


def run(target: Union[Application, Deployment], *, name: str = "default", route_prefix: Optional[str] = "/",
        blocking: bool = False, _blocking: bool = True, logging_config=None, http: bool = True,
        **kw) -> DeploymentHandle:
    from .._private import worker as w

    if isinstance(target, Deployment):
        target = target.bind()
    if not isinstance(target, Application):
        raise TypeError("serve.run expects an Application (deployment.bind(...))")
    specs: Dict[str, Dict] = {}
    ingress = target._collect(name, specs)
    app_logging = _logging_dict(logging_config)
    for s in specs.values():
        s.pop("_app", None)
        if s.get("logging_config") is None:
            s["logging_config"] = app_logging  # the application-level default
    ctrl = _get_controller()
    w.get(ctrl.deploy_application.remote(name, list(specs.values()), ingress, route_prefix))
    status = w.get(ctrl.wait_app_running.remote(name, 300.0))
    if status != "RUNNING":
        st = w.get(ctrl.status.remote())
        raise RuntimeError(f"Deploying app '{name}' failed: {st.get(name)}")
    if http and route_prefix is not None:
        _ensure_proxy()
    if _STATE["grpc"] is not None:
        _ensure_grpc_proxy()
    handle = DeploymentHandle(ingress, name)
    if blocking:
        while True:
            time.sleep(1)
    return handle


def delete(name: str, _blocking: bool = True):
    from .._private import worker as w

    w.get(_get_controller().delete_application.remote(name))


def status():
    from .._private import worker as w

    return _ServeStatus(w.get(_get_controller().status.remote()))


class _ServeStatus(dict):
    """``serve.status()``: the reference ``ServeStatus`` attributes (``applications`` ->
    ``status`` / ``message`` / ``deployments`` -> ``status`` / ``replica_states`` / ``message``)
    over the controller's plain dict, which stays readable by key."""

    @property
    def applications(self):
        return {k: _AppStatus(v) for k, v in self.items()}

    @property
    def proxies(self):
        return {}

    @property
    def target_capacity(self):
        return None


class _AppStatus(dict):
    @property
    def status(self):
        return self["status"]

    @property
    def message(self):
        return self.get("message") or ""

    @property
    def deployments(self):
        return {k: _DeploymentStatus(v) for k, v in self["deployments"].items()}


class _DeploymentStatus(dict):
    @property
    def status(self):
        return self["status"]

    @property
    def message(self):
        return self.get("message") or ""

    @property
    def replica_states(self):
        return {"RUNNING": int(self.get("replicas", 0))}


def shutdown():
    from .._private import worker as w

    # the next serve.start() begins from the default HTTP options again (a request_timeout_s or
    # port given to this instance must not leak into a later one in the same process)
    _STATE["http"] = {"host": "127.0.0.1", "port": 8000}
    if not w.is_initialized():
        _STATE.update(controller=None, proxy=None, grpc_proxy=None, grpc=None)
        return
    try:
        c = _STATE["controller"] or w.get_actor(CONTROLLER_NAME, namespace=NAMESPACE)
        w.get(c.shutdown.remote())
        w.kill(c)
    except Exception:
        pass
    try:
        p = _STATE["proxy"] or w.get_actor("SERVE_PROXY_ACTOR", namespace=NAMESPACE)
        w.get(p.shutdown.remote())
        w.kill(p)
    except Exception:
        pass
    try:
        g = _STATE["grpc_proxy"]
        if g is None and _STATE["grpc"] is not None:
            g = w.get_actor("SERVE_GRPC_PROXY_ACTOR", namespace=NAMESPACE)
        if g is not None:
            w.get(g.shutdown.remote())
            w.kill(g)
    except Exception:
        pass
    _STATE["controller"] = None
    _STATE["proxy"] = None
    _STATE["grpc_proxy"] = None
    _STATE["grpc"] = None
    from .handle import _Router

    _Router._routers.clear()


def get_app_handle(name: str) -> DeploymentHandle:
    from .._private import worker as w

    ingress = w.get(_get_controller().get_ingress.remote(name))
    if ingress is None:
        raise ValueError(f"Application '{name}' does not exist.")
    return DeploymentHandle(ingress, name)


def get_deployment_handle(deployment_name: str, app_name: Optional[str] = None) -> DeploymentHandle:
    return DeploymentHandle(deployment_name, app_name or "default")


def get_replica_context():
    from ._private.replica import _REPLICA_CTX

    ctx = _REPLICA_CTX.get("ctx")
    if ctx is None:
        raise RuntimeError("`serve.get_replica_context()` may only be called from within a Serve replica.")
    return ctx


# ------------------------------------------------------------------------------ ingress
def ingress(app):
    """Class decorator serving a FastAPI app from the deployment (``@serve.ingress(app)``).

    The FastAPI object itself is never shipped to replicas (its pydantic/starlette internals do
    not survive pickling by value); instead the route table is captured as a picklable recipe and
    each replica rebuilds an app whose class routes are bound to the replica's instance."""

    def deco(cls):
        cls._serve_ingress_spec = _capture_routes(app, cls)
        return cls

    return deco


def _capture_routes(app, cls):
    try:
        from fastapi.routing import APIRoute, APIWebSocketRoute
    except ImportError:
        raise ImportError("@serve.ingress requires fastapi")
    meta = {k: getattr(app, k, None) for k in ("title", "version", "description")}
    routes = []
    for r in app.router.routes:
        if isinstance(r, APIWebSocketRoute):
            fn = r.endpoint
            is_method = getattr(fn, "__qualname__", "").startswith(cls.__qualname__ + ".")
            routes.append({"kind": "websocket", "path": r.path, "endpoint": fn.__name__ if is_method else fn,
                           "is_method": is_method, "name": r.name})
            continue
        if not isinstance(r, APIRoute):
            continue  # docs/openapi routes are recreated by the replica's FastAPI()
        fn = r.endpoint
        is_method = getattr(fn, "__qualname__", "").startswith(cls.__qualname__ + ".")
        routes.append({"path": r.path, "endpoint": fn.__name__ if is_method else fn, "is_method": is_method,
                       "methods": sorted(r.methods or ()), "name": r.name, "status_code": r.status_code,
                       "response_model": r.response_model, "tags": list(r.tags or [])})
    return {"meta": meta, "routes": routes}


def _build_ingress_app(spec, instance):
    from fastapi import FastAPI

    app = FastAPI(**{k: v for k, v in spec["meta"].items() if v is not None})
    for r in spec["routes"]:
        ep = getattr(instance, r["endpoint"]) if r["is_method"] else r["endpoint"]
        if r.get("kind") == "websocket":
            app.add_api_websocket_route(r["path"], ep, name=r["name"])
            continue
        app.add_api_route(r["path"], ep, methods=r["methods"], name=r["name"], status_code=r["status_code"],
                          response_model=r["response_model"], tags=r["tags"] or None)
    return app
