"""Applying a declarative Serve config (reference: ``serve/_private/api.py`` ``serve_start`` +
``client.deploy_apps``, the controller's ``build_serve_application`` task in
``serve/_private/application_state.py``, and ``serve/scripts.py`` ``deploy`` / ``run`` / ``build``).

Each application is BUILT in a task that runs in the application's ``runtime_env`` (so a
``working_dir`` / ``py_modules`` holding the user's code is importable there, not necessarily in
the process applying the config): it imports ``import_path``, calls it with ``args`` if it is an
application builder, flattens the bound graph into deployment specs and applies the config's
per-deployment overrides. The specs (code blobs, init args, options) come back to the caller,
which hands them to the controller; replicas inherit the application's ``runtime_env``.
"""
from __future__ import annotations

import importlib
import time
from typing import Any, Dict, List, Optional, Tuple

_OVERRIDABLE = ("num_replicas", "max_ongoing_requests", "max_concurrent_queries", "user_config",
                "autoscaling_config", "ray_actor_options", "max_queued_requests", "health_check_period_s",
                "health_check_timeout_s", "graceful_shutdown_wait_loop_s", "graceful_shutdown_timeout_s",
                "placement_group_bundles", "placement_group_strategy", "logging_config", "route_prefix",
                "max_replicas_per_node")


def import_attr(path: str):
    """``module:attr.sub`` or ``module.attr``."""
    if ":" in path:
        mod, attr = path.split(":", 1)
    else:
        mod, attr = path.rsplit(".", 1)
    obj = importlib.import_module(mod)
    for part in attr.split("."):
        obj = getattr(obj, part)
    return obj


def build_application(import_path: str, args: Optional[Dict[str, Any]] = None):
    """The bound ``Application`` an import path names: an ``Application`` as is, a
    ``Deployment`` bound with no arguments, or a builder function called with ``args``."""
    from ..api import Application, Deployment

    target = import_attr(import_path)
    if isinstance(target, Deployment):
        if args:
            raise ValueError(f"{import_path} is a deployment, not an application builder: it takes no args")
        return target.bind()
    if isinstance(target, Application):
        if args:
            raise ValueError(f"{import_path} is an already bound application: it takes no args")
        return target
    if callable(target):
        app = target(dict(args or {}))
        if isinstance(app, Deployment):
            app = app.bind()
        if not isinstance(app, Application):
            raise TypeError(f"application builder {import_path} returned {type(app).__name__}, not an Application")
        return app
    raise TypeError(f"{import_path} is neither an Application, a Deployment nor an application builder")


def _merge_actor_options(base: Dict[str, Any], override: Dict[str, Any], app_env: Dict[str, Any]) -> Dict[str, Any]:
    out = dict(base)
    for k, v in (override or {}).items():
        if v is None or (k in ("runtime_env", "resources") and v == {}):
            continue
        out[k] = v
    env = dict(app_env or {})
    env.update(out.get("runtime_env") or {})
    if env:
        out["runtime_env"] = env
    return out


def build_specs(app_cfg: Dict[str, Any]) -> Tuple[List[Dict[str, Any]], str]:
    """(deployment specs, ingress name) of one application config (a ``ServeApplicationSchema``
    dict), overrides applied. Raises on an override naming a deployment the app does not have."""
    app = build_application(app_cfg["import_path"], app_cfg.get("args"))
    specs: Dict[str, Dict] = {}
    ingress = app._collect(app_cfg.get("name", "default"), specs)
    for s in specs.values():
        s.pop("_app", None)
    env = app_cfg.get("runtime_env") or {}
    # code version of a config-deployed app: the same import path, env and builder args build the
    # same code, so a re-deploy that only changes options does not restart replicas (their pickled
    # bodies can differ byte-wise between builds in different processes)
    import hashlib
    import json

    code_version = hashlib.sha1(json.dumps([app_cfg["import_path"], env, app_cfg.get("args") or {}],
                                           sort_keys=True, default=str).encode()).hexdigest()
    overrides = {d["name"]: d for d in app_cfg.get("deployments") or ()}
    unknown = set(overrides) - set(specs)
    if unknown:
        raise ValueError(f"the config overrides deployment(s) {sorted(unknown)} that application "
                         f"{app_cfg.get('name', 'default')!r} does not have (it has {sorted(specs)})")
    for name, s in specs.items():
        o = overrides.get(name, {})
        if o.get("num_replicas") is not None:
            if o["num_replicas"] == "auto":
                s["num_replicas"] = 1
                s["autoscaling_config"] = s.get("autoscaling_config") or {
                    "min_replicas": 1, "max_replicas": 100, "target_ongoing_requests": 2}
            else:
                s["num_replicas"] = int(o["num_replicas"])
                s["autoscaling_config"] = None
        if o.get("autoscaling_config") is not None:
            s["autoscaling_config"] = dict(o["autoscaling_config"])
        mo = o.get("max_ongoing_requests") or o.get("max_concurrent_queries")
        if mo:
            s["max_ongoing_requests"] = int(mo)
        if "user_config" in o:
            s["user_config"] = o["user_config"]
        from ..api import _LIFECYCLE_DEFAULTS, _lifecycle_options

        s.update(_lifecycle_options({k: o.get(k, s.get(k)) for k in _LIFECYCLE_DEFAULTS}))
        s["actor_options"] = _merge_actor_options(s.get("actor_options") or {}, o.get("ray_actor_options") or {}, env)
        from ..api import _placement_options

        placement = {k: (o[k] if o.get(k) is not None else s.get(k))
                     for k in ("placement_group_bundles", "placement_group_strategy", "max_replicas_per_node",
                               "logging_config")}
        if o.get("logging_config") is None and app_cfg.get("logging_config") is not None:
            placement["logging_config"] = app_cfg["logging_config"]  # application-level default
        s.update(_placement_options(dict(placement, ray_actor_options=s["actor_options"])))
        s["code_version"] = code_version
    return list(specs.values()), ingress


def _build_remote():
    from ... import remote

    @remote(num_cpus=0, max_retries=0)
    def _build_serve_application(app_cfg):
        return build_specs(app_cfg)

    return _build_serve_application


def build_specs_in_env(app_cfg: Dict[str, Any]):
    """``build_specs`` inside a task running in the application's runtime_env."""
    from ..._private.worker import get

    fn = _build_remote()
    env = app_cfg.get("runtime_env") or None
    return get((fn.options(runtime_env=env) if env else fn).remote(app_cfg))


def deploy_config(config, wait_running: bool = False, timeout_s: float = 300.0) -> Dict[str, str]:
    """Apply a ``ServeDeploySchema`` declaratively. Returns {app: status}."""
    from ..._private.worker import get
    from .. import api
    from ..schema import ProxyLocation, ServeDeploySchema

    if not isinstance(config, ServeDeploySchema):
        config = ServeDeploySchema.model_validate(config)
    grpc = config.grpc_options
    api.start(http_options={"host": config.http_options.host, "port": config.http_options.port},
              grpc_options=({"port": grpc.port, "grpc_servicer_functions": list(grpc.grpc_servicer_functions)}
                            if grpc.grpc_servicer_functions else None))
    ctrl = api._get_controller()
    built = []
    for app in config.applications:  # build every app first: a bad one deploys nothing
        cfg = app.model_dump(mode="json")
        specs, ingress = build_specs_in_env(cfg)
        built.append((app, cfg, specs, ingress))
    existing = set(get(ctrl.list_applications.remote()))
    for app, cfg, specs, ingress in built:
        get(ctrl.deploy_application.remote(app.name, specs, ingress, app.route_prefix, cfg))
    for name in existing - {a.name for a in config.applications}:
        get(ctrl.delete_application.remote(name))
    get(ctrl.set_deploy_config.remote(config.model_dump(mode="json", exclude_unset=True)))
    if config.proxy_location != ProxyLocation.Disabled and any(a.route_prefix for a in config.applications):
        api._ensure_proxy()
    out = {}
    for app in config.applications:
        out[app.name] = get(ctrl.wait_app_running.remote(app.name, timeout_s)) if wait_running else "DEPLOYING"
    return out


def build_config(import_paths: List[str], app_dir: Optional[str] = None) -> Dict[str, Any]:
    """``serve build``: a deployable config for the given import paths, every deployment listed
    with the options its code sets (edit the numbers, then ``serve deploy`` the file)."""
    import sys

    if app_dir:
        sys.path.insert(0, app_dir)
    apps = []
    multi = len(import_paths) > 1
    for i, path in enumerate(import_paths):
        name = path.replace(":", ".").split(".")[-1] if multi else "app1"
        app = build_application(path)
        specs: Dict[str, Dict] = {}
        app._collect(name, specs)
        deps = []
        for s in specs.values():
            d = {"name": s["name"], "num_replicas": s["num_replicas"] if not s.get("autoscaling_config") else "auto",
                 "max_ongoing_requests": s.get("max_ongoing_requests", 5)}
            if s.get("user_config") is not None:
                d["user_config"] = s["user_config"]
            if s.get("autoscaling_config"):
                d.pop("num_replicas")
                d["autoscaling_config"] = s["autoscaling_config"]
            if s.get("actor_options"):
                d["ray_actor_options"] = {k: v for k, v in s["actor_options"].items() if k != "runtime_env"}
            deps.append(d)
        apps.append({"name": name, "route_prefix": "/" if not multi else f"/{name}", "import_path": path,
                     "runtime_env": {}, "deployments": deps})
    return {"proxy_location": "EveryNode", "http_options": {"host": "0.0.0.0", "port": 8000},
            "grpc_options": {"port": 9000, "grpc_servicer_functions": []}, "applications": apps}


def wait_for_status(names, timeout_s: float = 300.0) -> Dict[str, str]:
    from ..._private.worker import get
    from .. import api

    ctrl = api._get_controller()
    deadline = time.time() + timeout_s
    out = {}
    for n in names:
        out[n] = get(ctrl.wait_app_running.remote(n, max(0.0, deadline - time.time())))
    return out
