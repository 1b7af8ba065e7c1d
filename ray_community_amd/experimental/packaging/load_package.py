"""``load_package``: a self-contained code package with its own runtime environment (reference:
``python/ray/experimental/packaging/load_package.py``).

A package is a directory with a YAML config::

    name: my_package
    description: ...
    interface_file: my_pkg/stubs.py     # remote functions / actor classes the driver may call
    runtime_env: {env_vars: {...}, pip: [...], ...}

``load_package(path)`` imports the interface file in the DRIVER (which may not have the package's
dependencies, so the file may import only ``ray`` at top level -- lines marked ``# noqa`` are
exempt) and returns an object whose attributes are the file's remote functions and actor classes,
bound to the package's runtime environment: with no ``working_dir`` in it, the package directory
itself is shipped as the working directory, so the stubs' lazy imports of the package's modules
resolve in the workers. A ``conda.yaml`` next to the config becomes the ``conda`` field.
GitHub URLs need network access, which this framework does not assume: only local paths load.
"""
from __future__ import annotations

import importlib.util
import os
import re
from typing import Any, Dict

import yaml

_ALLOWED_IMPORT = re.compile(r"^import ray(\s*(#.*)?)?$")


def load_package(config_path: str) -> "_RuntimePackage":
    config_path = os.path.expanduser(config_path)
    if config_path.startswith(("http://", "https://")):
        raise ValueError("load_package(): remote (GitHub) packages need network access; pass a local "
                         "path to the package's YAML config")
    if not os.path.exists(config_path):
        raise ValueError(f"Config file does not exist: {config_path}")
    with open(config_path) as f:
        config = yaml.safe_load(f) or {}
    for key in ("name", "interface_file"):
        if key not in config:
            raise ValueError(f"package config {config_path} has no '{key}'")
    base_dir = os.path.abspath(os.path.dirname(config_path))
    runtime_env: Dict[str, Any] = dict(config.get("runtime_env") or {})
    if "working_dir" not in runtime_env:
        runtime_env["working_dir"] = base_dir
    conda_yaml = os.path.join(base_dir, "conda.yaml")
    if os.path.exists(conda_yaml):
        if "conda" in runtime_env:
            raise ValueError("Both conda.yaml and a conda: section found in the package")
        with open(conda_yaml) as f:
            runtime_env["conda"] = yaml.safe_load(f)
    return _RuntimePackage(config["name"], config.get("description", ""),
                           os.path.join(base_dir, config["interface_file"]), runtime_env)


class _RuntimePackage:
    """The interface file's remote functions and actor classes, bound to the package's runtime
    environment (``pkg.my_func.remote(...)``, ``pkg.MyActor.remote(...)``); the runtime env
    itself is ``pkg._runtime_env``."""

    def __init__(self, name: str, desc: str, interface_file: str, runtime_env: dict):
        from ...actor import ActorClass
        from ...remote_function import RemoteFunction

        self._name = name
        self._description = desc
        self._interface_file = interface_file
        self._runtime_env = runtime_env
        _validate_interface_file(interface_file)
        spec = importlib.util.spec_from_file_location(f"_rca_pkg_{name}", interface_file)
        module = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(module)
        self._module = module
        for symbol in dir(module):
            if symbol.startswith("_"):
                continue
            value = getattr(module, symbol)
            if isinstance(value, (RemoteFunction, ActorClass)):
                setattr(self, symbol, value.options(runtime_env=runtime_env))

    def __repr__(self):
        return f"_RuntimePackage(name={self._name!r}, module={self._module!r}, runtime_env={self._runtime_env!r})"


def _validate_interface_file(interface_file: str):
    if not os.path.exists(interface_file):
        raise ValueError(f"Interface file does not exist: {interface_file}")
    with open(interface_file) as f:
        for line in f:
            line = line.rstrip("\n")
            if line.startswith(("import ", "from ")) and not _ALLOWED_IMPORT.match(line) and "noqa" not in line:
                raise ValueError(f"Interface files may import only `ray` at top level, found `{line}`: make it a "
                                 "lazy import inside the function, or add `# noqa` to allow it")
