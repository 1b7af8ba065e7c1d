"""Runtime environments (reference: ``python/ray/runtime_env/runtime_env.py``).

Supported fields (applied by the head when it starts a worker process for the env):
  * ``env_vars``      — dict of environment variables;
  * ``working_dir``   — local directory or ``.zip`` archive (unpacked once per session); the
                        worker chdirs into it and puts it first on ``sys.path``;
  * ``py_modules``    — local package directories / files added to ``sys.path``;
  * ``worker_process_setup_hook`` — ``"module.function"`` (or a callable) run at worker start;
  * ``pip`` / ``conda`` — there is no package index on the target machines, so these are
                        validated against what is importable instead of being installed; a
                        missing requirement fails the task with ``RuntimeEnvSetupError``.
Workers are pooled per distinct runtime env, so tasks with different envs never share a process.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Optional, Union

_KNOWN = {"env_vars", "working_dir", "py_modules", "pip", "conda", "container", "config", "excludes",
          "worker_process_setup_hook", "nsight", "image_uri", "_rca_setup_hook_blob"}


class RuntimeEnvSetupError(RuntimeError):
    pass


class RuntimeEnvConfig(dict):
    def __init__(self, setup_timeout_seconds: int = 600, eager_install: bool = True):
        if not isinstance(setup_timeout_seconds, int) or (setup_timeout_seconds <= 0 and setup_timeout_seconds != -1):
            raise ValueError("setup_timeout_seconds must be a positive int or -1")
        super().__init__(setup_timeout_seconds=setup_timeout_seconds, eager_install=bool(eager_install))


class RuntimeEnv(dict):
    def __init__(self, *, env_vars: Optional[Dict[str, str]] = None, working_dir: Optional[str] = None,
                 py_modules: Optional[List[str]] = None, pip: Union[None, List[str], Dict] = None,
                 conda: Union[None, str, Dict] = None, config: Optional[Dict] = None,
                 worker_process_setup_hook=None, **kwargs):
        super().__init__()
        unknown = set(kwargs) - _KNOWN
        if unknown:
            raise ValueError(f"unknown runtime_env field(s): {sorted(unknown)}")
        if env_vars is not None:
            if not isinstance(env_vars, dict) or not all(isinstance(k, str) and isinstance(v, str)
                                                         for k, v in env_vars.items()):
                raise TypeError("runtime_env['env_vars'] must be a Dict[str, str]")
            self["env_vars"] = dict(env_vars)
        if working_dir is not None:
            if not isinstance(working_dir, str):
                raise TypeError("runtime_env['working_dir'] must be a path string")
            self["working_dir"] = working_dir
        if py_modules is not None:
            if not isinstance(py_modules, (list, tuple)):
                raise TypeError("runtime_env['py_modules'] must be a list")
            self["py_modules"] = [str(p) if not hasattr(p, "__file__") else os.path.dirname(p.__file__)
                                  for p in py_modules]
        if pip is not None and conda is not None:
            raise ValueError("runtime_env cannot specify both 'pip' and 'conda'")
        if pip is not None:
            self["pip"] = pip
        if conda is not None:
            self["conda"] = conda
        if config is not None:
            self["config"] = dict(config)
        if worker_process_setup_hook is not None:
            if callable(worker_process_setup_hook):
                from ._private import serialization as ser

                self["_rca_setup_hook_blob"] = ser.dumps_function(worker_process_setup_hook).hex()
            elif isinstance(worker_process_setup_hook, str):
                self["worker_process_setup_hook"] = worker_process_setup_hook
            else:
                raise TypeError("worker_process_setup_hook must be a callable or 'module.function'")
        for k in ("container", "excludes", "nsight", "image_uri", "_rca_setup_hook_blob"):
            if k in kwargs:
                self[k] = kwargs[k]

    def env_vars(self) -> Dict[str, str]:
        return dict(self.get("env_vars") or {})

    def working_dir(self) -> Optional[str]:
        return self.get("working_dir")

    def py_modules(self) -> List[str]:
        return list(self.get("py_modules") or [])

    def pip_config(self) -> Dict:
        pip = self.get("pip")
        if pip is None:
            return {}
        if isinstance(pip, dict):
            return pip
        return {"packages": list(pip)}

    # ---- the reference's accessors (runtime_env/runtime_env.py). Environments are local
    # directories and env vars here: the uri getters return the local paths, and the fields
    # that need conda / containers / MPI / Nsight report what the dict holds.
    def set(self, name: str, value: Any) -> None:
        if name not in _KNOWN and name not in ("env_vars", "working_dir", "py_modules", "pip", "conda", "config"):
            raise ValueError(f"unknown runtime_env field {name!r}")
        self[name] = value

    def has_working_dir(self) -> bool:
        return self.get("working_dir") is not None

    def working_dir_uri(self) -> Optional[str]:
        return self.get("working_dir")

    def py_modules_uris(self) -> List[str]:
        return self.py_modules()

    def has_pip(self) -> bool:
        return self.get("pip") is not None

    def pip_uri(self) -> Optional[str]:
        return None

    def has_conda(self) -> bool:
        return self.get("conda") is not None

    def conda_uri(self) -> Optional[str]:
        return None

    def conda_env_name(self) -> Optional[str]:
        c = self.get("conda")
        return c if isinstance(c, str) else None

    def conda_config(self) -> Optional[str]:
        c = self.get("conda")
        return json.dumps(c, sort_keys=True) if isinstance(c, dict) else None

    def virtualenv_name(self) -> Optional[str]:
        return None

    def plugin_uris(self) -> List[str]:
        return []

    def plugins(self) -> List:
        return []

    def java_jars(self) -> List[str]:
        return list(self.get("java_jars") or [])

    def mpi(self) -> Optional[Dict]:
        return self.get("mpi")

    def nsight(self) -> Optional[Any]:
        return self.get("nsight")

    def has_py_container(self) -> bool:
        return bool(self.get("container"))

    def py_container_image(self) -> Optional[str]:
        return (self.get("container") or {}).get("image")

    def py_container_worker_path(self) -> Optional[str]:
        return (self.get("container") or {}).get("worker_path")

    def py_container_run_options(self) -> List:
        return list((self.get("container") or {}).get("run_options") or [])

    def get_extension(self, key, default=None):
        return self.get(key, default)

    def to_dict(self) -> Dict[str, Any]:
        return dict(self)

    def serialize(self) -> str:
        return json.dumps(self, sort_keys=True, default=str)

    @classmethod
    def deserialize(cls, s: str) -> "RuntimeEnv":
        return cls(**json.loads(s))


def validate(env) -> Optional[Dict]:
    if env is None:
        return None
    if isinstance(env, RuntimeEnv):
        return dict(env)
    if not isinstance(env, dict):
        raise TypeError(f"runtime_env must be a dict or RuntimeEnv, got {type(env).__name__}")
    hook = env.get("worker_process_setup_hook")
    rest = {k: v for k, v in env.items() if k != "worker_process_setup_hook"}
    return dict(RuntimeEnv(**rest, worker_process_setup_hook=hook))


def _requirement_names(pip) -> List[str]:
    pkgs = pip.get("packages", []) if isinstance(pip, dict) else list(pip or [])
    names = []
    for p in pkgs:
        n = str(p).strip()
        for sep in ("==", ">=", "<=", "~=", ">", "<", "[", ";", " "):
            n = n.split(sep)[0]
        if n:
            names.append(n)
    return names


def check_requirements(env: Dict):
    """Worker-side: pip/conda specs cannot be installed offline; they must already be importable."""
    import importlib.metadata as md

    missing = []
    for name in _requirement_names(env.get("pip")):
        try:
            md.version(name)
        except md.PackageNotFoundError:
            missing.append(name)
    if missing:
        raise RuntimeEnvSetupError(f"runtime_env pip requirement(s) not available on this node (no package "
                                   f"index): {missing}")


def apply_setup_hook(env: Dict):
    blob = env.get("_rca_setup_hook_blob")
    if blob:
        from ._private import serialization as ser

        ser.loads_function(bytes.fromhex(blob))()
    hook = env.get("worker_process_setup_hook")
    if hook:
        import importlib

        mod, _, fn = hook.rpartition(".")
        getattr(importlib.import_module(mod), fn)()


def prepare_working_dir(path: str, session_dir: str) -> str:
    """Zip archives are unpacked once per session; directories are used in place."""
    if os.path.isdir(path):
        return os.path.abspath(path)
    if path.endswith(".zip") and os.path.isfile(path):
        import hashlib
        import zipfile

        h = hashlib.sha1(os.path.abspath(path).encode() + str(os.path.getmtime(path)).encode()).hexdigest()[:12]
        dest = os.path.join(session_dir, "runtime_resources", f"working_dir_{h}")
        if not os.path.isdir(dest):
            tmp = dest + f".tmp{os.getpid()}"
            with zipfile.ZipFile(path) as z:
                z.extractall(tmp)
            entries = os.listdir(tmp)
            root = os.path.join(tmp, entries[0]) if len(entries) == 1 and os.path.isdir(
                os.path.join(tmp, entries[0])) else tmp
            os.replace(root, dest) if root != tmp else os.replace(tmp, dest)
        return dest
    raise ValueError(f"working_dir {path!r} must be an existing directory or .zip file (no remote URIs offline)")


__all__ = ["RuntimeEnv", "RuntimeEnvConfig", "RuntimeEnvSetupError"]


def mpi_init():
    """The reference's MPI runtime-env hook (``runtime_env/mpi.py``); MPI workers are not part of
    this runtime, so this only checks that an MPI launch is not expected."""
    import os as _os

    if _os.environ.get("OMPI_COMM_WORLD_SIZE") or _os.environ.get("PMI_SIZE"):
        raise NotImplementedError("MPI-launched workers are not supported; use torch.distributed / RCCL")
