"""``import ray`` compatibility alias for :mod:`ray_community_amd`.

User code written against the reference (``import ray``, ``from ray import train, tune``,
``from ray.rllib.algorithms.ppo import PPOConfig``, ``ray.util.collective`` ...) runs unchanged:
``ray`` IS the ``ray_community_amd`` module object and every ``ray.<sub>`` import resolves to the
very same module object as ``ray_community_amd.<sub>`` (no duplicate classes, so isinstance checks,
pickling and registries agree between the two spellings).
"""
import importlib
import importlib.abc
import importlib.util
import sys

_PKG = "ray_community_amd"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target: str):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):  # already executed under its real name
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith("ray."):
            return None
        real = _PKG + fullname[3:]
        if importlib.util.find_spec(real) is None:
            return None
        return importlib.util.spec_from_loader(fullname, _AliasLoader(real))


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

sys.modules[__name__] = importlib.import_module(_PKG)
