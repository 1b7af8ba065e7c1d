"""The reference's secondary module paths (``_private/import_paths.py``): every alias re-exports
the same objects as its defining module, and every optional-framework integration fails to
import with an ImportError that names the missing framework."""
import importlib

import pytest

import ray_community_amd  # noqa: F401 - installs the finder
from ray_community_amd._private import import_paths as ip


@pytest.mark.parametrize("alias", sorted(ip.ALIASES))
def test_alias_reexports_defining_module(alias):
    target, names = ip.ALIASES[alias]
    m = importlib.import_module(f"ray_community_amd.{alias}")
    src = importlib.import_module(f"ray_community_amd.{target}")
    assert m.__all__ == list(names) if names is not None else m.__all__
    for n in m.__all__:
        assert getattr(m, n) is getattr(src, n)


@pytest.mark.parametrize("pkg", sorted(ip.NEEDS))
def test_optional_integration_names_its_framework(pkg):
    with pytest.raises(ImportError, match=f"`{ip.NEEDS[pkg]}`"):
        importlib.import_module(f"ray_community_amd.{pkg}")


def test_unknown_submodule_still_fails_normally():
    with pytest.raises(ModuleNotFoundError):
        importlib.import_module("ray_community_amd.tune.no_such_module")
    from ray_community_amd.util.rpdb import set_trace
    from ray_community_amd.util.pdb import set_trace as st2

    assert set_trace is st2


@pytest.mark.parametrize("mod", sorted(ip.REMOVED))
def test_removed_apis_raise_deprecation(mod):
    with pytest.raises(DeprecationWarning, match="removed"):
        importlib.import_module(f"ray_community_amd.{mod}")
