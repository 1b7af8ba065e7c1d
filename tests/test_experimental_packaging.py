"""experimental.load_package (reference python/ray/experimental/packaging/load_package.py and its
example_pkg): the interface file's remote functions and actors run inside the package's runtime
environment, with the package directory shipped as the working directory."""
import textwrap

import pytest

import ray_community_amd as ray
from ray_community_amd.experimental import load_package


def _make_pkg(root, stubs):
    (root / "my_pkg").mkdir()
    (root / "my_pkg" / "__init__.py").write_text("")
    (root / "my_pkg" / "impl.py").write_text(textwrap.dedent("""
        import os

        def hello():
            return "hello from " + os.environ.get("PKG_MODE", "?")
    """))
    (root / "my_pkg" / "stubs.py").write_text(textwrap.dedent(stubs))
    (root / "ray_pkg.yaml").write_text(textwrap.dedent("""
        name: example_package
        description: a test package
        interface_file: my_pkg/stubs.py
        runtime_env:
            env_vars: {PKG_MODE: packaged}
    """))
    return str(root / "ray_pkg.yaml")


STUBS = """
    # only ray at top level: the driver need not have the package's dependencies
    import ray


    @ray.remote
    class MyActor:
        def __init__(self):
            from my_pkg import impl  # lazy: resolves in the package's working dir

            self.impl = impl

        def f(self):
            return self.impl.hello()


    @ray.remote
    def my_func():
        from my_pkg import impl

        return impl.hello()
"""


def test_load_package_runs_in_the_package_runtime_env(shutdown_only, tmp_path):
    cfg = _make_pkg(tmp_path, STUBS)
    ray.init(num_cpus=2)
    pkg = load_package(cfg)
    assert pkg._runtime_env["env_vars"] == {"PKG_MODE": "packaged"}
    assert pkg._runtime_env["working_dir"] == str(tmp_path)
    assert ray.get(pkg.my_func.remote()) == "hello from packaged"
    a = pkg.MyActor.remote()
    assert ray.get(a.f.remote()) == "hello from packaged"
    assert "example_package" in repr(pkg)


def test_load_package_rejects_bad_packages(tmp_path):
    bad = tmp_path / "bad"
    bad.mkdir()
    cfg = _make_pkg(bad, "import os\nimport ray\n")
    with pytest.raises(ValueError, match="only `ray`"):
        load_package(cfg)
    ok = tmp_path / "ok"
    ok.mkdir()
    cfg2 = _make_pkg(ok, "import os  # noqa\nimport ray\n")
    assert load_package(cfg2)._runtime_env["working_dir"] == str(ok)
    with pytest.raises(ValueError, match="does not exist"):
        load_package(str(tmp_path / "missing.yaml"))
    with pytest.raises(ValueError, match="network"):
        load_package("https://raw.githubusercontent.com/u/r/master/p/ray_pkg.yaml")
