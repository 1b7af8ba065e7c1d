"""runtime_env (reference tests: python/ray/tests/test_runtime_env*.py)."""
import os
import zipfile

import pytest

import ray_community_amd as ray
from ray_community_amd.runtime_env import RuntimeEnv


def test_runtime_env_validation():
    env = RuntimeEnv(env_vars={"A": "1"}, py_modules=["/tmp"])
    assert env.env_vars() == {"A": "1"} and env.py_modules() == ["/tmp"]
    with pytest.raises(TypeError):
        RuntimeEnv(env_vars={"A": 1})
    with pytest.raises(ValueError):
        RuntimeEnv(pip=["x"], conda="y")
    with pytest.raises(ValueError):
        RuntimeEnv(bogus=1)
    assert RuntimeEnv.deserialize(env.serialize()) == env


def test_working_dir_zip_py_modules_and_hook(shutdown_only, tmp_path):
    pkg = tmp_path / "src"
    pkg.mkdir()
    (pkg / "mymod_rca.py").write_text("VALUE = 41\n")
    (pkg / "data.txt").write_text("hello")
    zpath = tmp_path / "wd.zip"
    with zipfile.ZipFile(zpath, "w") as z:
        z.write(pkg / "mymod_rca.py", "mymod_rca.py")
        z.write(pkg / "data.txt", "data.txt")
    ray.init(num_cpus=2, runtime_env={"env_vars": {"JOB_LEVEL": "yes"}})

    @ray.remote(runtime_env={"working_dir": str(zpath)})
    def read():
        import mymod_rca

        with open("data.txt") as f:
            return mymod_rca.VALUE + 1, f.read(), os.environ.get("JOB_LEVEL")

    assert ray.get(read.remote()) == (42, "hello", "yes")

    def hook():
        os.environ["HOOKED"] = "1"

    @ray.remote(runtime_env={"worker_process_setup_hook": hook, "env_vars": {"B": "2"}})
    def hooked():
        return os.environ.get("HOOKED"), os.environ.get("B")

    assert ray.get(hooked.remote()) == ("1", "2")


def test_missing_pip_requirement_fails_task(shutdown_only):
    ray.init(num_cpus=1)

    @ray.remote(runtime_env={"pip": ["definitely-not-installed-pkg-xyz==1.0"]})
    def f():
        return 1

    with pytest.raises(Exception, match="not available"):
        ray.get(f.remote(), timeout=60)

    @ray.remote(runtime_env={"pip": ["numpy"]})
    def g():
        return 2

    assert ray.get(g.remote()) == 2
