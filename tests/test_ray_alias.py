"""``import ray`` alias: reference-style user code runs on ray_community_amd unchanged."""
import importlib


def test_alias_is_same_module_objects():
    import ray
    import ray_community_amd

    assert ray is ray_community_amd
    for sub in ("train", "train.torch", "tune", "data", "serve", "util.collective", "util.queue", "dag",
                "rllib.algorithms.ppo", "util.placement_group", "workflow", "job_submission"):
        a = importlib.import_module("ray." + sub)
        b = importlib.import_module("ray_community_amd." + sub)
        assert a is b, sub
    from ray.train import ScalingConfig
    from ray_community_amd.train import ScalingConfig as S2

    assert ScalingConfig is S2


def test_alias_unknown_submodule_raises():
    import pytest

    with pytest.raises(ModuleNotFoundError):
        importlib.import_module("ray.no_such_module_xyz")


def test_reference_style_program(shutdown_only):
    import ray

    ray.init(num_cpus=2)

    @ray.remote
    def square(x):
        return x * x

    @ray.remote
    class Counter:
        def __init__(self):
            self.n = 0

        def incr(self, k):
            self.n += k
            return self.n

    assert ray.get([square.remote(i) for i in range(4)]) == [0, 1, 4, 9]
    c = Counter.remote()
    ray.get([c.incr.remote(1) for _ in range(3)])
    assert ray.get(c.incr.remote(0)) == 3
    ref = ray.put({"a": 1})
    ready, _ = ray.wait([ref], timeout=5)
    assert ray.get(ready[0]) == {"a": 1}
