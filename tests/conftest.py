import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD MI355X GPU (HIP kernels, RCCL)")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def shutdown_only():
    yield None
    import ray_community_amd as ray

    ray.shutdown()


@pytest.fixture
def ray_start_regular(request):
    import ray_community_amd as ray

    params = getattr(request, "param", {}) or {}
    ctx = ray.init(num_cpus=params.get("num_cpus", 4), **{k: v for k, v in params.items() if k != "num_cpus"})
    yield ctx
    ray.shutdown()


@pytest.fixture
def ray_start_cluster():
    from ray_community_amd.cluster_utils import Cluster

    c = Cluster()
    yield c
    c.shutdown()
