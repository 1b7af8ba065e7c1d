"""Compiled-DAG tensor edges with TorchTensorType (reference: python/ray/dag/tests/experimental/
test_torch_tensor_dag.py). CPU: the hint is accepted and CPU tensors pass through; GPU: CUDA
tensors travel through HIP-IPC device slots (descriptor in the channel, one D2D copy per read)."""
import pytest
import torch

import ray_community_amd as ray
from ray_community_amd.dag import InputNode, TorchTensorType


@ray.remote
class _Stage:
    def __init__(self, scale, device):
        self.scale = scale
        self.device = device

    def make(self, n):
        return {"x": torch.arange(n, dtype=torch.float32, device=self.device) * self.scale, "n": n}

    def combine(self, d):
        assert d["x"].device.type == self.device
        return d["x"] * self.scale + d["n"]


def _pipeline(dev, gpus):
    a = _Stage.options(num_gpus=gpus).remote(2.0, dev)
    b = _Stage.options(num_gpus=gpus).remote(3.0, dev)
    with InputNode() as inp:
        mid = a.make.bind(inp).with_type_hint(TorchTensorType())
        out = b.combine.bind(mid).with_type_hint(TorchTensorType(transport="nccl"))
    return out.experimental_compile()


def test_type_hint_cpu_tensors(shutdown_only):
    ray.init(num_cpus=4, include_dashboard=False, log_to_driver=False)
    dag = _pipeline("cpu", 0)
    try:
        for n in (4, 7, 4):
            got = dag.execute(n).get(timeout=30)
            assert torch.equal(got, torch.arange(n, dtype=torch.float32) * 6 + n)
    finally:
        dag.teardown()


@pytest.mark.gpu
def test_type_hint_gpu_tensors_over_device_slots(shutdown_only):
    ray.init(num_cpus=4, num_gpus=1, include_dashboard=False, log_to_driver=False)
    dag = _pipeline("cuda", 0.5)
    try:
        for n in (1024, 4096, 1024, 1 << 20):
            got = dag.execute(n).get(timeout=60)
            assert got.is_cuda
            ref = torch.arange(n, dtype=torch.float32) * 6 + n
            assert torch.equal(got.cpu(), ref)
    finally:
        dag.teardown()
