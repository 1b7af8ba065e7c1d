"""Serve replica scheduler GPU locality on hardware (reference:
serve/_private/replica_scheduler/pow_2_scheduler.py prefers same-node replicas; on MI355X the
router also prefers a replica on the SAME GPU as a request's device tensor, which then crosses
no xGMI link)."""
import pytest
import torch

import ray_community_amd as ray
from ray_community_amd import serve
from ray_community_amd.serve.handle import _request_gpu, physical_gpu_ids

pytestmark = pytest.mark.gpu


@pytest.fixture
def serve_gpu():
    ray.init(num_cpus=8, include_dashboard=False, log_to_driver=False)
    yield
    serve.shutdown()
    ray.shutdown()


def _deploy(num_gpus):
    @serve.deployment(num_replicas=2, max_ongoing_requests=8, ray_actor_options={"num_cpus": 0, "num_gpus": num_gpus})
    class Where:
        def __call__(self, x):
            import os

            import torch as t

            assert x.is_cuda  # the device tensor arrived on this replica's GPU
            phys = physical_gpu_ids([x.device.index if x.device.index is not None else t.cuda.current_device()])
            return os.getpid(), phys[0], float(x.float().sum())

    return serve.run(Where.bind(), name="loc")


def test_device_tensor_requests_run_on_the_callers_gpu(serve_gpu):
    """One GPU: both replicas share GPU 0 (num_gpus 0.5), so both are in the same-GPU tier; every
    request carrying a CUDA tensor is recognised as a GPU-0 request and served on GPU 0."""
    h = _deploy(0.5)
    x = torch.arange(16, device="cuda", dtype=torch.float32)
    gpu = _request_gpu((x,), {})
    assert gpu == physical_gpu_ids([torch.cuda.current_device()])[0]
    outs = [h.remote(x + i).result(timeout_s=60) for i in range(8)]
    assert {o[1] for o in outs} == {gpu}
    assert [o[2] for o in outs] == [float((x + i).sum()) for i in range(8)]
    from ray_community_amd.serve.handle import _Router

    router = _Router._routers[("loc", "Where")]
    assert len(router.locations) == 2
    assert all(gpu in (loc.get("gpus") or ()) for loc in router.locations.values())


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs: one replica per GPU")
def test_device_tensor_goes_to_the_replica_on_its_gpu(serve_gpu):
    """Two replicas on two GPUs: a tensor on cuda:k is always served by the replica on physical
    GPU k (same-GPU tier), never copied over xGMI to the other replica."""
    h = _deploy(1)
    for dev in range(2):
        x = torch.ones(1024, device=f"cuda:{dev}")
        want = physical_gpu_ids([dev])[0]
        got = {h.remote(x).result(timeout_s=60)[1] for _ in range(16)}
        assert got == {want}, (dev, got)
