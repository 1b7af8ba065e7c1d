"""The framework's own data-parallel path over RCCL: TorchTrainer(num_workers=2, use_gpu=True) runs
the Llama train step with DistributedDataParallel (bucketed all-reduce) and ShardedDataParallel
(in-place, aliased reduce-scatter / all-gather of the flat buffers, parallel/fsdp.py) and follows
the world-1 trajectory of the same global batch (reference: python/ray/train/torch/config.py
_setup_torch_process_group + the DDP path of train_loop_utils.prepare_model). Needs two GPUs: the
driver's 1-GPU box skips it; the gloo world-2 / world-8 rehearsals of the same code are
tests/test_parallel.py."""
import pytest
import torch

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (RCCL over xGMI)")]

STEPS = 3


def _data(world):
    g = torch.Generator().manual_seed(11)
    return torch.randint(0, 1024, (2 * world, 129), generator=g)


def _build(mode, device):
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW, ShardedAdamW, ShardedDataParallel

    torch.manual_seed(0)
    net = build_llama("llama3-tiny", device=device, num_layers=2)
    if mode == "zero":
        wrap = ShardedDataParallel(net, bucket_cap_mb=0.05, reduce_dtype=torch.float32)
        opt = ShardedAdamW(wrap, lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
    else:
        wrap = DistributedDataParallel(net, bucket_cap_mb=0.05, reduce_dtype=torch.float32)
        opt = FlatAdamW(wrap.flat, lr=1e-2, weight_decay=0.1, max_grad_norm=1.0)
    return net, wrap, opt


def _loop(config):
    import torch.distributed as dist

    from ray_community_amd import train

    mode = config["mode"]
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device())
    net, wrap, opt = _build(mode, dev)
    toks = _data(world)[2 * rank: 2 * rank + 2].to(dev)
    losses = []
    for _ in range(STEPS):
        loss = wrap(toks[:, :-1], toks[:, 1:])
        loss.backward()
        wrap.finish_gradient_sync()
        opt.step(wrap.grad_scale)
        opt.zero_grad()
        lt = loss.detach().float().reshape(1)
        dist.all_reduce(lt)
        losses.append(float(lt) / world)
    if mode == "zero":
        wrap.wait_all_gathers()
    params = torch.cat([p.detach().float().reshape(-1) for p in net.parameters()]).cpu()
    train.report({"losses": losses, "params": params.tolist(), "backend": dist.get_backend()})


def _world1(world):
    dev = torch.device("cuda", 0)
    net, wrap, opt = _build("ddp", dev)
    init = torch.cat([p.detach().float().reshape(-1) for p in net.parameters()]).cpu()
    toks = _data(world).to(dev)
    losses = []
    for _ in range(STEPS):
        loss = sum(wrap(toks[2 * r: 2 * r + 2, :-1], toks[2 * r: 2 * r + 2, 1:]) for r in range(world)) / world
        loss.backward()
        wrap.finish_gradient_sync()
        opt.step(wrap.grad_scale)
        opt.zero_grad()
        losses.append(float(loss))
    params = torch.cat([p.detach().float().reshape(-1) for p in net.parameters()]).cpu()
    return losses, init, params


@pytest.mark.parametrize("mode", ["ddp", "zero"])
def test_torchtrainer_two_gpus_rccl_follows_world1(mode):
    import ray_community_amd as ray
    from ray_community_amd.train import ScalingConfig
    from ray_community_amd.train.torch import TorchTrainer

    ref_losses, init, ref_params = _world1(2)
    ray.init(num_gpus=2, include_dashboard=False, log_to_driver=False)
    try:
        res = TorchTrainer(_loop, train_loop_config={"mode": mode},
                           scaling_config=ScalingConfig(num_workers=2, use_gpu=True)).fit()
    finally:
        ray.shutdown()
    assert res.error is None, res.error
    m = res.metrics
    assert m["backend"] == "nccl"  # RCCL
    for a, b in zip(m["losses"], ref_losses):
        assert abs(a - b) < 2e-2 * abs(ref_losses[0]), (m["losses"], ref_losses)
    got = torch.tensor(m["params"])
    moved = (ref_params - init).norm()
    assert moved > 0 and (got - ref_params).norm() / moved < 0.1, ((got - ref_params).norm() / moved).item()
