"""ResNet-50 image-classification training loop (BASELINE.json config "Ray Train TorchTrainer
ResNet-50 DDP bf16").

Reference workload: ``release/nightly_tests/dataset/multi_node_train_benchmark.py:262-370``
(torchvision resnet50, SGD lr 0.1 momentum 0.9, cross-entropy, 224x224, img/s). Here:
  * raw uint8 NHWC pixel batches (what an image datasource yields) are normalised on the GPU by
    the HIP ``image_normalize`` kernel straight into channels_last bf16 — inside the timed step;
  * NHWC activations end to end (MIOpen NHWC convolutions), bf16 autocast, fp32 parameters;
  * the framework's flat-buffer DDP (bucketed RCCL all-reduce overlapped with backward) and a
    flat SGD update (one pass over the whole model).
Synthetic images/labels of the configured shape (no dataset download is possible here).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist
import torch.nn.functional as F


def _dist_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def build_resnet_training(batch_size=256, image_size=224, num_classes=1000, lr=0.1, momentum=0.9,
                          bucket_cap_mb=64.0, device=None, seed=0, amp=True):
    from .. import ops
    from ..models.resnet import resnet50
    from ..parallel import DistributedDataParallel, FlatSGD

    device = device or torch.device("cuda", torch.cuda.current_device())
    rank, world = _dist_info()
    torch.manual_seed(seed)
    net = resnet50(num_classes=num_classes, device=device, channels_last=device.type == "cuda")
    ddp = DistributedDataParallel(net, bucket_cap_mb=bucket_cap_mb)
    opt = FlatSGD(ddp.flat, lr=lr, momentum=momentum)
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    use_amp = amp and device.type == "cuda"

    def batch():
        imgs = torch.randint(0, 256, (batch_size, image_size, image_size, 3), device=device, dtype=torch.uint8,
                             generator=g)
        labels = torch.randint(0, num_classes, (batch_size,), device=device, generator=g)
        return imgs, labels

    def step(imgs_u8, labels):
        x = ops.image_normalize(imgs_u8, dtype=torch.bfloat16 if use_amp else torch.float32,
                                channels_last=device.type == "cuda")
        with torch.autocast(device.type, dtype=torch.bfloat16, enabled=use_amp):
            logits = ddp(x)
        loss = F.cross_entropy(logits.float(), labels)
        loss.backward()
        ddp.finish_gradient_sync()
        opt.step(grad_scale=ddp.grad_scale)
        opt.zero_grad()
        return loss

    return net, ddp, opt, batch, step


def resnet_train_loop_per_worker(config: dict):
    """Train-loop entry point. Config keys: batch_size (per worker), image_size, steps, warmup,
    num_classes, device. Reports ``images_per_s`` for the whole job and ``ms_per_step``."""
    from . import report

    dev_kind = config.get("device", "cuda")
    device = None if dev_kind == "cuda" else torch.device(dev_kind)
    sync = torch.cuda.synchronize if dev_kind == "cuda" else (lambda: None)
    steps, warmup = int(config.get("steps", 20)), int(config.get("warmup", 5))
    bs = int(config.get("batch_size", 256))
    net, ddp, opt, batch, step = build_resnet_training(
        batch_size=bs, image_size=int(config.get("image_size", 224)), num_classes=int(config.get("num_classes", 1000)),
        lr=float(config.get("lr", 0.1)), device=device)
    rank, world = _dist_info()
    data = [batch() for _ in range(2)]
    loss = None
    for i in range(warmup):
        loss = step(*data[i % 2])
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(*data[i % 2])
    sync()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], device="cuda" if dev_kind == "cuda" else "cpu", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    metrics = {
        "loss": float(loss.item()) if loss is not None else float("nan"),
        "elapsed_s": el,
        "ms_per_step": 1000.0 * el / max(steps, 1),
        "images_per_s": steps * bs * world / el if el > 0 else 0.0,
        "world_size": world,
        "mem_gb": torch.cuda.max_memory_allocated() / 1e9 if dev_kind == "cuda" else 0.0,
    }
    report(metrics)
    return metrics
