"""Llama pre-training loop (the Ray Train Llama-3-8B DDP headline workload).

``llama_train_loop_per_worker(config)`` is a regular Train worker function: it runs under
``TorchTrainer`` (one actor per GPU, process group over RCCL) and equally under an external
``torchrun`` launch (one process per GPU). It builds the model directly on the GPU, wraps it
in the framework's bucketed RCCL DDP, steps the fused flat AdamW, and reports timing.
Synthetic token data of the configured shape (no dataset download is possible here).
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist


def _dist_info():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def build_llama_training(model="llama3-8b", seq_len=4096, micro_batch=2, lr=3e-4, bucket_cap_mb=256.0,
                         device=None, seed=1234, max_grad_norm=1.0, parallel="ddp", grad_reduce_dtype="bf16",
                         overlap_optimizer=False, grad_norm_side_stream=False, **model_overrides):
    """``parallel``: "ddp" (replicated AdamW after a bucketed all-reduce; the default, as the
    headline metric is DDP), "zero" (reduce-scatter, sharded AdamW, all-gather overlapped with the
    next forward — parallel/fsdp.py), "fsdp" (ZeRO-3: parameters sharded too, each block's weights
    all-gathered just in time and freed after use -- parallel/fully_sharded.py; what lets
    ``llama3-70b`` train on 8 GPUs) or "auto" (zero when world > 1: the AdamW pass, ~9 % of a
    1-GPU step, shrinks by 1/world). ``grad_reduce_dtype``: "bf16" (gradients reduced in the
    compute dtype) or "fp32" (widened to fp32 before the collective, torch-DDP-under-AMP parity).
    ``overlap_optimizer`` (DDP): the HBM-bound AdamW update runs bucket by bucket on a side stream
    overlapped with the next forward (``FlatAdamW.overlap_with_forward``). Off by default: on the
    8B step it measured 368 vs 366 ms serial -- the forward's 256-VGPR GEMM workgroups fill every
    SIMD, so AdamW waves cannot be co-resident and only time-slice with them.
    ``grad_norm_side_stream`` (DDP): take the clip norm's sum of squares per finished bucket on a
    side stream during backward instead of one pass before AdamW. Off by default: on the 8B step
    the side-stream kernels (68 per step) compete with the memory-bound backward kernels for HBM
    and the main stream lost more than the 16 GB pass costs (342.3 vs 344.0 ms median,
    scripts/step_ab.py --arms norm_side,norm_main, profiles/llama8b_r6_cpath_baseline.md)."""
    from ..models import build_llama
    from ..parallel import (DistributedDataParallel, FlatAdamW, FullyShardedAdamW, FullyShardedDataParallel,
                            ShardedAdamW, ShardedDataParallel)

    device = device or torch.device("cuda", torch.cuda.current_device())
    rank, world = _dist_info()
    if parallel == "auto":
        parallel = "zero" if world > 1 else "ddp"
    rdt = {"bf16": None, "fp32": torch.float32}[grad_reduce_dtype]
    torch.manual_seed(seed)
    net = build_llama(model, device=device, max_seq_len=max(seq_len, 256), **model_overrides)
    if parallel == "zero":
        ddp = ShardedDataParallel(net, bucket_cap_mb=bucket_cap_mb, reduce_dtype=rdt)
        opt = ShardedAdamW(ddp, lr=lr, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=max_grad_norm)
    elif parallel == "fsdp":
        ddp = FullyShardedDataParallel(net, reduce_dtype=rdt)
        opt = FullyShardedAdamW(ddp, lr=lr, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=max_grad_norm)
    elif parallel == "ddp":
        ddp = DistributedDataParallel(net, bucket_cap_mb=bucket_cap_mb, reduce_dtype=rdt,
                                      precompute_grad_norm=bool(grad_norm_side_stream) and max_grad_norm is not None
                                      and max_grad_norm > 0)
        opt = FlatAdamW(ddp.flat, lr=lr, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=max_grad_norm)
        if overlap_optimizer:
            opt.overlap_with_forward(net)
    else:
        raise ValueError(f"unknown parallel mode {parallel!r}")
    net.parallel_mode = parallel
    g = torch.Generator(device=device)
    g.manual_seed(seed + rank)
    V = net.cfg.vocab_size

    def batch():
        t = torch.randint(0, V, (micro_batch, seq_len + 1), device=device, generator=g)
        return t[:, :-1].contiguous(), t[:, 1:].contiguous()

    def step(tokens, labels):
        loss = ddp(tokens, labels)
        loss.backward()
        ddp.finish_gradient_sync()
        opt.step(grad_scale=ddp.grad_scale)
        opt.zero_grad()
        return loss

    return net, ddp, opt, batch, step


def llama_train_loop_per_worker(config: dict):
    """Train-loop entry point. Config keys: model, seq_len, micro_batch, steps, warmup, lr,
    bucket_cap_mb. Reports ``tokens_per_s`` (this worker) and ``ms_per_step``."""
    from . import report

    dev_kind = config.get("device", "cuda")
    device = None if dev_kind == "cuda" else torch.device(dev_kind)
    sync = torch.cuda.synchronize if dev_kind == "cuda" else (lambda: None)
    steps = int(config.get("steps", 10))
    warmup = int(config.get("warmup", 3))
    seq_len = int(config.get("seq_len", 4096))
    mb = int(config.get("micro_batch", 2))
    net, ddp, opt, batch, step = build_llama_training(
        model=config.get("model", "llama3-8b"), seq_len=seq_len, micro_batch=mb, lr=config.get("lr", 3e-4),
        bucket_cap_mb=config.get("bucket_cap_mb", 256.0), device=device, parallel=config.get("parallel", "ddp"),
        grad_reduce_dtype=config.get("grad_reduce_dtype", "bf16"),
        overlap_optimizer=bool(config.get("overlap_optimizer", False)),
        **config.get("model_overrides", {}))
    rank, world = _dist_info()
    data = [batch() for _ in range(2)]
    loss = None
    for i in range(warmup):
        loss = step(*data[i % 2])
    sync()
    if world > 1:
        dist.barrier()
    sync()
    timer = getattr(ddp, "comm_timer", None)
    if timer is not None:
        timer.take_ms()
        timer.enabled = dev_kind == "cuda" and world > 1
    t0 = time.perf_counter()
    for i in range(steps):
        loss = step(*data[i % 2])
    sync()
    if world > 1:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    # compute-stream stall on collectives (events around every wait: what overlap did not hide)
    exposed = timer.take_ms() / max(steps, 1) if timer is not None and timer.enabled else 0.0
    if timer is not None:
        timer.enabled = False
    ex_t = torch.tensor([exposed], dtype=torch.float64, device="cuda" if dev_kind == "cuda" else "cpu")
    if world > 1:
        dist.all_reduce(ex_t, op=dist.ReduceOp.MAX)
    exposed = float(ex_t.item())
    # every rank's own timed-loop wall time (stragglers show up as a max/min spread); the job's
    # elapsed time is the slowest rank's
    dev = "cuda" if dev_kind == "cuda" else "cpu"
    if world > 1:
        all_el = [torch.zeros(1, device=dev, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(all_el, torch.tensor([el], device=dev, dtype=torch.float64))
        rank_el = [float(t.item()) for t in all_el]
    else:
        rank_el = [el]
    el = max(rank_el)
    tokens = steps * mb * seq_len * world
    metrics = {
        "loss": float(loss.item()) if loss is not None else float("nan"),
        "elapsed_s": el,
        "ms_per_step": 1000.0 * el / max(steps, 1),
        "tokens_per_s": tokens / el if el > 0 else 0.0,
        "world_size": world,
        "mem_gb": torch.cuda.max_memory_allocated() / 1e9 if dev_kind == "cuda" else 0.0,
        "flops_per_token": net.cfg.flops_per_token(seq_len),
        "parallel": net.parallel_mode,
        "grad_reduce_dtype": config.get("grad_reduce_dtype", "bf16"),
        "exposed_comm_ms": exposed,
        "rank_ms_per_step": [round(1000.0 * e / max(steps, 1), 3) for e in rank_el],
    }
    if dev_kind == "cuda":
        from .torch.config import group_info

        metrics["process_group"] = group_info(torch.cuda.current_device())
    report(metrics)
    return metrics
