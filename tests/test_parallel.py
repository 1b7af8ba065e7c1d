"""Multi-process (gloo, world_size 2) tests of the data-parallel building blocks: flat-buffer DDP
and ZeRO sharded data parallel must produce the same trajectory as single-process training on
the concatenated batch (reference behaviour: torch DDP / FSDP under ``prepare_model``)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed=0):
    from ray_community_amd.models import build_llama

    torch.manual_seed(seed)
    return build_llama("llama3-tiny", dtype=torch.float32, num_layers=2)


def _worker(rank, world, port, mode, steps, out_dir, bucket_mb):
    import torch.distributed as dist

    from ray_community_amd.parallel import (DistributedDataParallel, FlatAdamW, FullyShardedAdamW,
                                            FullyShardedDataParallel, ShardedAdamW, ShardedDataParallel)

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)  # world x default threads would oversubscribe the 8 CPUs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100)
    toks = torch.randint(0, 1024, (2 * world, 33))
    mine = toks[2 * rank: 2 * rank + 2]
    net = _model()
    if mode == "zero":
        wrap = ShardedDataParallel(net, bucket_cap_mb=bucket_mb)
        opt = ShardedAdamW(wrap, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    elif mode.startswith("fsdp"):
        wrap = FullyShardedDataParallel(net, reduce_dtype=torch.float32 if mode == "fsdp_f32" else None)
        opt = FullyShardedAdamW(wrap, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    else:
        wrap = DistributedDataParallel(net, bucket_cap_mb=bucket_mb)
        opt = FlatAdamW(wrap.flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for _ in range(steps):
        loss = wrap(mine[:, :-1], mine[:, 1:])
        loss.backward()
        wrap.finish_gradient_sync()
        opt.step(wrap.grad_scale)
        opt.zero_grad()
    if mode == "zero":
        wrap.wait_all_gathers()
    sd = wrap.state_dict() if mode.startswith("fsdp") else net.state_dict()  # fsdp: collective gather
    if rank == 0:
        torch.save({k: v.detach().clone() for k, v in sd.items()}, os.path.join(out_dir, f"{mode}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _single(steps, world):
    nt = torch.get_num_threads()
    torch.set_num_threads(1)  # the ranks' thread count: same CPU reduction orders
    try:
        return _single_run(steps, world)
    finally:
        torch.set_num_threads(nt)


def _single_run(steps, world):
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    torch.manual_seed(100)
    toks = torch.randint(0, 1024, (2 * world, 33))
    net = _model()
    wrap = DistributedDataParallel(net)
    opt = FlatAdamW(wrap.flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for _ in range(steps):
        # mean over ranks of per-rank mean losses == mean over the full batch (equal shard sizes)
        loss = sum(wrap(toks[2 * r: 2 * r + 2, :-1], toks[2 * r: 2 * r + 2, 1:]) for r in range(world)) / world
        loss.backward()
        opt.step()
        opt.zero_grad()
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


@pytest.mark.parametrize("mode,bucket_mb", [("ddp", 0.05), ("ddp", 256.0), ("zero", 0.05), ("zero", 256.0),
                                            ("fsdp", None), ("fsdp_f32", None)])
def test_data_parallel_matches_single_process(tmp_path, mode, bucket_mb):
    world, steps = 2, 3
    # tiny buckets -> many buckets, padding and out-of-order gathers are exercised; one big bucket
    # -> a bucket must wait for every gradient in it (fused-wgrad callback + AccumulateGrad hook
    # both report a weight: counted once)
    mp.spawn(_worker, args=(world, _port(), mode, steps, str(tmp_path), bucket_mb), nprocs=world, join=True)
    got = torch.load(os.path.join(tmp_path, f"{mode}.pt"), weights_only=True)
    ref = _single(steps, world)
    for k in ref:
        assert torch.allclose(got[k], ref[k], atol=2e-5, rtol=1e-4), (k, (got[k] - ref[k]).abs().max())


def test_flat_bucket_alignment():
    from ray_community_amd.parallel.flat import FlatParameters

    net = _model()
    fp = FlatParameters(net, bucket_cap_mb=0.05, bucket_align=64 * 3)
    assert len(fp.buckets) > 3
    for b in fp.buckets:
        assert b.start % 192 == 0 and b.end % 192 == 0 and b.end > b.start
    assert fp.buckets[-1].end == fp.numel
    for b0, b1 in zip(fp.buckets, fp.buckets[1:]):
        assert b0.end == b1.start
    # every parameter lies inside its bucket
    for p, off in zip(fp.params, fp.offsets):
        b = fp.buckets[fp.param_bucket[id(p)]]
        assert b.start <= off and off + p.numel() <= b.end
    # decay/no-decay split on a bucket boundary
    assert any(b.start == fp.decay_end for b in fp.buckets)


def test_adamw_transposed_segments_cover_flat_buffer():
    """The segment table of the W^T-refreshing AdamW update covers [0, numel) exactly once, in
    order, with matrix segments exactly on the 64-multiple fused weights, 1-D segments split at
    the weight-decay boundary, and consecutive first-block indices."""
    import torch

    from ray_community_amd.parallel import FlatAdamW
    from ray_community_amd.parallel.flat import FlatParameters
    from ray_community_amd.parallel.fused_linear import FusedWgradLinear

    m = torch.nn.ModuleList([torch.nn.Linear(64, 37), torch.nn.LayerNorm(37), FusedWgradLinear(37, 256),
                             FusedWgradLinear(256, 384), torch.nn.LayerNorm(384), FusedWgradLinear(384, 128),
                             FusedWgradLinear(128, 256), FusedWgradLinear(128, 64)]).to(torch.bfloat16)
    flat = FlatParameters(m)
    opt = FlatAdamW(flat, lr=1e-3)
    opt._setup_transposed()
    segs = opt._segs.tolist()
    cur, blk, mats = 0, 0, 0
    for off, n, b0, wt, R, C, decay, _ in segs:
        assert off == cur and b0 == blk and n > 0
        if wt:
            mats += 1
            assert R % 128 == 0 and C % 128 == 0 and R * C == n
            blk += (R // 128) * (C // 128)
        else:
            blk += (n + 4095) // 4096
            assert (off < flat.decay_end) == bool(decay) and (off + n <= flat.decay_end or off >= flat.decay_end)
        cur = off + n
    assert cur == flat.numel and blk == opt._seg_blocks and mats == 3
    for p in opt._wt_params:
        assert tuple(p._rca_wt.shape) == (p.shape[1], p.shape[0])


@pytest.mark.parametrize("mode", ["ddp", "zero", "fsdp"])
def test_world8_data_parallel_matches_single_process(tmp_path, mode):
    """The driver's N=8 launch shape, rehearsed on gloo: 8 ranks (2 sequences each) follow the
    single-process trajectory on the 16-sequence batch for DDP, ZeRO-1/2 and ZeRO-3."""
    world, steps = 8, 3
    mp.spawn(_worker, args=(world, _port(), mode, steps, str(tmp_path), 0.05 if mode != "fsdp" else None),
             nprocs=world, join=True)
    got = torch.load(os.path.join(tmp_path, f"{mode}.pt"), weights_only=True)
    ref = _single(steps, world)
    for k in ref:
        # 8-way sums in another order: AdamW (lr 1e-2) turns ~1e-7 gradient noise into <= 1e-4 steps
        assert torch.allclose(got[k], ref[k], atol=1e-4, rtol=2e-4), (k, (got[k] - ref[k]).abs().max())


def _bf16_worker(rank, world, port, steps, out_dir):
    import torch.distributed as dist

    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)  # world x default threads would oversubscribe the 8 CPUs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(7)
    toks = torch.randint(0, 1024, (2 * world, 65))
    mine = toks[2 * rank: 2 * rank + 2]
    for reduce in ("bf16", "fp32"):  # same init, same data: only the collective's dtype differs
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", dtype=torch.bfloat16, num_layers=2)  # bf16 weights + grads
        wrap = DistributedDataParallel(net, bucket_cap_mb=0.05,
                                       reduce_dtype=torch.float32 if reduce == "fp32" else None)
        opt = FlatAdamW(wrap.flat, lr=3e-3, weight_decay=0.1, max_grad_norm=1.0)
        losses = []
        for _ in range(steps):
            loss = wrap(mine[:, :-1], mine[:, 1:])
            loss.backward()
            wrap.finish_gradient_sync()
            opt.step(wrap.grad_scale)
            opt.zero_grad()
            lt = loss.detach().float().reshape(1)
            dist.all_reduce(lt)
            losses.append(float(lt) / world)
        if rank == 0:
            torch.save(torch.tensor(losses), os.path.join(out_dir, f"bf16_{reduce}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_bf16_gradient_reduction_tracks_fp32_at_world8(tmp_path):
    """The bench's N>1 default reduces bf16 gradients in bf16 (half the xGMI bytes of torch DDP's
    fp32 reduction under AMP). At world 8 the global-batch loss curve over 12 AdamW steps tracks the
    fp32-reduced run: every step's loss within 0.5 % of the initial loss (measured: 0.23 %, the
    gap growing only as the tiny model memorises its batch), the total loss drop within 1 %."""
    world, steps = 8, 12
    mp.spawn(_bf16_worker, args=(world, _port(), steps, str(tmp_path)), nprocs=world, join=True)
    a = torch.load(os.path.join(tmp_path, "bf16_bf16.pt"), weights_only=True)
    b = torch.load(os.path.join(tmp_path, "bf16_fp32.pt"), weights_only=True)
    gap = ((a - b).abs().max() / b[0]).item()
    assert gap < 5e-3, (gap, a.tolist(), b.tolist())
    drop_a, drop_b = (a[0] - a[-1]).item(), (b[0] - b[-1]).item()
    assert drop_b > 3.0 and abs(drop_a - drop_b) / drop_b < 1e-2, (drop_a, drop_b)
