"""ZeRO-3 (``parallel/fully_sharded.py``): unsharded equivalence at world 1, gradient
accumulation and state-dict round trips at world 2 (gloo), the self-launched bench in fsdp mode,
and the HBM model that puts Llama-3-70B on 8 x 288 GB (reference: torch FSDP behind
``prepare_model(parallel_strategy="fsdp")``, ``python/ray/train/torch/train_loop_utils.py:175``)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(seed=0, layers=3):
    from ray_community_amd.models import build_llama

    torch.manual_seed(seed)
    return build_llama("llama3-tiny", dtype=torch.float32, num_layers=layers)


def _ref_train(toks_list, steps):
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    net = _model()
    wrap = DistributedDataParallel(net)
    opt = FlatAdamW(wrap.flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for _ in range(steps):
        loss = sum(wrap(t[:, :-1], t[:, 1:]) for t in toks_list) / len(toks_list)
        loss.backward()
        opt.step()
        opt.zero_grad()
    return {k: v.detach().clone() for k, v in net.state_dict().items()}


def test_world1_matches_flat_adamw():
    from ray_community_amd.parallel import FullyShardedAdamW, FullyShardedDataParallel

    torch.manual_seed(5)
    toks = torch.randint(0, 1024, (2, 33))
    ref = _ref_train([toks], 3)
    net = _model()
    f = FullyShardedDataParallel(net)
    assert [u.name for u in f.units] == ["root", "unit0", "unit1", "unit2"]
    opt = FullyShardedAdamW(f, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for _ in range(3):
        loss = f(toks[:, :-1], toks[:, 1:])
        loss.backward()
        f.finish_gradient_sync()
        opt.step()
        opt.zero_grad()
    got = f.state_dict()
    for k in ref:
        assert torch.allclose(got[k], ref[k], atol=2e-5, rtol=1e-4), (k, (got[k] - ref[k]).abs().max())
    # world 1 is zero-copy: parameters are views of the local shard buffer
    p = next(net.parameters())
    assert p.untyped_storage().data_ptr() == f.local_data.untyped_storage().data_ptr()


def _accum_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from ray_community_amd.parallel import FullyShardedAdamW, FullyShardedDataParallel

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(7)
    toks = torch.randint(0, 1024, (4 * world, 33))
    net = _model()
    f = FullyShardedDataParallel(net)
    opt = FullyShardedAdamW(f, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    for _ in range(2):
        # two micro-batches per step: each reduce-scatters and accumulates into the local shard
        for mbi in range(2):
            t = toks[4 * rank + 2 * mbi: 4 * rank + 2 * mbi + 2]
            loss = f(t[:, :-1], t[:, 1:]) / 2
            loss.backward()
            f.finish_gradient_sync()
        opt.step()
        opt.zero_grad()
    sd = f.state_dict()
    # every unit is freed again between steps (only the root stays gathered)
    assert all(u.full.untyped_storage().nbytes() == 0 for u in f.units[1:])
    # state-dict round trip into a fresh wrapper (different init) reproduces the weights
    net2 = _model(seed=99)
    f2 = FullyShardedDataParallel(net2)
    f2.load_state_dict(sd)
    sd2 = f2.state_dict()
    for k in sd:
        assert torch.equal(sd[k], sd2[k]), k
    # optimizer shard round trip
    osd = opt.state_dict()
    opt2 = FullyShardedAdamW(f2, lr=1e-2)
    opt2.load_state_dict(osd)
    assert torch.equal(opt2.m, opt.m) and torch.equal(opt2.master, opt.master)
    if rank == 0:
        torch.save(sd, os.path.join(out_dir, "accum.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_world2_gradient_accumulation_and_state_dict(tmp_path):
    world = 2
    mp.spawn(_accum_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    got = torch.load(os.path.join(tmp_path, "accum.pt"), weights_only=True)
    torch.manual_seed(7)
    toks = torch.randint(0, 1024, (4 * world, 33))
    ref = _ref_train([toks[2 * i: 2 * i + 2] for i in range(2 * world)], 2)
    # accumulating two reduced micro-batch gradients differs from one backward over the union only
    # by fp32 summation order, which AdamW's normalisation amplifies on near-zero gradients
    for k in ref:
        d = (got[k] - ref[k]).abs()
        assert d.max() < 1e-3 and d.mean() < 2e-6, (k, d.max(), d.mean())


def test_memory_model_70b_fits_8_gpus():
    from ray_community_amd.models.llama import PRESETS
    from ray_community_amd.parallel import estimate_memory_gb

    cfg = PRESETS["llama3-70b"]
    m8 = estimate_memory_gb(cfg, world=8, micro_batch=1, seq_len=4096)
    assert m8["total"] < 288 * 0.95, m8
    m1 = estimate_memory_gb(cfg, world=1, micro_batch=1, seq_len=4096)
    assert m1["total"] > 288, m1  # does not fit unsharded
    # the 8B model's replicated-DDP footprint is what bench measures (~170 GB peak)
    m = estimate_memory_gb(PRESETS["llama3-8b"], world=1, micro_batch=2, seq_len=4096)
    assert 150 < m["total"] < 190, m


def test_bench_fsdp_two_workers_cpu(tmp_path):
    env = dict(os.environ)
    env.pop("RCA_ADDRESS", None)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--model", "llama3-tiny", "--seq-len", "128", "--device", "cpu", "--parallel", "fsdp"]
    out = subprocess.run(cmd, cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallel_mode"] == "fsdp" and rec["value"] > 0
    assert "ZeRO-3" in rec["config"]["data_parallel"]


@pytest.mark.gpu
def test_fsdp_world1_gpu_matches_ddp():
    """bf16 on the GPU through the fused HIP AdamW: ZeRO-3 at world 1 ~= DDP + FlatAdamW."""
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import (DistributedDataParallel, FlatAdamW, FullyShardedAdamW,
                                            FullyShardedDataParallel)

    torch.manual_seed(3)
    toks = torch.randint(0, 1024, (2, 129), device="cuda")
    out = []
    for mode in ("ddp", "fsdp"):
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", device="cuda")
        if mode == "ddp":
            w = DistributedDataParallel(net)
            opt = FlatAdamW(w.flat, lr=1e-3)
        else:
            w = FullyShardedDataParallel(net)
            opt = FullyShardedAdamW(w, lr=1e-3)
        for _ in range(3):
            loss = w(toks[:, :-1], toks[:, 1:])
            loss.backward()
            w.finish_gradient_sync()
            opt.step(w.grad_scale)
            opt.zero_grad()
        torch.cuda.synchronize()
        sd = w.state_dict() if mode == "fsdp" else {k: v.detach().cpu() for k, v in net.state_dict().items()}
        out.append(sd)
    # not bitwise: the embedding backward accumulates with atomics and the grad-norm sum runs over
    # a different buffer layout -> last-bit gradient differences, which AdamW can turn into at most
    # ~2 * lr per step on near-zero-gradient elements, plus one bf16 ulp of the rounded weight
    for k in out[0]:
        a, b = out[0][k].float().cpu(), out[1][k].float().cpu()
        d = (a - b).abs()
        assert (d <= 3 * 2 * 1e-3 + a.abs() * 2 ** -7).all() and d.mean() < 1e-4, (k, d.max(), d.mean())
