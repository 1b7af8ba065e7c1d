"""Diagnostic: DDP precompute_grad_norm (side-stream per-bucket sums of squares during backward)
vs the post-backward norm, on the 8B-shaped model (optionally fewer layers), 256 MB buckets.
Prints per-step grad norms and losses for both paths."""
import argparse
import json

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(pre, layers, steps, seq, mb):
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    torch.manual_seed(1234)
    net = build_llama("llama3-8b", device="cuda", max_seq_len=seq, num_layers=layers)
    ddp = DistributedDataParallel(net, bucket_cap_mb=256.0, precompute_grad_norm=pre)
    opt = FlatAdamW(ddp.flat, lr=3e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0)
    opt.track_grad_norm = True
    g = torch.Generator(device="cuda")
    g.manual_seed(1234)
    V = net.cfg.vocab_size
    data = []
    for _ in range(2):
        t = torch.randint(0, V, (mb, seq + 1), device="cuda", generator=g)
        data.append((t[:, :-1].contiguous(), t[:, 1:].contiguous()))
    out = []
    for i in range(steps):
        loss = ddp(*data[i % 2])
        loss.backward()
        ddp.finish_gradient_sync()
        pre_s = float(ddp.flat.precomputed_sumsq.item()) if ddp.flat.precomputed_sumsq is not None else None
        post = float(torch.sum(ddp.flat.grad.float() ** 2).item())
        opt.step(ddp.grad_scale)
        out.append({"loss": float(loss.item()), "norm": opt.grad_norm(), "pre_sumsq": pre_s, "post_sumsq": post})
        opt.zero_grad()
    del ddp, opt, net
    torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--mb", type=int, default=2)
    a = ap.parse_args()
    for pre in (False, True):
        print(json.dumps({"precompute": pre, "steps": run(pre, a.layers, a.steps, a.seq, a.mb)}), flush=True)
