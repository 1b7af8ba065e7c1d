"""Diagnostic: is the grad-norm mismatch of test_ddp_norm_gpu nondeterminism or a stream race?"""
import sys
import torch
from ray_community_amd.models import build_llama
from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

toks = torch.randint(0, 1024, (2, 129), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
grads = []
for pre in (False, False, True, True):
    torch.manual_seed(0)
    net = build_llama("llama3-tiny", device="cuda")
    ddp = DistributedDataParallel(net, bucket_cap_mb=0.5, precompute_grad_norm=pre)
    opt = FlatAdamW(ddp.flat, lr=1e-3, max_grad_norm=0.05)
    opt.track_grad_norm = True
    loss = ddp(toks[:, :-1], toks[:, 1:])
    loss.backward()
    ddp.finish_gradient_sync()
    torch.cuda.synchronize()
    g = ddp.flat.grad.float().clone()
    pn = ddp.flat.precomputed_sumsq.item() ** 0.5 if ddp.flat.precomputed_sumsq is not None else None
    print("pre", pre, "loss", loss.item(), "true norm", g.norm().item(), "precomputed", pn, flush=True)
    grads.append(g)
    for bi, b in enumerate(ddp.flat.buckets):
        pass
for i in range(1, 4):
    d = (grads[i] - grads[0]).abs()
    print(i, "max diff vs run0", d.max().item(), "nnz diff", (d > 0).sum().item())
    if d.max() > 0:
        idx = (d > 0).nonzero()[:, 0]
        names = set()
        for n, p, off in ddp.flat.param_slices():
            lo, hi = off, off + p.numel()
            if ((idx >= lo) & (idx < hi)).any():
                names.add(n)
        print("   differing params:", sorted(names))
