"""Diagnose overlapped-AdamW mismatches: serial vs serial, overlap+sync, overlap."""
import torch

from ray_community_amd.models import build_llama
from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

DEV = "cuda"


def run(overlap, sync_after_step, iters=3):
    torch.manual_seed(0)
    net = build_llama("llama3-tiny", device=DEV)
    ddp = DistributedDataParallel(net, bucket_cap_mb=0.2)
    opt = FlatAdamW(ddp.flat, lr=1e-3, max_grad_norm=0.5)
    if overlap:
        opt.overlap_with_forward(net)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    toks = torch.randint(0, 1024, (2, 128), device=DEV, generator=torch.Generator(device=DEV).manual_seed(5))
    outs = []
    for _ in range(iters):
        grad = torch.randn(ddp.flat.numel, device=DEV, generator=g).to(torch.bfloat16) * 0.01
        ddp.flat.grad.copy_(grad)
        opt.step(1.0)
        opt.zero_grad()
        if sync_after_step:
            torch.cuda.synchronize()
        with torch.no_grad():
            outs.append(net(toks).clone())
    torch.cuda.synchronize()
    return outs, ddp.flat.data.clone()


base, d0 = run(False, False)
for name, ov, sy in [("serial2", False, False), ("overlap+sync", True, True), ("overlap", True, False)]:
    o, d = run(ov, sy)
    print(name, [torch.equal(a, b) for a, b in zip(base, o)], "data equal", torch.equal(d0, d),
          "maxdiff", [float((a.float() - b.float()).abs().max()) for a, b in zip(base, o)])
