"""Microbenchmark + fp32 check of the grad sum-of-squares kernel (one 256 MB bf16 DDP bucket)."""
import time

import torch

from ray_community_amd import ops

x = torch.randn(128 << 20, device="cuda", dtype=torch.bfloat16)
ref = x.float().pow(2).sum().item()
out = ops.grad_sumsq([x])
torch.cuda.synchronize()
assert abs(out.item() - ref) / ref < 1e-4, (out.item(), ref)
for _ in range(3):
    ops.grad_sumsq([x], out=out)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    ops.grad_sumsq([x], out=out)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print(f"sumsq 256 MB bf16: {dt * 1e6:.1f} us, {x.numel() * 2 / dt / 1e12:.2f} TB/s, rel err {abs(out.item() - ref) / ref:.2e}")
