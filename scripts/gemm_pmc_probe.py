"""o_proj weight-gradient product (dW[4096,4096] = gy^T x, T = 8192) three ways, for a PMC pass:
hand gfx950 GEMM on the natural operands, hipBLASLt on transposed copies, hipBLASLt natural."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402

T, N, K = 8192, 4096, 4096
gy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
gt, xt = ops.transpose(gy), ops.transpose(x)
for _ in range(int(os.environ.get("ITERS", 5))):
    ops.gemm(gy, x, a_kmajor=True, b_kmajor=True, out=dw)
    torch.mm(gt, xt.t(), out=dw)
    torch.mm(gy.t(), x, out=dw)
torch.cuda.synchronize()
print("ok")
