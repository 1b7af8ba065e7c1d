"""o_proj forward product (y[8192,4096] = x[8192,4096] w[4096,4096]^T, both operands k-contiguous)
for PMC passes: hand GEMM variants ($VARIANTS, default 7,6) and hipBLASLt (torch.mm)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402

M, N, K = 8192, 4096, 4096
x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
lib = ops._lib.lib()
for _ in range(int(os.environ.get("ITERS", 5))):
    for v in [int(v) for v in os.environ.get("VARIANTS", "7,6").split(",")]:
        lib.rca_gemm_set_variant(v)
        ops.gemm(x, w, out=y)
    torch.mm(x, w.t(), out=y)
torch.cuda.synchronize()
print("ok")
