"""o_proj forward product (y[8192,4096] = x[8192,4096] w[4096,4096]^T, both operands k-contiguous)
three ways, for PMC passes: hand GEMM variants 6 and 3, and hipBLASLt (torch.mm)."""
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
    lib.rca_gemm_set_variant(6)
    ops.gemm(x, w, out=y)
    lib.rca_gemm_set_variant(3)
    ops.gemm(x, w, out=y)
    torch.mm(x, w.t(), out=y)
torch.cuda.synchronize()
print("ok")
