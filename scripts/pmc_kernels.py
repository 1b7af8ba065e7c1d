"""Kernel set for rocprofv3 PMC passes (scripts/gpu_pmc.sh): the hot kernels of the Llama-3-8B
step at their bench shapes, a few dispatches each -- gfx950 flash attention fwd + bwd
(B=2, S=4096, Hq=32, Hkv=8, D=128, causal), the hand MFMA GEMM and hipBLASLt on the gate|up
forward shape (8192 x 28672 x 4096), fused-residual RMSNorm fwd + bwd (8192 x 4096), SwiGLU fwd
+ bwd and the fused AdamW over 256 M parameters."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402


def main():
    dev = "cuda"
    it = int(os.environ.get("PMC_ITERS", 2))
    B, S, Hq, Hk, D = 2, 4096, 32, 8, 128
    qkv = torch.randn(B * S, (Hq + 2 * Hk) * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B * S, Hq * D, device=dev, dtype=torch.bfloat16)
    for _ in range(it):
        ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True).backward(do)
    del qkv, do
    M, N, K = 8192, 28672, 4096
    a = torch.rand(M, K, device=dev, dtype=torch.bfloat16) - 0.5
    w = torch.rand(N, K, device=dev, dtype=torch.bfloat16) - 0.5
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    for _ in range(it):
        ops.gemm(a, w, out=c)
        torch.matmul(a, w.t(), out=c)
    del a, w, c
    x = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(8192, 4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.ones(4096, device=dev, dtype=torch.bfloat16, requires_grad=True)
    for _ in range(it):
        h, res = ops.rms_norm(x, g, 1e-5, r)
        (h.float().sum() + res.float().sum()).backward()
    gu = torch.randn(8192, 2 * 14336, device=dev, dtype=torch.bfloat16, requires_grad=True)
    for _ in range(it):
        ops.swiglu(gu).backward(torch.ones(8192, 14336, device=dev, dtype=torch.bfloat16))
    from ray_community_amd.parallel import FlatAdamW
    from ray_community_amd.parallel.flat import FlatParameters

    net = torch.nn.Linear(16384, 16384, bias=False, device=dev, dtype=torch.bfloat16)
    flat = FlatParameters(net)
    flat.grad.normal_()
    opt = FlatAdamW(flat, lr=1e-4, max_grad_norm=0.0)
    for _ in range(it):
        opt.step()
    torch.cuda.synchronize()
    print("pmc kernels done", flush=True)


if __name__ == "__main__":
    main()
