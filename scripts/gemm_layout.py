"""Operand-layout study of the Llama-3-8B backward GEMMs on MI355X (hipBLASLt via torch).

wgrad dW[N,K] = gy[T,N]^T @ x[T,K]: both operands have the reduction dim T outermost. Compare with
the same product on pre-transposed, reduction-contiguous copies (gyT[N,T] @ xT[K,T]^T), and price
the transposes. dgrad dx = gy @ W[N,K]: compare with a reduction-contiguous W^T copy.
"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_tune import shapes, timeit  # noqa: E402


def main():
    dev = "cuda"
    print(f"{'gemm':22s} {'TxKxN':>20s} {'cur ms':>8s} {'TF':>6s} {'alt ms':>8s} {'TF':>6s} {'transp ms':>9s}", flush=True)
    tot_cur = tot_alt = 0.0
    for name, kind, T, K, N in shapes():
        if kind == "fwd" or name.startswith("lm_head"):
            continue
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        gy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * T * K * N
        if kind == "wgrad":
            dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
            gyT, xT = gy.t().contiguous(), x.t().contiguous()
            cur = timeit(lambda: torch.mm(gy.t(), x, out=dw))
            alt = timeit(lambda: torch.mm(gyT, xT.t(), out=dw))
            tr = timeit(lambda: (gy.t().contiguous(), x.t().contiguous()))
            ref = torch.mm(gy.t().float()[:64], x.float())
            assert torch.allclose(torch.mm(gyT, xT.t())[:64].float(), ref, rtol=2e-2, atol=2.0)
        else:
            wT = w.t().contiguous()
            cur = timeit(lambda: torch.matmul(gy, w))
            alt = timeit(lambda: F.linear(gy, wT))
            tr = timeit(lambda: w.t().contiguous())
        tot_cur += cur
        tot_alt += alt + tr
        print(f"{name:22s} {f'{T}x{K}x{N}':>20s} {cur*1e3:8.3f} {fl/cur/1e12:6.0f} {alt*1e3:8.3f} {fl/alt/1e12:6.0f} "
              f"{tr*1e3:9.3f}", flush=True)
        del x, w, gy
        torch.cuda.empty_cache()
    print(f"per-layer backward GEMMs: current {tot_cur*1e3:.2f} ms, alt+transposes {tot_alt*1e3:.2f} ms")


if __name__ == "__main__":
    main()
