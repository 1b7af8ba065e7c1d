"""Per-product layout policy for the Llama-3-8B backward GEMMs on MI355X.

For every backward product of one 8B layer and the lm_head, times (same process, interleaved):
  nat   hipBLASLt on the natural operands (reduction dim outermost on one or both operands)
  tr    hipBLASLt on reduction-contiguous copies (GEMM only)
  tA/tB the ops.transpose pass that makes each copy (HBM-rate LDS-tiled HIP kernel)
  hand  the gfx950 hand GEMM (ops.gemm) on the natural operands
One JSON line per product; fused_linear's policy table is read off these numbers.
"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402


def timeit(fn, iters=10, reps=3):
    best = 1e9
    for _ in range(reps):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        best = min(best, (time.perf_counter() - t0) / iters)
    return best


def main():
    dev = "cuda"
    T, H, I, V, kv = 8192, 4096, 14336, 128256, 1024
    lin = {"qkv": (H, H + 2 * kv), "o": (H, H), "gu": (H, 2 * I), "down": (I, H), "lm": (H, V)}
    tot = {}
    for name, (K, N) in lin.items():
        x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        gy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
        dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(T, K, device=dev, dtype=torch.bfloat16)
        # dgrad dx[T,K] = gy[T,N] @ w[N,K]
        wt = ops.transpose(w)
        r = {"name": f"{name}_dgrad", "T": T, "K": K, "N": N}
        r["nat"] = timeit(lambda: torch.matmul(gy, w, out=dx))
        r["tr"] = timeit(lambda: torch.mm(gy, wt.t(), out=dx))
        r["tB"] = timeit(lambda: ops.transpose(w, out=wt))
        if ops.gemm_supported(T, K, N, gy, w, dx):
            r["hand"] = timeit(lambda: ops.gemm(gy, w, b_kmajor=True, out=dx))
        print(json.dumps({k: (round(v * 1e3, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del wt
        # wgrad dw[N,K] = gy^T @ x
        gt, xt = ops.transpose(gy), ops.transpose(x)
        r = {"name": f"{name}_wgrad", "T": T, "K": K, "N": N}
        r["nat"] = timeit(lambda: torch.mm(gy.t(), x, out=dw))
        r["tr"] = timeit(lambda: torch.mm(gt, xt.t(), out=dw))
        r["tA"] = timeit(lambda: ops.transpose(gy, out=gt))
        r["tB"] = timeit(lambda: ops.transpose(x, out=xt))
        r["trA_only"] = timeit(lambda: torch.mm(gt, x, out=dw))
        r["trB_only"] = timeit(lambda: torch.mm(gy.t(), xt.t(), out=dw))
        if ops.gemm_supported(N, K, T, gy, x, dw):
            r["hand"] = timeit(lambda: ops.gemm(gy, x, a_kmajor=True, b_kmajor=True, out=dw))
        print(json.dumps({k: (round(v * 1e3, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del gt, xt, x, w, gy, dw, dx
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
