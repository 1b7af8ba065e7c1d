"""hipBLASLt vs rocBLAS (torch.backends.cuda.preferred_blas_library) on the Llama-3-8B GEMMs in
the layouts the step issues (forward TN, dgrad on W^T, wgrad on transposed copies)."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F


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
    T, H, I, V, kv = 8192, 4096, 14336, 128256, 1024
    lin = {"qkv": (H, H + 2 * kv), "o": (H, H), "gu": (H, 2 * I), "down": (I, H), "lm": (H, V)}
    tot = {}
    for name, (K, N) in lin.items():
        x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        gy = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
        wt, gt, xt = w.t().contiguous(), gy.t().contiguous(), x.t().contiguous()
        dw = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        cases = {"fwd": lambda: F.linear(x, w), "dgrad": lambda: F.linear(gy, wt),
                 "wgrad": lambda: torch.mm(gt, xt.t(), out=dw)}
        for kind, fn in cases.items():
            r = {"name": f"{name}_{kind}"}
            for lib in ("hipblaslt", "cublas"):
                torch.backends.cuda.preferred_blas_library(lib)
                r[lib] = round(timeit(fn) * 1e3, 4)
                tot[lib] = tot.get(lib, 0.0) + r[lib]
            print(json.dumps(r), flush=True)
        del x, w, gy, wt, gt, xt, dw
        torch.cuda.empty_cache()
    torch.backends.cuda.preferred_blas_library("hipblaslt")
    print(json.dumps({"total_ms_per_layer_set": tot}), flush=True)


if __name__ == "__main__":
    main()
