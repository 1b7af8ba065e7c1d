"""Llama-3-8B training GEMMs on MI355X: default hipBLASLt heuristic vs TunableOp-selected solutions.

    python scripts/gemm_tune.py --tune --out ray_community_amd/ops/tuned/gemm_mi355x.csv

Shapes are exactly the ones the training step issues (T = micro_batch * seq_len tokens):
forward ``F.linear(x[T,K], W[N,K])``, input grad ``gy[T,N] @ W[N,K]`` and weight grad
``gy[T,N]^T @ x[T,K]`` (written into the flat grad buffer). Prints TFLOP/s per shape for both.
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F


def shapes(T=8192, H=4096, I=14336, V=128256, kv=1024):
    lin = {"qkv": (H, H + 2 * kv), "o": (H, H), "gate_up": (H, 2 * I), "down": (I, H), "lm_head": (H, V)}
    out = []
    for name, (K, N) in lin.items():
        out.append((f"{name}.fwd", "fwd", T, K, N))
        out.append((f"{name}.dgrad", "dgrad", T, K, N))
        out.append((f"{name}.wgrad", "wgrad", T, K, N))
        # the layouts the training step issues with RCA_BWD_TRANSPOSED=1 (parallel/fused_linear.py):
        # dgrad = F.linear(gy, W^T) and wgrad = gy^T @ (x^T)^T on producer-transposed copies
        out.append((f"{name}.dgrad_tr", "dgrad_tr", T, K, N))
        out.append((f"{name}.wgrad_tr", "wgrad_tr", T, K, N))
    return out


def make(kind, T, K, N, dev):
    x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    gy = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
    dw = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    if kind == "fwd":
        return lambda: F.linear(x, w)
    if kind == "dgrad":
        return lambda: torch.matmul(gy, w)
    if kind == "dgrad_tr":
        wt = w.t().contiguous()
        return lambda: F.linear(gy, wt)
    if kind == "wgrad_tr":
        gt, xt = gy.t().contiguous(), x.t().contiguous()
        return lambda: torch.mm(gt, xt.t(), out=dw)
    return lambda: torch.mm(gy.t(), x, out=dw)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def _heartbeat():
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(30)
            print(f"  ... {time.time() - t0:.0f}s", flush=True)

    threading.Thread(target=beat, daemon=True).start()


def main():
    _heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", action="store_true")
    ap.add_argument("--out", default="gpurun_out/gemm_tuned.csv")
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--tune-ms", type=int, default=30, help="TunableOp time budget per candidate solution")
    ap.add_argument("--table", default=None, help="compare default vs an existing tuned table (no tuning)")
    a = ap.parse_args()
    dev = "cuda"
    res = {}
    for name, kind, T, K, N in shapes(a.tokens):
        fn = make(kind, T, K, N, dev)
        res[name] = [timeit(fn), None]
        torch.cuda.empty_cache()
    if a.table:
        import torch.cuda.tunable as tun

        tun.enable(True)
        tun.tuning_enable(False)
        tun.read_file(a.table)
        for name, kind, T, K, N in shapes(a.tokens):
            res[name][1] = timeit(make(kind, T, K, N, dev))
            torch.cuda.empty_cache()
    elif a.tune:
        import torch.cuda.tunable as tun

        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_filename(a.out)
        if os.path.exists(a.out):
            tun.read_file(a.out)  # resume: shapes already in the table are not re-tuned
        tun.set_max_tuning_duration(a.tune_ms)
        tun.set_max_tuning_iterations(10)
        for name, kind, T, K, N in shapes(a.tokens):
            fn = make(kind, T, K, N, dev)
            fn()  # tunes this shape
            torch.cuda.synchronize()
            print(f"tuned {name}", flush=True)
            torch.cuda.empty_cache()
        tun.tuning_enable(False)  # the table is written to a.out when the process exits
        for name, kind, T, K, N in shapes(a.tokens):
            fn = make(kind, T, K, N, dev)
            res[name][1] = timeit(fn)
            torch.cuda.empty_cache()
    tot0 = tot1 = 0.0
    print(f"{'gemm':16s} {'M x N x K':>22s} {'default ms':>10s} {'TF/s':>7s} {'tuned ms':>9s} {'TF/s':>7s}")
    for name, kind, T, K, N in shapes(a.tokens):
        fl = 2.0 * T * K * N
        t0, t1 = res[name]
        tot0 += t0
        tot1 += t1 or t0
        m, n, k = {"fwd": (T, N, K), "dgrad": (T, K, N), "wgrad": (N, K, T), "dgrad_tr": (T, K, N),
                   "wgrad_tr": (N, K, T)}[kind]
        s1 = f"{1e3 * t1:9.3f} {fl / t1 / 1e12:7.0f}" if t1 else ""
        print(f"{name:16s} {f'{m}x{n}x{k}':>22s} {1e3 * t0:10.3f} {fl / t0 / 1e12:7.0f} {s1}", flush=True)
    print(f"per-layer-set total: default {1e3 * tot0:.2f} ms, tuned {1e3 * tot1:.2f} ms")


if __name__ == "__main__":
    sys.exit(main())
