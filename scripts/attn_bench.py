"""Attention backend microbenchmark on MI355X: SDPA flash (aotriton / ck) fwd+bwd at the
Llama-3-8B bench shape (B=2, Hq=32, Hkv=8, S=4096, D=128, causal)."""
import time

import torch
import torch.nn.functional as F


def bench(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    B, Hq, Hk, S, D = 2, 32, 8, 4096, 128
    dev = "cuda"
    q = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, Hk, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, Hk, S, D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B, Hq, S, D, device=dev, dtype=torch.bfloat16)
    flops_f = 4 * B * Hq * S * S * D / 2
    libs = ["default"]
    try:
        print("preferred rocm fa lib:", torch.backends.cuda.preferred_rocm_fa_library())
        libs = ["aotriton", "ck"]
    except Exception as e:
        print("no preferred_rocm_fa_library:", e)
    for lib in libs:
        try:
            if lib != "default":
                torch.backends.cuda.preferred_rocm_fa_library(lib)
            for gqa in (True, False):
                def fwd():
                    if gqa:
                        return F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True)
                    kk = k.repeat_interleave(Hq // Hk, dim=1)
                    vv = v.repeat_interleave(Hq // Hk, dim=1)
                    return F.scaled_dot_product_attention(q, kk, vv, is_causal=True)

                def fb():
                    o = fwd()
                    o.backward(do)

                with torch.nn.attention.sdpa_kernel(torch.nn.attention.SDPBackend.FLASH_ATTENTION):
                    tf = bench(fwd)
                    tfb = bench(fb)
                print(f"{lib:9s} gqa={gqa}: fwd {tf:.2f} ms ({flops_f/tf/1e9:.0f} TF)  fwd+bwd {tfb:.2f} ms "
                      f"(bwd {tfb-tf:.2f} ms, {2.5*flops_f/(tfb-tf)/1e9:.0f} TF)")
        except Exception as e:
            print(lib, "failed:", repr(e)[:300])


if __name__ == "__main__":
    main()
