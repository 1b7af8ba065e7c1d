"""Attention microbenchmark on MI355X at the Llama-3-8B bench shape (B=2, Hq=32, Hkv=8, S=4096,
D=128, causal): the framework's gfx950 flash attention vs torch SDPA (aotriton)."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402


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
    B, Hq, Hk, S, D = 2, 32, 8, int(os.environ.get("ATTN_S", 4096)), 128
    dev = "cuda"
    qkv = torch.randn(B * S, (Hq + 2 * Hk) * D, device=dev, dtype=torch.bfloat16, requires_grad=True)
    do = torch.randn(B * S, Hq * D, device=dev, dtype=torch.bfloat16)
    flops_f = 4 * B * Hq * S * S * D / 2

    def run(name, fwd):
        def fb():
            fwd().backward(do)
        tf = bench(fwd)
        tfb = bench(fb)
        print(f"{name:10s}: fwd {tf:.3f} ms ({flops_f / tf / 1e9:.0f} TF)  fwd+bwd {tfb:.3f} ms "
              f"(bwd {tfb - tf:.3f} ms, {2.5 * flops_f / (tfb - tf) / 1e9:.0f} TF)", flush=True)

    run("rca-hip", lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
    if os.environ.get("ATTN_BWD_AB"):  # interleaved A/B of the backward modes (0: recompute dQ, 1: dS tiles)
        lib = ops._lib.lib()
        for _ in range(3):
            for mode in (0, 1):
                prev = lib.rca_attn_set_bwd_mode(mode)
                run(f"bwd-mode{mode}", lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
                lib.rca_attn_set_bwd_mode(prev)
    if os.environ.get("ATTN_NOPS_AB"):  # interleaved A/B of the dS kernel's MFMA wait states
        lib = ops._lib.lib()
        for _ in range(3):
            for n in (3, 1):
                prev = lib.rca_attn_set_hs_nops(n)
                run(f"nops-{n}", lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
                lib.rca_attn_set_hs_nops(prev)
    if os.environ.get("ATTN_DQQW_AB"):  # interleaved A/B: dQ-from-dS with 1 or 2 query blocks per wave
        lib = ops._lib.lib()
        for _ in range(3):
            for qw in (1, 2):
                prev = lib.rca_attn_set_dq_qw(qw)
                run(f"dq-qw{qw}", lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
                lib.rca_attn_set_dq_qw(prev)
    if os.environ.get("ATTN_FWDNW_AB"):  # interleaved A/B: 4-wave (2 WG/CU) vs 8-wave (256-row WG) forward
        lib = ops._lib.lib()
        for _ in range(3):
            for nw in (4, 8):
                prev = lib.rca_attn_set_fwd_nw(nw)
                run(f"fwd-nw{nw}", lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
                lib.rca_attn_set_fwd_nw(prev)
    if os.environ.get("ATTN_WIDE_AB"):  # interleaved A/B of the forward variants
        lib = ops._lib.lib()
        for _ in range(3):
            for mode in (0, 1, 2):
                prev = lib.rca_attn_set_fwd_mode(mode)
                run(f"fwd-{('narrow', 'wide', 'hs')[mode]}",
                    lambda: ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
                lib.rca_attn_set_fwd_mode(prev)

    def sdpa():
        q = qkv[:, : Hq * D].view(B, S, Hq, D).transpose(1, 2)
        k = qkv[:, Hq * D: (Hq + Hk) * D].view(B, S, Hk, D).transpose(1, 2)
        v = qkv[:, (Hq + Hk) * D:].view(B, S, Hk, D).transpose(1, 2)
        return F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True).transpose(1, 2).reshape(
            B * S, Hq * D)

    with torch.nn.attention.sdpa_kernel(torch.nn.attention.SDPBackend.FLASH_ATTENTION):
        run("sdpa", sdpa)


if __name__ == "__main__":
    main()
