"""Llama-3 decoder (the model behind the Ray Train Llama-3-8B DDP headline benchmark).

MI355X-first layout choices:
  * fused QKV projection ([T, (Hq + 2*Hkv) * D]) with RoPE applied IN PLACE on its q/k heads
    by one HIP kernel (no q/k copies);
  * fused gate|up projection feeding the HIP SwiGLU kernel;
  * residual add fused into the following RMSNorm (HIP kernel emits both the new residual
    stream and the normalised activations; its backward adds the residual gradient);
  * HIP cross-entropy writing dlogits in place over the 128k-vocab logits, or (``fused_ce``)
    lm_head + CE fused chunk by chunk so the T x 128k logits are never materialised;
  * activations kept resident (no recomputation) — 288 GB HBM holds a full 8B replica with
    fp32 master weights + AdamW states + seq-4096 activations per GPU.
Attention is the framework's own MFMA flash-attention HIP kernels (``ops.attention``: causal,
GQA, XCD-grouped workgroup order); GEMMs are hipBLASLt via torch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..parallel.fused_linear import FusedEmbedding, FusedWgradLinear, swiglu_down


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    max_seq_len: int = 8192
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    init_std: float = 0.02
    name: str = "llama"
    attn_impl: str = "hip"  # "hip" (gfx950 flash attention kernels) | "sdpa" (torch SDPA / aotriton)
    fused_ce: bool = False  # chunked lm_head + one-pass HIP CE (parallel/fused_linear.py): no T x V logits
    ce_chunk: int = 0       # tokens per fused-CE chunk (0: <= 1 GiB of logits per chunk)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    def num_params(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        kv = self.num_kv_heads * self.head_dim
        per_layer = H * (H + 2 * kv) + H * H + 2 * H * I + I * H + 2 * H
        emb = V * H * (1 if self.tie_embeddings else 2)
        return L * per_layer + emb + H

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token: 6 * matmul params + causal attention (fwd+bwd)."""
        H, L = self.hidden_size, self.num_layers
        n_matmul = self.num_params() - self.vocab_size * H * (0 if self.tie_embeddings else 1) - (2 * L + 1) * H
        attn = 6 * L * H * seq_len  # 12*L*H*S/2 (causal): QK^T + PV, fwd + 2x bwd
        return 6 * n_matmul + attn


PRESETS = {
    "llama3-8b": LlamaConfig(name="llama3-8b"),
    "llama3-70b": LlamaConfig(hidden_size=8192, intermediate_size=28672, num_layers=80, num_heads=64, num_kv_heads=8,
                              name="llama3-70b"),
    "llama3-1b": LlamaConfig(hidden_size=2048, intermediate_size=8192, num_layers=16, num_heads=32, num_kv_heads=8,
                             tie_embeddings=True, name="llama3-1b"),
    "llama3-tiny": LlamaConfig(vocab_size=1024, hidden_size=256, intermediate_size=512, num_layers=2, num_heads=4,
                               num_kv_heads=2, max_seq_len=256, name="llama3-tiny"),
}


class RMSNorm(nn.Module):
    def __init__(self, dim, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x, residual=None):
        return ops.rms_norm(x, self.weight, self.eps, residual)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        D = cfg.head_dim
        self.qkv = FusedWgradLinear(cfg.hidden_size, (cfg.num_heads + 2 * cfg.num_kv_heads) * D)
        self.o = FusedWgradLinear(cfg.num_heads * D, cfg.hidden_size)

    def forward(self, x, cs, B, S, positions=None):
        cfg = self.cfg
        D, Hq, Hk = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
        T = B * S
        qkv = self.qkv(x)  # [T, (Hq+2Hk)*D]
        qkv = ops.apply_rope_(qkv, cs, S, Hq, Hk, D, positions)
        if qkv.is_cuda and cfg.attn_impl == "hip" and ops.flash_attention_supported(S, D, Hq, Hk):
            # gfx950 flash attention straight off the fused projection; backward fills dqkv directly
            return self.o(ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True))
        q = qkv[:, : Hq * D].view(B, S, Hq, D).transpose(1, 2)
        k = qkv[:, Hq * D: (Hq + Hk) * D].view(B, S, Hk, D).transpose(1, 2)
        v = qkv[:, (Hq + Hk) * D:].view(B, S, Hk, D).transpose(1, 2)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=(Hk != Hq))
        o = o.transpose(1, 2).reshape(T, Hq * D)
        return self.o(o)


class MLP(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.gate_up = FusedWgradLinear(cfg.hidden_size, 2 * cfg.intermediate_size)
        self.down = FusedWgradLinear(cfg.intermediate_size, cfg.hidden_size)

    def forward(self, x):
        # On the flat-gradient GPU path SwiGLU also writes act^T (the down projection's wgrad
        # operand), and the backward's down dgrad GEMM applies the SwiGLU backward in its epilogue,
        # writing d(gate|up) and its transpose for the gate_up wgrad (parallel/fused_linear.py).
        return swiglu_down(self.gate_up(x), self.down)


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attn_norm = RMSNorm(cfg.hidden_size, cfg.norm_eps)
        self.attn = Attention(cfg)
        self.mlp_norm = RMSNorm(cfg.hidden_size, cfg.norm_eps)
        self.mlp = MLP(cfg)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        # untied: the lookup's gradient goes straight into the flat buffer; tied, the weight also
        # gets the lm-head gradient, so both must meet in autograd's single accumulation
        self.embed = (nn.Embedding if cfg.tie_embeddings else FusedEmbedding)(cfg.vocab_size, cfg.hidden_size)
        self.layers = nn.ModuleList([Block(cfg) for _ in range(cfg.num_layers)])
        self.norm = RMSNorm(cfg.hidden_size, cfg.norm_eps)
        self.lm_head = None if cfg.tie_embeddings else FusedWgradLinear(cfg.hidden_size, cfg.vocab_size)
        self._cs = {}
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = self.cfg.init_std
        out_std = std / math.sqrt(2 * self.cfg.num_layers)
        for name, p in self.named_parameters():
            if p.dim() == 1:
                p.fill_(1.0)
            elif name.endswith("o.weight") or name.endswith("down.weight"):
                p.normal_(0.0, out_std)
            else:
                p.normal_(0.0, std)

    def rope_table(self, device):
        key = str(device)
        t = self._cs.get(key)
        if t is None:
            t = ops.rope_cos_sin(self.cfg.max_seq_len, self.cfg.head_dim, self.cfg.rope_theta).to(device)
            self._cs[key] = t
        return t

    def hidden_states(self, tokens, positions=None):
        B, S = tokens.shape
        cs = self.rope_table(tokens.device)
        residual = self.embed(tokens).view(B * S, -1)
        h = self.layers[0].attn_norm(residual) if len(self.layers) else residual
        for i, blk in enumerate(self.layers):
            a = blk.attn(h, cs, B, S, positions)
            h, residual = blk.mlp_norm(a, residual=residual)
            m = blk.mlp(h)
            nxt = self.layers[i + 1].attn_norm if i + 1 < len(self.layers) else self.norm
            h, residual = nxt(m, residual=residual)
        if not len(self.layers):
            h = self.norm(residual)
        return h  # [T, H], final-normed

    def logits(self, h):
        if self.lm_head is not None:
            return self.lm_head(h)
        return F.linear(h, self.embed.weight)

    def forward(self, tokens, labels=None, positions=None):
        h = self.hidden_states(tokens, positions)
        if labels is not None and self.cfg.fused_ce and h.is_cuda:
            if self.lm_head is not None:  # through the module call so wrapper hooks still fire
                return self.lm_head(h, labels=labels.reshape(-1), ce_chunk=self.cfg.ce_chunk)
            from ..parallel.fused_linear import linear_cross_entropy

            return linear_cross_entropy(h, self.embed.weight, labels.reshape(-1), chunk_tokens=self.cfg.ce_chunk)
        logits = self.logits(h)
        if labels is None:
            return logits.view(*tokens.shape, -1)
        return ops.cross_entropy(logits, labels.reshape(-1), inplace_backward=True)


def build_llama(name_or_cfg="llama3-8b", device=None, dtype=torch.bfloat16, **overrides) -> Llama:
    cfg = PRESETS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg
    if overrides:
        cfg = LlamaConfig(**{**cfg.__dict__, **overrides})
    if device is not None and str(device).startswith("cuda"):
        with torch.device(device):
            m = Llama(cfg)
    else:
        m = Llama(cfg)
    return m.to(dtype=dtype)
