"""Linear layers whose weight gradient is produced directly inside the flat gradient buffer.

With ``FlatParameters`` every ``weight.grad`` is a view into one contiguous buffer. A stock
``nn.Linear`` backward computes ``dW`` into a fresh tensor and autograd's AccumulateGrad then adds
it into that view (an extra HBM round trip per weight, plus the buffer's zero-fill every step).
Here the backward GEMM writes ``dW`` straight into the view: ``mm(..., out=view)`` on the first
accumulation after ``zero_grad`` (the flat buffer's zero-fill skips these regions) and
``addmm_`` for later micro-batches (gradient accumulation). The DDP bucket bookkeeping that
AccumulateGrad hooks would have done is notified directly (``_rca_grad_ready``).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops

# RCA_BWD_TRANSPOSED=0 keeps the plain (transposed-operand) GEMM calls, for A/B measurements
_TRANSPOSED = os.environ.get("RCA_BWD_TRANSPOSED", "1") != "0"


class _LinearWgradIntoFlat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, x_t):
        # x_t: the input already transposed ([K, T], by its producer): saved instead of x, which
        # backward only needs for the weight gradient
        ctx.save_for_backward(x_t if x_t is not None else x)
        ctx.has_t = x_t is not None
        ctx.weight = weight
        return F.linear(x, weight)

    @staticmethod
    def backward(ctx, gy):
        (xs,) = ctx.saved_tensors
        w = ctx.weight
        g2 = gy.reshape(-1, gy.shape[-1])
        g_t = ops.pop_grad_transposed(g2)
        if ctx.has_t:
            x_t, x2 = xs, None
        else:
            x_t, x2 = None, xs.reshape(-1, xs.shape[-1])
        tr = _use_transposed(g2, x2, w, x_t)
        if ctx.needs_input_grad[0]:
            gx = _dgrad(gy, g2, w) if tr else torch.matmul(gy, w)
        else:
            gx = None
        view = _flat_view(w, g2.dtype)
        if view is None:
            return gx, _wgrad(g2, x2, tr, g_t=g_t, x_t=x_t).to(w.dtype), None
        _wgrad(g2, x2, tr, out=view, accumulate=not _take_fresh(w), g_t=g_t, x_t=x_t)
        _notify(w)
        return gx, None, None


class _SwiGLUDownIntoFlat(torch.autograd.Function):
    """``down(swiglu(gu))`` with the down projection's dW going into the flat gradient buffer and
    its input gradient never materialised: backward runs the fused gfx950 GEMM whose epilogue
    applies the SwiGLU backward (``ops.gemm_swiglu_bwd``: dgu and dgu^T straight from the dh
    accumulators), replacing the dh GEMM output + the separate ``swiglu_bwd_tr`` pass.
    Forward = ``ops.swiglu(gu, with_transposed=True)`` (act^T feeds the down wgrad) + ``F.linear``."""

    @staticmethod
    def forward(ctx, gu, weight):
        act, act_t = ops.swiglu(gu.detach(), with_transposed=True)
        ctx.save_for_backward(gu, act_t)
        ctx.weight = weight
        return F.linear(act, weight)

    @staticmethod
    def backward(ctx, gy):
        gu, act_t = ctx.saved_tensors
        w = ctx.weight
        g2 = gy.reshape(-1, gy.shape[-1])
        g_t = ops.pop_grad_transposed(g2)
        dgu = None
        if ctx.needs_input_grad[0]:
            wt = weight_t(w)
            if ops.gemm_swiglu_bwd_supported(g2, wt, gu):
                dgu, dgu_t = ops.gemm_swiglu_bwd(g2, wt, gu)
                ops.put_grad_transposed(dgu, dgu_t)
            else:  # the unfused pair: dh GEMM, then the SwiGLU backward (+ transposed copy)
                dgu = ops.swiglu_backward(gu, F.linear(g2, wt), with_transposed=True)
        view = _flat_view(w, g2.dtype)
        if view is None:
            return dgu, _wgrad(g2, None, True, g_t=g_t, x_t=act_t).to(w.dtype)
        _wgrad(g2, None, True, out=view, accumulate=not _take_fresh(w), g_t=g_t, x_t=act_t)
        _notify(w)
        return dgu, None


def swiglu_down(gu, down: "FusedWgradLinear"):
    """``down(swiglu(gu))``: the fused path when the down weight writes into a flat gradient
    buffer and the operands fit the fused kernel's contract; otherwise the two separate ops."""
    w = down.weight
    if (gu.is_cuda and torch.is_grad_enabled() and w.requires_grad and getattr(w, "_rca_flat_grad", False)
            and _FUSE_SWIGLU_BWD and gu.dim() == 2 and ops.transpose_supported(gu)
            and gu.shape[0] % 256 == 0 and w.shape[1] % 256 == 0 and w.shape[0] % 128 == 0):
        return _SwiGLUDownIntoFlat.apply(gu, w)
    if gu.is_cuda and torch.is_grad_enabled() and getattr(w, "_rca_flat_grad", False):
        act, act_t = ops.swiglu(gu, with_transposed=True)
        return down(act, x_t=act_t)
    return down(ops.swiglu(gu))


# RCA_FUSE_SWIGLU_BWD=1 selects the fused down dgrad + SwiGLU backward. Off by default: in the 8B
# step it measured 357.6 vs 354.1 ms/step unfused (profiles/gemm_r4.md): the epilogue still moves
# g, u, dgu and dgu^T (1.4 GB per layer), so the fusion only saves dh's write + read, less than
# the hand GEMM's gap to hipBLASLt on this product plus the epilogue's own issue cost.
_FUSE_SWIGLU_BWD = os.environ.get("RCA_FUSE_SWIGLU_BWD", "0") == "1"


# Per-shape input-gradient plans, (out_features, in_features) of the weight -> plan. "hand": the
# gfx950 GEMM (variant 7) on gy and the W^T copy instead of hipBLASLt. gate_up of the 8B model:
# 1,564-1,569 vs 1,533 TF/s (profiles/gemm_r4_v7.json, gpurun_out/r4h_gemm.json).
_DGRAD_PLAN = {(28672, 4096): "hand"}
_DGRAD_PLANS_ON = os.environ.get("RCA_DGRAD_PLAN", "1") != "0"


def _dgrad(gy, g2, w):
    """gy @ W on the reduction-contiguous W^T copy (hipBLASLt, or the hand GEMM per plan)."""
    wt = weight_t(w)
    if _DGRAD_PLANS_ON and _DGRAD_PLAN.get(tuple(w.shape)) == "hand" and ops.gemm_supported(
            g2.shape[0], wt.shape[0], g2.shape[1], g2, wt):
        return ops.gemm(g2, wt).view(*gy.shape[:-1], wt.shape[0])
    return F.linear(gy, wt)


def weight_t(w):
    """``w.t().contiguous()``: the W^T copy the fused AdamW update (``parallel/optim.py::
    FlatAdamW._setup_transposed``) or the ZeRO forward pre-hook keeps current when it is valid, else a transpose pass (into that buffer
    when the weight has one, so later uses in the same step reuse it)."""
    wt = getattr(w, "_rca_wt", None)
    if wt is None:
        return ops.transpose(w)
    key = (w._version, w._rca_wt_epoch[0])
    ev = getattr(w, "_rca_wt_ev", None)
    if ev is not None:  # produced on a side stream (ZeRO: fsdp.ShardedDataParallel._refresh_wt)
        torch.cuda.current_stream(wt.device).wait_event(ev)
        w._rca_wt_ev = None
    if w._rca_wt_key != key:
        ops.transpose(w, out=wt)
        w._rca_wt_key = key
    return wt


def _use_transposed(g2, x2, w, x_t=None) -> bool:
    # Reduction-contiguous operands: both backward products have their reduction dim as the
    # OUTER dim of one (dgrad: W) or both (wgrad: gy, x) operands, which hipBLASLt runs at
    # 0.93-1.33 PF/s at the 8B shapes; on transposed copies the same products run at
    # 1.29-1.58 PF/s (scripts/gemm_layout.py). The copies come from one HBM-rate HIP pass each.
    x_ok = (x_t is not None and x_t.is_cuda and x_t.is_contiguous()) or (x2 is not None and ops.transpose_supported(x2))
    return _TRANSPOSED and ops.transpose_supported(g2) and x_ok and ops.transpose_supported(w)


# Per-shape weight-gradient plans, (dW rows, dW cols, tokens) -> plan, measured on 1x MI355X
# (scripts/gemm_policy.py, profiles/gemm_policy_r3.md) against the default (hipBLASLt on both
# operands transposed, producer copies free):
#   "hand": the gfx950 hand GEMM on the natural token-outer operands (no transposes). o_proj:
#           0.222 ms vs 0.187 + 2 x 0.026 transposes = 0.240 ms.
#   "trB":  only the activation is transposed; hipBLASLt reads the gradient token-outer. lm_head:
#           6.67 + 0.03 ms vs 5.83 + 0.92 (the 2.1 GB dlogits transpose) + 0.03 ms.
_WGRAD_PLAN = {(4096, 4096, 8192): "hand", (128256, 4096, 8192): "trB"}
_PLANS_ON = os.environ.get("RCA_WGRAD_PLAN", "1") != "0"


def _wgrad_plan(g2, x2, x_t, g_t, out):
    if not _PLANS_ON or g_t is not None:
        return None
    N, T = g2.shape[1], g2.shape[0]
    K = x_t.shape[0] if x_t is not None else x2.shape[1]
    plan = _WGRAD_PLAN.get((N, K, T))
    if plan == "hand" and (x2 is None or out is None or not ops.gemm_supported(N, K, T, g2, x2, out)):
        return None
    return plan


def _wgrad(g2, x2, tr, out=None, accumulate=False, g_t=None, x_t=None):
    """dW = g2^T @ x2 (into ``out``, accumulating when asked). ``g_t`` / ``x_t``: transposed
    copies a producer already wrote (no transpose pass for them)."""
    plan = _wgrad_plan(g2, x2, x_t, g_t, out) if tr else None
    if plan == "hand":
        return ops.gemm(g2, x2, a_kmajor=True, b_kmajor=True, out=out, accumulate=accumulate)
    if plan == "trB":
        a = g2.t()
        b = (x_t if x_t is not None else ops.transpose(x2)).t()
        return out.addmm_(a, b) if (out is not None and accumulate) else torch.mm(a, b, out=out)
    if tr:
        a = g_t if g_t is not None else ops.transpose(g2)
        b = (x_t if x_t is not None else ops.transpose(x2)).t()
    else:
        a = g2.t() if g_t is None else g_t
        b = x2 if x_t is None else x_t.t()
    if out is None:
        return torch.mm(a, b)
    if accumulate:
        return out.addmm_(a, b)
    return torch.mm(a, b, out=out)


def _flat_view(w, dtype):
    """``w.grad`` when it is a fused-wgrad view into a flat gradient buffer of ``dtype``."""
    view = w.grad
    if view is None or not getattr(w, "_rca_flat_grad", False) or view.dtype != dtype:
        return None
    return view


def _take_fresh(w) -> bool:
    fresh = getattr(w, "_rca_grad_fresh", False)
    if fresh:
        w._rca_grad_fresh = False
    return fresh


def _notify(w):
    cb = getattr(w, "_rca_grad_ready", None)
    if cb is not None:
        cb(w)


class _FusedLinearCrossEntropy(torch.autograd.Function):
    """mean CE(h @ W^T, labels) with the logits produced and consumed chunk by chunk.

    The loss is the last op of the step, so its gradients are computed in FORWARD while each
    logits chunk is hot: lm_head GEMM (hipBLASLt) -> one-pass HIP CE kernel that overwrites the
    chunk with ``(softmax - onehot) / n_valid`` -> dgrad (dh chunk) and wgrad (accumulated dW)
    GEMMs. Backward only scales by the incoming gradient (a device scalar: no host sync).
    Peak extra memory: one ``chunk x V`` bf16 logits buffer + dW, instead of the full ``T x V``
    logits plus their gradient.
    """

    @staticmethod
    def forward(ctx, h, weight, labels, ignore_index, chunk):
        T, H = h.shape
        V = weight.shape[0]
        labels = labels.reshape(-1)
        valid = labels != ignore_index
        inv_n = (1.0 / valid.sum().clamp_min(1).float()).reshape(1)
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        rows = torch.empty(T, device=h.device, dtype=torch.float32)
        dh = torch.empty_like(h) if need_h else None
        dw = torch.empty_like(weight) if need_w else None
        buf = torch.empty(min(chunk, T), V, device=h.device, dtype=h.dtype)
        wt = weight_t(weight) if (need_h and _TRANSPOSED and ops.transpose_supported(weight)) else None
        for i, c0 in enumerate(range(0, T, chunk)):
            c1 = min(T, c0 + chunk)
            hc, lg = h[c0:c1], buf[: c1 - c0]
            torch.mm(hc, weight.t(), out=lg)
            rows[c0:c1] = ops.ce_fused_(lg, labels[c0:c1], inv_n, ignore_index)
            if need_h:
                if wt is not None:
                    torch.mm(lg, wt.t(), out=dh[c0:c1])
                else:
                    torch.mm(lg, weight, out=dh[c0:c1])
            if need_w:
                _wgrad(lg, hc, _use_transposed(lg, hc, weight), out=dw, accumulate=i > 0)
        ctx.save_for_backward(dh, dw)
        ctx.weight = weight
        return rows.sum() * inv_n[0]

    @staticmethod
    def backward(ctx, g):
        dh, dw = ctx.saved_tensors
        w = ctx.weight
        gh = dh.mul_(g) if dh is not None else None
        if dw is None:
            return gh, None, None, None, None
        view = _flat_view(w, dw.dtype)
        if view is None:
            return gh, dw.mul_(g), None, None, None
        if _take_fresh(w):
            torch.mul(dw, g, out=view)
        else:
            view.addcmul_(dw, g.reshape(1, 1).to(dw.dtype))
        _notify(w)
        return gh, None, None, None, None


def linear_cross_entropy(h, weight, labels, ignore_index: int = -100, chunk_tokens: int = 0):
    """Mean cross-entropy of ``h @ weight.T`` against ``labels`` without materialising the full
    logits (GPU: chunked, fused HIP CE; CPU: the plain PyTorch reference).
    ``chunk_tokens`` = 0 picks chunks of <= 1 GiB of bf16 logits."""
    V = weight.shape[0]
    if not h.is_cuda or not ops.ce_fused_supported(V) or h.dtype != torch.bfloat16:
        return F.cross_entropy(F.linear(h, weight).float(), labels.reshape(-1), ignore_index=ignore_index)
    if chunk_tokens <= 0:
        chunk_tokens = max(256, (1 << 30) // (2 * V) // 256 * 256)
    return _FusedLinearCrossEntropy.apply(h.contiguous(), weight, labels, ignore_index, int(chunk_tokens))


class FusedWgradLinear(nn.Linear):
    """``nn.Linear`` (no bias) whose dW lands directly in the flat gradient buffer."""

    def __init__(self, in_features, out_features, bias=False, device=None, dtype=None):
        if bias:
            raise ValueError("FusedWgradLinear has no bias")
        super().__init__(in_features, out_features, bias=False, device=device, dtype=dtype)
        self.weight._rca_fused_wgrad = True

    def forward(self, x, labels=None, ignore_index: int = -100, ce_chunk: int = 0, x_t=None):
        """``labels`` given: returns the mean cross-entropy of ``x @ W^T`` through the fused,
        chunked linear + CE path (the full logits are never materialised). ``x_t``: ``x``
        already transposed by its producer (saved for the weight gradient instead of ``x``)."""
        if labels is not None:
            return linear_cross_entropy(x, self.weight, labels, ignore_index, ce_chunk)
        if torch.is_grad_enabled() and self.weight.requires_grad and getattr(self.weight, "_rca_flat_grad", False):
            return _LinearWgradIntoFlat.apply(x, self.weight, x_t)
        return F.linear(x, self.weight)


class _EmbeddingIntoFlat(torch.autograd.Function):
    """Embedding lookup whose weight gradient goes straight into the flat gradient buffer instead
    of a dense ``V x H`` gradient tensor that AccumulateGrad then adds into it (for Llama-3-8B a
    1 GB temporary plus a 3 GB add pass per step): torch's deterministic, fp32-accumulating
    embedding backward runs over the step's UNIQUE token ids only (<= T rows), and those rows are
    added into the buffer with one non-colliding ``index_put_``."""

    @staticmethod
    def forward(ctx, idx, weight):
        ctx.save_for_backward(idx)
        ctx.weight = weight
        return F.embedding(idx, weight)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        w = ctx.weight
        g2 = g.reshape(-1, g.shape[-1])
        view = w.grad
        flat_idx = idx.reshape(-1)
        if (view is not None and view.dtype == g2.dtype and view.is_contiguous()
                and getattr(w, "_rca_grad_ready", None) is not None):
            uniq, inv = torch.unique(flat_idx, return_inverse=True)
            rows = torch.ops.aten.embedding_dense_backward(g2, inv, uniq.numel(), -1, False)
            view.index_put_((uniq,), rows, accumulate=True)
            w._rca_grad_ready(w)
            return None, None
        return None, torch.ops.aten.embedding_dense_backward(g2, flat_idx, w.shape[0], -1, False)


class FusedEmbedding(nn.Embedding):
    """``nn.Embedding`` whose gradient lands directly in the flat gradient buffer."""

    def forward(self, idx):
        if (torch.is_grad_enabled() and self.weight.requires_grad and idx.is_cuda and self.padding_idx is None
                and self.max_norm is None and not self.sparse):
            return _EmbeddingIntoFlat.apply(idx, self.weight)
        return super().forward(idx)

