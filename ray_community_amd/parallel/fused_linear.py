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
    def forward(ctx, x, weight):
        ctx.save_for_backward(x)
        ctx.weight = weight
        return F.linear(x, weight)

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        w = ctx.weight
        g2 = gy.reshape(-1, gy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        # Reduction-contiguous operands: both backward products have their reduction dim as the
        # OUTER dim of one (dgrad: W) or both (wgrad: gy, x) operands, which hipBLASLt runs at
        # 0.93-1.33 PF/s at the 8B shapes; on transposed copies the same products run at
        # 1.29-1.58 PF/s (scripts/gemm_layout.py). The copies come from one HBM-rate HIP pass each.
        tr = _TRANSPOSED and ops.transpose_supported(g2) and ops.transpose_supported(x2) and ops.transpose_supported(w)
        if ctx.needs_input_grad[0]:
            gx = F.linear(gy, ops.transpose(w)) if tr else torch.matmul(gy, w)
        else:
            gx = None
        if tr:
            a, b = ops.transpose(g2), ops.transpose(x2).t()
        else:
            a, b = g2.t(), x2
        view = w.grad
        if view is None or not getattr(w, "_rca_flat_grad", False) or view.dtype != g2.dtype:
            return gx, torch.mm(a, b).to(w.dtype)  # plain autograd accumulation
        if getattr(w, "_rca_grad_fresh", False):
            torch.mm(a, b, out=view)
            w._rca_grad_fresh = False
        else:
            view.addmm_(a, b)
        cb = getattr(w, "_rca_grad_ready", None)
        if cb is not None:
            cb(w)
        return gx, None


class FusedWgradLinear(nn.Linear):
    """``nn.Linear`` (no bias) whose dW lands directly in the flat gradient buffer."""

    def __init__(self, in_features, out_features, bias=False, device=None, dtype=None):
        if bias:
            raise ValueError("FusedWgradLinear has no bias")
        super().__init__(in_features, out_features, bias=False, device=device, dtype=dtype)
        self.weight._rca_fused_wgrad = True

    def forward(self, x):
        if torch.is_grad_enabled() and self.weight.requires_grad and getattr(self.weight, "_rca_flat_grad", False):
            return _LinearWgradIntoFlat.apply(x, self.weight)
        return F.linear(x, self.weight)
