"""Flat parameter / gradient storage.

All trainable parameters of a module become views into ONE contiguous buffer, and their
``.grad`` views into ONE contiguous gradient buffer. This is what lets the framework
  * all-reduce gradients in a few large, contiguous buckets with zero packing copies
    (xGMI ring collectives are per-link bandwidth bound: fewer, larger messages win), and
  * run AdamW as one streaming HIP kernel over the whole model instead of a multi-tensor loop.

Parameters are laid out in REVERSE registration order (≈ the order in which backward produces
their gradients), decayed matrices first and the tiny no-decay vectors (norm weights, biases)
last, so gradient buckets fill front to back during backward.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional

import torch
import torch.nn as nn

ALIGN = 64  # elements; keeps every view 128-B aligned for 16-B vector access


def _round_up(n, a=ALIGN):
    return (n + a - 1) // a * a


def register_grad_ready(params, fn) -> list:
    """Call ``fn(p)`` exactly once per backward when ``p``'s gradient is final.

    Two sources report readiness: the post-accumulate-grad hook (AccumulateGrad), and the
    fused-wgrad linears (``parallel/fused_linear.py``), which write dW straight into the flat
    buffer and call ``p._rca_grad_ready``. The engine still runs the leaf's AccumulateGrad node
    (with an undefined gradient) after such a backward, so its hook fires too; the callback marks
    the parameter so that the hook call that follows is swallowed instead of counted twice.
    """

    def on_accumulate(p):
        if getattr(p, "_rca_grad_counted", False):
            p._rca_grad_counted = False
            return
        fn(p)

    def on_fused(p):
        p._rca_grad_counted = True
        fn(p)

    handles = []
    for p in params:
        handles.append(p.register_post_accumulate_grad_hook(on_accumulate))
        p._rca_grad_ready = on_fused
        p._rca_grad_counted = False
    return handles


def default_no_decay(name: str, p: torch.Tensor) -> bool:
    return p.dim() < 2 or name.endswith(".bias")


@dataclass
class Bucket:
    index: int
    start: int
    end: int
    params: List[nn.Parameter]


class FlatParameters:
    def __init__(self, module: nn.Module, bucket_cap_mb: float = 256.0,
                 no_decay: Callable[[str, torch.Tensor], bool] = default_no_decay, grad_dtype=None,
                 bucket_align: int = ALIGN):
        """``bucket_align``: every bucket starts and ends on a multiple of this many elements
        (sharded data parallel uses world * ALIGN so each bucket splits into equal per-rank,
        128-B aligned chunks for in-place reduce-scatter / all-gather)."""
        seen = set()
        named = []
        for name, p in module.named_parameters():
            if not p.requires_grad or id(p) in seen:
                continue
            seen.add(id(p))
            named.append((name, p))
        decay = [(n, p) for n, p in reversed(named) if not no_decay(n, p)]
        nodecay = [(n, p) for n, p in reversed(named) if no_decay(n, p)]
        self.names = [n for n, _ in decay + nodecay]
        self.params = [p for _, p in decay + nodecay]
        if not self.params:
            raise ValueError("module has no trainable parameters")
        if bucket_align % ALIGN:
            raise ValueError(f"bucket_align must be a multiple of {ALIGN}")
        dev = self.params[0].device
        dtype = self.params[0].dtype
        self.dtype = dtype
        self.device = dev
        gdt = grad_dtype or dtype
        esz = torch.empty((), dtype=gdt).element_size()
        cap = max(1, int(bucket_cap_mb * 1024 * 1024 / esz))
        # layout + buckets in one pass: contiguous ranges of the flat buffers; the no-decay tail
        # always gets its own bucket(s) (tiny, all-reduced last)
        offs: List[int] = []
        bounds = []  # (start, end, params)
        cur: List[nn.Parameter] = []
        start = o = 0
        n_decay = len(decay)
        self.decay_end = None
        for i, p in enumerate(self.params):
            n = _round_up(p.numel())
            if cur and (o + n - start > cap or i == n_decay):
                end = _round_up(o, bucket_align)
                bounds.append((start, end, cur))
                cur, start, o = [], end, end
            if i == n_decay:
                self.decay_end = o
            offs.append(o)
            o += n
            cur.append(p)
        end = _round_up(o, bucket_align)
        bounds.append((start, end, cur))
        if self.decay_end is None:
            self.decay_end = end
        self.bucket_align = bucket_align
        self.numel = end
        self.offsets = offs
        self.data = torch.zeros(end, dtype=dtype, device=dev)
        self.grad = torch.zeros(end, dtype=gdt, device=dev)
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                n = p.numel()
                self.data[off: off + n].copy_(p.data.reshape(-1))
                p.data = self.data[off: off + n].view_as(p)
                if gdt == dtype:
                    p.grad = self.grad[off: off + n].view_as(p)
        self.grad_is_view = gdt == dtype
        # wider buffer the data-parallel wrappers reduce into (fp32 gradient reduction); when set,
        # optimizers read their gradients from it instead of ``grad``
        self.reduced_grad: Optional[torch.Tensor] = None
        # device scalar: sum of squares of this step's final gradients, taken by the DDP wrapper
        # bucket by bucket during backward; consumed (and cleared) by the optimizer step
        self.precomputed_sumsq: Optional[torch.Tensor] = None
        self.buckets: List[Bucket] = [Bucket(i, s, e, ps) for i, (s, e, ps) in enumerate(bounds)]
        self.param_bucket = {}
        for b in self.buckets:
            for p in b.params:
                self.param_bucket[id(p)] = b.index
        self.param_offset = {id(p): off for p, off in zip(self.params, offs)}
        # Fused-wgrad linears (parallel/fused_linear.py) overwrite their gradient region on the first
        # accumulation, so zero_grad only has to clear the tail holding everything else -- valid
        # when all fused weights precede all other parameters in the layout.
        self.fused = [p for p in self.params if getattr(p, "_rca_fused_wgrad", False) and self.grad_is_view]
        fused_ids = {id(p) for p in self.fused}
        first_other = next((i for i, p in enumerate(self.params) if id(p) not in fused_ids), len(self.params))
        if self.fused and all(id(p) not in fused_ids for p in self.params[first_other:]):
            self.zero_start = offs[first_other] if first_other < len(self.params) else end
            for p in self.fused:
                p._rca_flat_grad = True
                p._rca_grad_fresh = True
        else:
            self.fused = []
            self.zero_start = 0

    def adopt_grad(self, p):
        """Make ``p.grad`` the flat-buffer view again if something replaced it (a torch optimizer's
        ``zero_grad(set_to_none=True)`` drops the view, and the next backward then accumulates into
        a fresh tensor that the bucket collectives would never see): copy the fresh gradient into
        the parameter's slot and re-point ``p.grad`` at it. No-op in the normal case."""
        if not self.grad_is_view:
            return
        g = p.grad
        if g is None:
            return
        off = self.param_offset[id(p)]
        if g.data_ptr() != self.grad.data_ptr() + off * self.grad.element_size():
            view = self.grad[off: off + p.numel()]
            view.copy_(g.reshape(-1))
            p.grad = view.view_as(p)

    def finalize_fresh_range(self, bucket):
        """``finalize_fresh`` restricted to one bucket's parameters."""
        for p in bucket.params:
            if getattr(p, "_rca_grad_fresh", False) and getattr(p, "_rca_flat_grad", False):
                off = self.param_offset[id(p)]
                self.grad[off: off + p.numel()].zero_()
                p._rca_grad_fresh = False

    def finalize_fresh(self):
        """Zero the regions of fused weights that received no gradient since zero_grad."""
        for p in self.fused:
            if p._rca_grad_fresh:
                off = self.param_offset[id(p)]
                self.grad[off: off + p.numel()].zero_()
                p._rca_grad_fresh = False

    def zero_grad(self):
        self.grad[self.zero_start:].zero_()
        for p in self.fused:
            p._rca_grad_fresh = True
        if self.grad_is_view:
            for p, off in zip(self.params, self.offsets):
                if p.grad is None or p.grad.data_ptr() != self.grad[off:].data_ptr():
                    p.grad = self.grad[off: off + p.numel()].view_as(p)

    @property
    def step_grad(self) -> torch.Tensor:
        """The gradient buffer an optimizer step should read."""
        return self.reduced_grad if self.reduced_grad is not None else self.grad

    def param_slices(self, name_filter: Optional[Callable[[str], bool]] = None):
        for n, p, off in zip(self.names, self.params, self.offsets):
            if name_filter is None or name_filter(n):
                yield n, p, off

    def __len__(self):
        return self.numel
