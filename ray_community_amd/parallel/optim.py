"""Fused flat AdamW with fp32 master weights.

One HIP kernel launch per weight-decay group streams (fp32 master, bf16/f32 grad, m, v) ->
(master, m, v, bf16 model weights) at HBM rate. Gradient averaging (1/world from DDP) and
global-norm clipping (norm read from device memory) are folded into the same pass, so the
step needs no host synchronisation and no extra elementwise passes.
Works on any ``FlatParameters`` (CPU tensors use the PyTorch reference math).

Master format (``master_format``): "split" (the GPU bf16 default) keeps only the LOW 16 bits of
each fp32 master beside the bf16 model weight, which holds the high half rounded (the pair
reconstructs the master bit-exactly; ``ops.reference.split_master``): 26 instead of 28 B of HBM
traffic per parameter per step and 2 B/param less memory. "fp32" keeps a separate fp32 master.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from .. import ops
from ..ops._lib import check, lib, stream_ptr
from .flat import FlatParameters


class FlatAdamW:
    def __init__(self, flat: FlatParameters, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: Optional[float] = 1.0, master_weights: bool = True,
                 lr_schedule=None, master_format: str = "auto"):
        self.flat = flat
        self.lr = lr
        self.b1, self.b2 = betas
        self.eps = eps
        self.wd = weight_decay
        self.max_grad_norm = max_grad_norm
        self.lr_schedule = lr_schedule
        self.step_count = 0
        dev = flat.device
        self.master_weights = master_weights and flat.dtype != torch.float32
        self.split_master = _use_split(master_format, self.master_weights, flat.data)
        self.lo = torch.zeros(flat.numel, dtype=torch.int16, device=dev) if self.split_master else None
        self._master = None if self.split_master else (flat.data.float() if self.master_weights else flat.data)
        self.m = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        self.v = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self.last_grad_norm = None  # device tensor (sum of squares, pre-scale)
        self.track_grad_norm = False
        self._ov = None  # forward-overlap state (overlap_with_forward)
        # transposed bf16 weights W^T refreshed by the update itself (see _setup_transposed)
        self.transposed_weights = (self.split_master and flat.data.is_cuda
                                   and os.environ.get("RCA_ADAMW_WT", "1") != "0")
        self._wt_epoch = [0]  # bumped whenever the weights change outside the fused update
        self._wt_params = None
        self._segs = None

    # ------------------------------------------------------------------ forward overlap
    def overlap_with_forward(self, module: "torch.nn.Module", enabled: bool = True):
        """Run the update bucket by bucket on a side HIP stream, overlapped with the NEXT forward.

        AdamW is HBM-bound (28 B/param: ~37 ms for 8B params at ~6 TB/s) while the forward is
        MFMA-bound, so instead of a serial optimizer pass the update of each gradient bucket is
        issued on its own stream in the order the next forward consumes the weights (the no-decay
        tail holding the norm weights, then buckets from the END of the layout = the first
        layers) and a forward pre-hook on every module with parameters waits only for the
        buckets holding those parameters. A forward hook on the root waits for the whole update
        (and the gradient zeroing that follows it) before the loss is returned, so backward never
        races the optimizer. Same update rule and result as the serial step.
        """
        if self._ov is not None:
            for h in self._ov["hooks"]:
                h.remove()
            self._ov = None
        if not enabled or not self.flat.device.type == "cuda":
            return self
        flat = self.flat
        mod_buckets = {}
        hooks = []
        for m in module.modules():
            bis = sorted({flat.param_bucket[id(p)] for p in m.parameters(recurse=False) if id(p) in flat.param_bucket})
            if bis:
                mod_buckets[id(m)] = bis
                hooks.append(m.register_forward_pre_hook(self._ov_pre_forward))
        hooks.append(module.register_forward_hook(self._ov_post_forward))
        tail = [b.index for b in flat.buckets if b.start >= flat.decay_end]
        order = tail + [b.index for b in reversed(flat.buckets) if b.index not in tail]
        self._ov = {"stream": torch.cuda.Stream(device=flat.device), "mod_buckets": mod_buckets, "hooks": hooks,
                    "order": order, "events": [None] * len(flat.buckets), "done": None,
                    "evs": [torch.cuda.Event() for _ in flat.buckets], "done_ev": torch.cuda.Event()}
        return self

    def _ov_pre_forward(self, m, args):
        ov = self._ov
        if ov is None or ov["done"] is None:  # no update in flight
            return
        cur = torch.cuda.current_stream(self.flat.device)
        for bi in ov["mod_buckets"].get(id(m), ()):
            ev = ov["events"][bi]
            if ev is not None:
                cur.wait_event(ev)
                ov["events"][bi] = None

    def _ov_post_forward(self, m, args, out):
        self.wait_pending_update()

    def wait_pending_update(self):
        """Make the current stream wait for an in-flight overlapped update (no host sync)."""
        ov = self._ov
        if ov is not None and ov["done"] is not None:
            torch.cuda.current_stream(self.flat.device).wait_event(ov["done"])
            ov["done"] = None
            ov["events"] = [None] * len(self.flat.buckets)

    @property
    def param_groups(self):  # minimal torch.optim compatibility for LR schedulers / logging
        return [{"lr": self.lr, "weight_decay": self.wd}]

    def current_lr(self) -> float:
        return self.lr_schedule(self.step_count) if self.lr_schedule else self.lr

    @property
    def master(self) -> torch.Tensor:
        """The fp32 master weights (with the split format: reconstructed, a fresh tensor)."""
        if self.split_master:
            return ops.reference.join_master(self.flat.data, self.lo)
        return self._master

    def _setup_transposed(self):
        """W^T buffers for the fused-wgrad linear weights + the segment table of the update.

        Each ``FusedWgradLinear`` weight W [R, C] (R, C multiples of 128) gets a persistent bf16
        ``W^T`` [C, R] (``p._rca_wt``) that the segmented update kernel rewrites from the new
        weights in the same pass (one extra 2-B write per parameter); the backward dgrad reads it
        instead of transposing W (``parallel/fused_linear.py::weight_t``). Validity is keyed on
        (p._version, epoch): in-place edits of a weight or a bumped epoch (load_state_dict,
        sync_master, an update that did not refresh W^T) make the backward fall back to a
        transpose pass into the same buffer."""
        flat = self.flat
        mats = []
        for p in flat.fused:
            if p.dim() == 2 and p.shape[0] % 128 == 0 and p.shape[1] % 128 == 0:
                p._rca_wt = torch.empty(p.shape[1], p.shape[0], dtype=p.dtype, device=p.device)
                p._rca_wt_key = None
                p._rca_wt_epoch = self._wt_epoch
                mats.append((flat.param_offset[id(p)], p))
        mats.sort(key=lambda t: t[0])
        rows, blk = [], 0

        def add_range(s, e):
            nonlocal blk
            # split at the weight-decay boundary: a 1-D segment carries one decay flag
            for a, b in ((s, min(e, flat.decay_end)), (max(s, flat.decay_end), e)):
                if b > a:
                    rows.append([a, b - a, blk, 0, 0, 0, int(a < flat.decay_end), 0])
                    blk += (b - a + 4095) // 4096

        cur = 0
        for off, p in mats:
            add_range(cur, off)
            R, C = p.shape
            rows.append([off, p.numel(), blk, p._rca_wt.data_ptr(), R, C, int(off < flat.decay_end), 0])
            blk += (R // 128) * (C // 128)
            cur = off + p.numel()
        add_range(cur, flat.numel)
        self._wt_params = [p for _, p in mats]
        self._segs = torch.tensor(rows, dtype=torch.int64, device=flat.device)
        self._seg_blocks = blk

    def sync_master(self):
        """Re-read model weights into the fp32 master copy (after load_state_dict)."""
        self._wt_epoch[0] += 1
        if self.split_master:
            self.lo.zero_()
        elif self.master_weights:
            self._master.copy_(self.flat.data.float())

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        self.step_count += 1
        t = self.step_count
        lr = self.current_lr()
        bc1 = 1.0 - self.b1 ** t
        bc2 = 1.0 - self.b2 ** t
        flat = self.flat
        flat.finalize_fresh()
        g = flat.step_grad
        clip = self.max_grad_norm if self.max_grad_norm and self.max_grad_norm > 0 else 0.0
        pre, flat.precomputed_sumsq = flat.precomputed_sumsq, None
        if clip or self.track_grad_norm:
            if pre is not None and pre.device == self._sumsq.device:
                self._sumsq.copy_(pre)  # taken during backward (DistributedDataParallel precompute_grad_norm)
            else:
                ops.grad_sumsq([g], out=self._sumsq)
            self.last_grad_norm = self._sumsq  # sqrt taken lazily by grad_norm()
        self._grad_scale = grad_scale
        segs = [(0, flat.decay_end, self.wd), (flat.decay_end, flat.numel, 0.0)]
        self._wt_epoch[0] += 1  # every update changes W: W^T is stale unless refreshed below
        if g.is_cuda:
            if g.dtype not in (torch.bfloat16, torch.float32):
                raise TypeError(f"unsupported grad dtype {g.dtype}")
            ov = self._ov
            if ov is None and self.transposed_weights:
                if self._segs is None:
                    self._setup_transposed()
                check(lib().rca_adamw_split_seg(
                    flat.data.data_ptr(), self.lo.data_ptr(), g.data_ptr(), 0 if g.dtype == torch.bfloat16 else 1,
                    self.m.data_ptr(), self.v.data_ptr(), self._segs.data_ptr(), self._segs.shape[0],
                    self._seg_blocks, lr, self.b1, self.b2, self.eps, self.wd, bc1, bc2, grad_scale,
                    self._sumsq.data_ptr() if clip else 0, float(clip), stream_ptr(g.device)), "adamw_split_seg")
                ep = self._wt_epoch[0]
                for p in self._wt_params:
                    p._rca_wt_key = (p._version, ep)
                return
            if ov is None:
                for s, e, wd in segs:
                    self._launch(g, s, e, wd, lr, bc1, bc2, grad_scale, clip, stream_ptr(g.device))
                return
            # overlapped: the side stream starts once the gradients (and their norm) are final
            self.wait_pending_update()
            main = torch.cuda.current_stream(g.device)
            side = ov["stream"]
            side.wait_stream(main)
            sp = side.cuda_stream
            for bi in ov["order"]:
                b = flat.buckets[bi]
                wd = self.wd if b.start < flat.decay_end else 0.0
                self._launch(g, b.start, min(b.end, flat.numel), wd, lr, bc1, bc2, grad_scale, clip, sp)
                ev = ov["evs"][bi]
                ev.record(side)
                ov["events"][bi] = ev
            ov["done_ev"].record(side)
            ov["done"] = ov["done_ev"]
            ov["pending_zero"] = True
        else:
            coef = 1.0
            if clip:
                nrm = math.sqrt(float(self._sumsq)) * abs(grad_scale)
                coef = min(1.0, clip / (nrm + 1e-6))
            master = self.master
            for s, e, wd in segs:
                if e <= s:
                    continue
                ops.reference.adamw_ref(master[s:e], g[s:e], self.m[s:e], self.v[s:e], lr, self.b1, self.b2,
                                        self.eps, wd, t, grad_mul=grad_scale, clip=coef)
            if self.split_master:
                hi, lo = ops.reference.split_master(master)
                flat.data.copy_(hi)
                self.lo.copy_(lo)
            elif self.master_weights:
                flat.data.copy_(master.to(flat.dtype))

    def _launch(self, g, s, e, wd, lr, bc1, bc2, grad_scale, clip, st):
        n = e - s
        if n <= 0:
            return
        flat = self.flat
        gdt = 0 if g.dtype == torch.bfloat16 else 1
        if self.split_master:
            check(lib().rca_adamw_split(flat.data.data_ptr() + s * 2, self.lo.data_ptr() + s * 2,
                                        g.data_ptr() + s * g.element_size(), gdt, self.m.data_ptr() + s * 4,
                                        self.v.data_ptr() + s * 4, n, lr, self.b1, self.b2, self.eps, wd, bc1, bc2,
                                        grad_scale, self._sumsq.data_ptr() if clip else 0, float(clip), st),
                  "adamw_split")
            return
        p16 = flat.data.data_ptr() + s * flat.data.element_size() if self.master_weights else 0
        check(lib().rca_adamw(self._master.data_ptr() + s * self._master.element_size(), p16,
                              g.data_ptr() + s * g.element_size(), gdt, self.m.data_ptr() + s * 4,
                              self.v.data_ptr() + s * 4, n, lr, self.b1, self.b2, self.eps, wd, bc1, bc2, grad_scale,
                              self._sumsq.data_ptr() if clip else 0, float(clip), st), "adamw")

    def grad_norm(self) -> float:
        """Global grad norm of the last step (host sync — call only for logging)."""
        if self.last_grad_norm is None:
            return 0.0
        return math.sqrt(float(self.last_grad_norm.item())) * abs(getattr(self, "_grad_scale", 1.0))

    def zero_grad(self, set_to_none: bool = False):
        ov = self._ov
        if ov is not None and ov.get("pending_zero") and ov["done"] is not None:
            # the update is still reading the gradients on the side stream: zero behind it there
            ov["pending_zero"] = False
            side = ov["stream"]
            with torch.cuda.stream(side):
                self.flat.zero_grad()
            ov["done"].record(side)
            return
        self.flat.zero_grad()

    def state_dict(self):
        self.wait_pending_update()
        return {"step": self.step_count, "m": self.m, "v": self.v, "master": self.master if self.master_weights else None,
                "lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps, "wd": self.wd}

    def load_state_dict(self, sd):
        self._wt_epoch[0] += 1
        self.step_count = sd["step"]
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        if self.master_weights and sd.get("master") is not None:
            if self.split_master:
                hi, lo = ops.reference.split_master(sd["master"].to(self.flat.device))
                self.flat.data.copy_(hi)
                self.lo.copy_(lo)
            else:
                self._master.copy_(sd["master"])
                self.flat.data.copy_(self._master.to(self.flat.dtype))


def _use_split(master_format: str, master_weights: bool, data: torch.Tensor) -> bool:
    """"auto": the split master on GPU bf16 models; "split" / "fp32" force the choice."""
    if master_format not in ("auto", "split", "fp32"):
        raise ValueError(f"master_format must be auto|split|fp32, got {master_format!r}")
    ok = master_weights and data.dtype == torch.bfloat16
    if master_format == "split" and not ok:
        raise ValueError("the split master format needs bf16 model weights with master_weights=True")
    if master_format == "auto":
        return ok and data.is_cuda and os.environ.get("RCA_ADAMW_SPLIT", "1") != "0"
    return master_format == "split"


class FlatSGD:
    """SGD with (Nesterov) momentum and weight decay over a ``FlatParameters`` buffer.

    The whole model is one contiguous tensor, so the update is three streaming passes over the
    flat buffers regardless of how many layers the model has (ResNet-50: 161 tensors -> 1).
    ``grad_scale`` (1/world from DDP) is folded into the momentum update.
    Reference semantics: ``torch.optim.SGD`` (momentum buffer initialised to the first gradient).
    """

    def __init__(self, flat: FlatParameters, lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 0.0,
                 nesterov: bool = False, lr_schedule=None):
        self.flat = flat
        self.lr = lr
        self.momentum = momentum
        self.wd = weight_decay
        self.nesterov = nesterov
        self.lr_schedule = lr_schedule
        self.step_count = 0
        self.buf = torch.zeros(flat.numel, dtype=flat.grad.dtype, device=flat.device) if momentum else None

    @property
    def param_groups(self):
        return [{"lr": self.lr, "momentum": self.momentum, "weight_decay": self.wd}]

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0):
        self.step_count += 1
        lr = self.lr_schedule(self.step_count) if self.lr_schedule else self.lr
        self.flat.finalize_fresh()
        p, g = self.flat.data, self.flat.step_grad
        if grad_scale != 1.0:
            g.mul_(grad_scale)
        if self.wd:
            # decay only the matrices/conv kernels (the flat layout puts them first)
            g[: self.flat.decay_end].add_(p[: self.flat.decay_end], alpha=self.wd)
        d = g
        if self.buf is not None:
            if self.step_count == 1:
                self.buf.copy_(g)
            else:
                self.buf.mul_(self.momentum).add_(g)
            d = g.add(self.buf, alpha=self.momentum) if self.nesterov else self.buf
        p.add_(d.to(p.dtype), alpha=-lr)

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def state_dict(self):
        return {"step": self.step_count, "buf": self.buf, "lr": self.lr, "momentum": self.momentum, "wd": self.wd}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        if self.buf is not None and sd.get("buf") is not None:
            self.buf.copy_(sd["buf"])
