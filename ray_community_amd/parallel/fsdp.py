"""Sharded data parallelism (ZeRO stage 1/2) over RCCL: reduce-scatter gradients, shard the
optimizer, all-gather the updated weights.

Reference: ``python/ray/train/torch/train_loop_utils.py`` (``prepare_model(...,
parallel_strategy="fsdp")`` wraps torch FSDP). Here sharding is built on the framework's flat
buffers (``FlatParameters``) so every collective is ONE in-place RCCL call on a contiguous
bucket view:

  * buckets are padded to ``world * 64`` elements; rank ``r`` owns chunk ``r`` of every bucket;
  * backward: the moment a bucket's last gradient lands, an async in-place
    ``reduce_scatter_tensor`` (SUM) leaves the summed chunk in this rank's slice of the flat grad
    buffer (same bytes on the wire as half an all-reduce; overlapped with the rest of backward);
  * ``ShardedAdamW``: fp32 master weights and AdamW moments exist only for owned chunks
    (16 B/param / world instead of 16 B/param), the fused HIP AdamW kernel runs once per owned
    chunk (1/world of the elementwise work), the global grad norm for clipping is a scalar
    all-reduce of per-shard sums of squares (no host sync);
  * after the update, async in-place ``all_gather_into_tensor`` per bucket redistributes the bf16
    weights; a forward pre-hook on each module waits only for the buckets holding that module's
    parameters, so the gathers overlap the next forward pass (issued in the order forward needs
    them: the no-decay tail, then buckets from the end of the layout = the first layers).

On xGMI's point-to-point links reduce-scatter + all-gather move the same bytes as one ring
all-reduce, so the win is the optimizer pass (and HBM), not the wire.

W^T copies: the backward's input-gradient GEMMs read each fused linear weight transposed
(``fused_linear.weight_t``). Under DDP the replicated optimizer writes W^T in its update pass;
here a rank updates only its chunks and the full W arrives by all-gather, so W^T is produced by
one LDS-tiled transpose per weight on a side stream, launched by the forward pre-hook right
after the weight's gather is waited on. It overlaps the (compute-bound) forward GEMMs instead of
sitting in front of the backward's dgrad, which waits on its event only when it needs W^T.
``RCA_ZERO_WT=0`` turns it off (dgrad then transposes in line, as before).
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import ops
from .ddp import CommWaitTimer
from .flat import ALIGN, FlatParameters, register_grad_ready
from .optim import _use_split


class ShardedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, process_group=None, bucket_cap_mb: float = 256.0, broadcast_buffers=True,
                 reduce_dtype=None):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.flat = FlatParameters(module, bucket_cap_mb=bucket_cap_mb, bucket_align=ALIGN * self.world)
        # fp32 gradient reduction: see DistributedDataParallel(reduce_dtype=...)
        self.reduce_dtype = reduce_dtype or self.flat.grad.dtype
        self.comm_timer = CommWaitTimer()
        if self.world > 1 and self.reduce_dtype != self.flat.grad.dtype:
            self.flat.reduced_grad = torch.zeros(self.flat.numel, dtype=self.reduce_dtype, device=self.flat.device)
        self._sync = True
        self._rs: List[Optional[object]] = [None] * len(self.flat.buckets)
        self._ag: List[Optional[object]] = [None] * len(self.flat.buckets)
        self._pending = [len(b.params) for b in self.flat.buckets]
        self._hooks = []
        if self.world > 1:
            src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
            dist.broadcast(self.flat.data, src=src, group=process_group)
            if broadcast_buffers:
                for b in module.buffers():
                    dist.broadcast(b, src=src, group=process_group)
            self._hooks += register_grad_ready(self.flat.params, self._on_grad)
        # W^T copies of the fused linear weights, refreshed on a side stream after each gather
        self._wt_epoch = [0]  # bumped by every optimizer update / weight load (W changed)
        self._wt_stream = None
        self._module_wt: Dict[int, List[nn.Parameter]] = {}
        wt_ids = set()
        if os.environ.get("RCA_ZERO_WT", "1") != "0" and self.flat.data.is_cuda:
            for p in self.flat.fused:
                if p.dim() == 2 and p.shape[0] % 128 == 0 and p.shape[1] % 128 == 0:
                    p._rca_wt = torch.empty(p.shape[1], p.shape[0], dtype=p.dtype, device=p.device)
                    p._rca_wt_key = None
                    p._rca_wt_epoch = self._wt_epoch
                    p._rca_wt_ev = None
                    wt_ids.add(id(p))
        # forward pre-hooks: wait for the all-gathers of the buckets this module's own params live in
        self._module_buckets: Dict[int, List[int]] = {}
        for m in module.modules():
            own = [p for p in m.parameters(recurse=False) if id(p) in self.flat.param_bucket]
            bis = sorted({self.flat.param_bucket[id(p)] for p in own})
            wts = [p for p in own if id(p) in wt_ids]
            if wts:
                self._module_wt[id(m)] = wts
            if bis:
                self._module_buckets[id(m)] = bis
                self._hooks.append(m.register_forward_pre_hook(self._pre_forward))

    # ------------------------------------------------------------------ shards
    def shard_range(self, bi: int):
        """[start, end) of this rank's chunk of bucket ``bi`` in the flat buffers."""
        b = self.flat.buckets[bi]
        c = (b.end - b.start) // self.world
        s = b.start + self.rank * c
        return s, s + c

    # ------------------------------------------------------------------ backward
    def _on_grad(self, p):
        if not self._sync:
            return
        self.flat.adopt_grad(p)
        bi = self.flat.param_bucket[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._launch_rs(bi)

    def _launch_rs(self, bi):
        b = self.flat.buckets[bi]
        s, e = self.shard_range(bi)
        g = self.flat.grad
        if self.flat.reduced_grad is not None:
            g = self.flat.reduced_grad
            g[b.start: b.end].copy_(self.flat.grad[b.start: b.end])
        self._rs[bi] = dist.reduce_scatter_tensor(g[s:e], g[b.start: b.end], group=self.pg, async_op=True)

    def finish_gradient_sync(self):
        """Reduce-scatter buckets whose grads never arrived (unused params) and wait for all."""
        if self.world <= 1:
            return
        if any(w is None for w in self._rs):
            self.flat.finalize_fresh()
        for bi, w in enumerate(self._rs):
            if w is None:
                self._launch_rs(bi)
        with self.comm_timer.region():
            for bi, w in enumerate(self._rs):
                if w is not None:
                    w.wait()
                self._rs[bi] = None
        self._pending = [len(b.params) for b in self.flat.buckets]

    # ------------------------------------------------------------------ weights
    def gather_order(self):
        nb = len(self.flat.buckets)
        tail = [b.index for b in self.flat.buckets if b.start >= self.flat.decay_end]
        return tail + [bi for bi in range(nb - 1, -1, -1) if bi not in tail]

    def launch_all_gather(self, bi: int):
        if self.world <= 1:
            return
        b = self.flat.buckets[bi]
        s, e = self.shard_range(bi)
        self._ag[bi] = dist.all_gather_into_tensor(self.flat.data[b.start: b.end], self.flat.data[s:e],
                                                   group=self.pg, async_op=True)

    def wait_all_gathers(self, buckets=None):
        with self.comm_timer.region():
            for bi in (range(len(self._ag)) if buckets is None else buckets):
                w = self._ag[bi]
                if w is not None:
                    w.wait()
                    self._ag[bi] = None

    def _pre_forward(self, m, args):
        bis = self._module_buckets.get(id(m))
        if bis and any(self._ag[bi] is not None for bi in bis):
            self.wait_all_gathers(bis)
        wts = self._module_wt.get(id(m))
        if wts and torch.is_grad_enabled():
            self._refresh_wt(wts)

    def _refresh_wt(self, wts):
        """Transpose the stale W^T copies of ``wts`` on the side stream (after everything the
        current stream has queued, i.e. the gathers just waited on); the dgrad waits on the
        recorded event (``fused_linear.weight_t``)."""
        ep = self._wt_epoch[0]
        stale = [p for p in wts if p._rca_wt_key != (p._version, ep)]
        if not stale:
            return
        main = torch.cuda.current_stream(self.flat.device)
        if self._wt_stream is None:
            self._wt_stream = torch.cuda.Stream(self.flat.device)
        side = self._wt_stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for p in stale:
                ops.transpose(p.detach(), out=p._rca_wt)
                p._rca_wt_key = (p._version, ep)
            ev = torch.cuda.Event()
            ev.record(side)
        for p in stale:
            p._rca_wt_ev = ev

    def invalidate_wt(self):
        """The weights are about to change (optimizer update, load): every W^T copy is stale, and
        transposes still reading the old W (a dgrad that never ran) must finish first."""
        self._wt_epoch[0] += 1
        if self._wt_stream is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._wt_stream)

    # ------------------------------------------------------------------ module API
    def forward(self, *args, **kwargs):
        if self._sync:
            self._pending = [len(b.params) for b in self.flat.buckets]
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world if self.world > 1 else 1.0

    def zero_grad(self, set_to_none: bool = False):
        self.flat.zero_grad()

    def state_dict(self, *a, **k):
        self.wait_all_gathers()
        return self.module.state_dict(*a, **k)

    def load_state_dict(self, sd, strict=True):
        self.wait_all_gathers()
        self.invalidate_wt()
        return self.module.load_state_dict(sd, strict=strict)


class ShardedAdamW:
    """AdamW over this rank's chunks of a ``ShardedDataParallel`` model (fp32 master + moments
    for owned elements only); same update rule as ``FlatAdamW`` / ``torch.optim.AdamW``."""

    def __init__(self, sdp: ShardedDataParallel, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: Optional[float] = 1.0, lr_schedule=None,
                 master_format: str = "auto"):
        self.sdp = sdp
        flat = sdp.flat
        self.lr, (self.b1, self.b2), self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.lr_schedule = lr_schedule
        self.step_count = 0
        self.master_weights = flat.dtype != torch.float32
        self.chunks = []  # (bucket index, flat start, flat end, local offset, weight decay)
        lo = 0
        for b in flat.buckets:
            s, e = sdp.shard_range(b.index)
            self.chunks.append((b.index, s, e, lo, weight_decay if b.start < flat.decay_end else 0.0))
            lo += e - s
        self.local_numel = lo
        dev = flat.device
        # split master (optim.py): the owned chunks' bf16 weights hold the high halves, ``lo`` the
        # low 16 bits; needs 8-element-aligned chunks for the vector kernel
        aligned = all(s % 8 == 0 and o % 8 == 0 for _, s, _, o, _ in self.chunks)
        fmt = master_format if aligned or master_format == "fp32" else ("fp32" if master_format == "auto" else "unaligned")
        if fmt == "unaligned":
            raise ValueError("split master format needs 8-element-aligned shard chunks")
        self.split_master = _use_split(fmt, self.master_weights, flat.data)
        self.lo = torch.zeros(lo, dtype=torch.int16, device=dev) if self.split_master else None
        self._master = None
        if not self.split_master:
            self._master = torch.empty(lo, dtype=torch.float32, device=dev)
            for _, s, e, o, _ in self.chunks:
                self._master[o: o + e - s].copy_(flat.data[s:e])
        self.m = torch.zeros(lo, dtype=torch.float32, device=dev)
        self.v = torch.zeros(lo, dtype=torch.float32, device=dev)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._grad_scale = 1.0

    @property
    def param_groups(self):
        return [{"lr": self.lr, "weight_decay": self.wd}]

    def current_lr(self) -> float:
        return self.lr_schedule(self.step_count) if self.lr_schedule else self.lr

    def _hi_local(self) -> torch.Tensor:
        flat = self.sdp.flat
        return torch.cat([flat.data[s:e] for _, s, e, _, _ in self.chunks]) if self.chunks else flat.data[:0]

    @property
    def master(self) -> torch.Tensor:
        """fp32 master of the owned elements (split format: reconstructed, a fresh tensor)."""
        if self.split_master:
            return ops.reference.join_master(self._hi_local(), self.lo)
        return self._master

    @torch.no_grad()
    def step(self, grad_scale: Optional[float] = None):
        sdp, flat = self.sdp, self.sdp.flat
        grad_scale = sdp.grad_scale if grad_scale is None else grad_scale
        self._grad_scale = grad_scale
        self.step_count += 1
        t = self.step_count
        lr = self.current_lr()
        bc1, bc2 = 1.0 - self.b1 ** t, 1.0 - self.b2 ** t
        flat.finalize_fresh()
        sdp.invalidate_wt()
        g = flat.step_grad
        clip = self.max_grad_norm if self.max_grad_norm and self.max_grad_norm > 0 else 0.0
        if clip:
            ops.grad_sumsq([g[s:e] for _, s, e, _, _ in self.chunks], out=self._sumsq)
            if sdp.world > 1:
                dist.all_reduce(self._sumsq, group=sdp.pg)
        # update chunks in the order the next forward needs them, launching each bucket's gather
        order = {bi: k for k, bi in enumerate(sdp.gather_order())}
        for bi, s, e, o, wd in sorted(self.chunks, key=lambda c: order[c[0]]):
            n = e - s
            if n > 0:
                if g.is_cuda:
                    from ..ops._lib import check, lib, stream_ptr

                    if g.dtype not in (torch.bfloat16, torch.float32):
                        raise TypeError(f"unsupported grad dtype {g.dtype}")
                    gdt = 0 if g.dtype == torch.bfloat16 else 1
                    if self.split_master:
                        check(lib().rca_adamw_split(flat.data.data_ptr() + s * 2, self.lo.data_ptr() + o * 2,
                                                    g.data_ptr() + s * g.element_size(), gdt,
                                                    self.m.data_ptr() + o * 4, self.v.data_ptr() + o * 4, n, lr,
                                                    self.b1, self.b2, self.eps, wd, bc1, bc2, grad_scale,
                                                    self._sumsq.data_ptr() if clip else 0, float(clip),
                                                    stream_ptr(g.device)), "adamw_split")
                        sdp.launch_all_gather(bi)
                        continue
                    p16 = flat.data.data_ptr() + s * flat.data.element_size() if self.master_weights else 0
                    mp = self._master.data_ptr() + o * 4 if self.master_weights else 0
                    if not self.master_weights:  # fp32 model: update the flat data in place
                        mp = flat.data.data_ptr() + s * 4
                    check(lib().rca_adamw(mp, p16, g.data_ptr() + s * g.element_size(), gdt,
                                          self.m.data_ptr() + o * 4, self.v.data_ptr() + o * 4, n, lr, self.b1,
                                          self.b2, self.eps, wd, bc1, bc2, grad_scale,
                                          self._sumsq.data_ptr() if clip else 0, float(clip), stream_ptr(g.device)),
                          "adamw")
                else:
                    coef = 1.0
                    if clip:
                        nrm = math.sqrt(float(self._sumsq)) * abs(grad_scale)
                        coef = min(1.0, clip / (nrm + 1e-6))
                    if self.split_master:
                        master = ops.reference.join_master(flat.data[s:e], self.lo[o: o + n])
                    else:
                        master = self._master[o: o + n] if self.master_weights else flat.data[s:e]
                    ops.reference.adamw_ref(master, g[s:e], self.m[o: o + n], self.v[o: o + n], lr, self.b1, self.b2,
                                            self.eps, wd, t, grad_mul=grad_scale, clip=coef)
                    if self.split_master:
                        hi, lo_ = ops.reference.split_master(master)
                        flat.data[s:e].copy_(hi)
                        self.lo[o: o + n].copy_(lo_)
                    elif self.master_weights:
                        flat.data[s:e].copy_(master.to(flat.dtype))
            sdp.launch_all_gather(bi)

    def grad_norm(self) -> float:
        return math.sqrt(float(self._sumsq.item())) * abs(self._grad_scale)

    def zero_grad(self, set_to_none: bool = False):
        self.sdp.flat.zero_grad()

    def state_dict(self):
        """This rank's shard of the optimizer state (save one file per rank)."""
        return {"step": self.step_count, "m": self.m, "v": self.v, "master": self.master, "rank": self.sdp.rank,
                "world": self.sdp.world, "lr": self.lr, "betas": (self.b1, self.b2), "eps": self.eps, "wd": self.wd}

    def load_state_dict(self, sd):
        if sd.get("world", self.sdp.world) != self.sdp.world:
            raise ValueError("sharded optimizer state was saved with a different world size")
        self.step_count = sd["step"]
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.sdp.invalidate_wt()
        flat = self.sdp.flat
        master = sd["master"].to(flat.device)
        with torch.no_grad():
            if self.split_master:
                hi, lo = ops.reference.split_master(master)
                self.lo.copy_(lo)
            elif self._master is not None:
                self._master.copy_(master)
            for bi, s, e, o, _ in self.chunks:
                if self.split_master:
                    flat.data[s:e].copy_(hi[o: o + e - s])
                elif self.master_weights:
                    flat.data[s:e].copy_(master[o: o + e - s].to(flat.dtype))
                self.sdp.launch_all_gather(bi)
