"""Fully sharded data parallelism (ZeRO stage 3): parameters, gradients and optimizer state are
all sharded over the data-parallel group; each unit's full bf16 weights exist only while that
unit runs.

Reference: ``python/ray/train/torch/train_loop_utils.py:29-31,175-179`` (``prepare_model(...,
parallel_strategy="fsdp")`` wraps torch FSDP). Design here, for 8 x 288 GB MI355X over xGMI:

  * **units**: one per transformer block (``module.layers[i]`` by default) plus a root unit with
    everything else (embedding, final norm, lm_head). Every unit is ONE flat buffer (decayed
    matrices first, no-decay vectors last, 64-element aligned views) padded to ``world * 64``;
    rank ``r`` permanently holds chunk ``r`` in a single contiguous local buffer, so the whole
    optimizer step is a handful of fused HIP AdamW launches over local memory.
  * **gather**: the unit's full buffer is re-materialised by growing its storage and issuing one
    in-place ``all_gather_into_tensor``; the module parameters are permanent views of that
    buffer, so tensors autograd saved during forward see the re-gathered data in backward.
    Freeing is ``untyped_storage().resize_(0)`` (stream-ordered in the caching allocator).
  * **forward**: a pre-hook on every module owning parameters gathers its unit (waits only on
    that unit's collective) and prefetches the next unit in the recorded forward order; the
    previous block unit is freed as soon as the next one starts (``reshard_after_forward``);
    the root unit stays resident (it is used at both ends of the step).
  * **backward**: the first gradient reaching any output of a unit's modules (a tensor hook
    installed by a forward hook) re-gathers that unit, materialises its full gradient buffer
    with ``param.grad`` views into it (the fused-wgrad linears write dW there directly) and
    prefetches the previous unit; when the unit's last gradient lands, one async in-place
    ``reduce_scatter_tensor`` (SUM) leaves the rank's chunk in the local gradient shard, and the
    unit's full weights are freed. At most two full gradient buffers are in flight.
  * **world == 1** degenerates to unsharded training with zero copies (the full buffers ARE the
    local shards).

Memory per GPU ~= 16 B/param / world (bf16 weights + grads, fp32 master + m + v) + two gathered
units + activations: see ``estimate_memory_gb`` (Llama-3-70B on 8 GPUs fits in 288 GB).
"""
from __future__ import annotations

import contextlib
import math
from typing import Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import ops
from .flat import ALIGN, _round_up, default_no_decay, register_grad_ready

_FREE, _GATHERING, _READY = 0, 1, 2


class _Unit:
    def __init__(self, index: int, name: str, named_params, world: int, rank: int):
        self.index, self.name = index, name
        decay = [(n, p) for n, p in named_params if not default_no_decay(n, p)]
        nodecay = [(n, p) for n, p in named_params if default_no_decay(n, p)]
        self.names = [n for n, _ in decay + nodecay]
        self.params = [p for _, p in decay + nodecay]
        self.offsets: List[int] = []
        o = 0
        for i, p in enumerate(self.params):
            if i == len(decay):
                o = _round_up(o)
            self.offsets.append(o)
            o += _round_up(p.numel())
        self.decay_end = self.offsets[len(decay)] if nodecay else o
        self.numel = max(_round_up(o, ALIGN * world), ALIGN * world)
        self.shard = self.numel // world
        self.rank = rank
        self.full: Optional[torch.Tensor] = None       # [numel] model dtype, storage resized
        self.full_grad: Optional[torch.Tensor] = None  # [numel] model dtype, storage resized
        self.local: Optional[torch.Tensor] = None      # [shard] view of the rank's weight shard
        self.local_grad: Optional[torch.Tensor] = None  # [shard] view of the rank's grad shard
        self.local_off = 0                             # offset of this unit's shard in the local buffers
        self.state = _FREE
        self.stale = False       # local shard updated since the full buffer was gathered
        self.work = None         # in-flight all-gather
        self.bwd_ready = False   # full grad buffer materialised for this backward
        self.bwd_done = False    # reduce-scatter launched in this backward
        self.grad_fresh = True   # local grad shard holds nothing since zero_grad
        self.pending = len(self.params)

    @property
    def shard_range(self):
        return self.rank * self.shard, (self.rank + 1) * self.shard


def _storage_resize(t: torch.Tensor, nbytes: int):
    st = t.untyped_storage()
    if st.nbytes() != nbytes:
        st.resize_(nbytes)


class FullyShardedDataParallel(nn.Module):
    """ZeRO-3 wrapper. Pair it with ``FullyShardedAdamW``; call ``finish_gradient_sync()`` after
    ``backward()`` (as with the framework's DDP)."""

    def __init__(self, module: nn.Module, process_group=None, unit_modules: Optional[List[nn.Module]] = None,
                 device=None, reduce_dtype=None, reshard_after_forward: bool = True, prefetch: bool = True,
                 sync_module_states: bool = True):
        super().__init__()
        self.module = module
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.reshard_after_forward = reshard_after_forward
        self.prefetch = prefetch
        params0 = [p for p in module.parameters() if p.requires_grad]
        if not params0:
            raise ValueError("module has no trainable parameters")
        self.device = torch.device(device) if device is not None else params0[0].device
        self.dtype = params0[0].dtype
        self.reduce_dtype = reduce_dtype or self.dtype
        from .ddp import CommWaitTimer

        self.comm_timer = CommWaitTimer()
        if unit_modules is None:
            layers = getattr(module, "layers", None)
            unit_modules = list(layers) if isinstance(layers, nn.ModuleList) else []
        # ---- assign parameters to units (root = everything not inside a unit module)
        owner: Dict[int, int] = {}
        named_by_unit: List[list] = [[] for _ in range(len(unit_modules) + 1)]
        seen = set()
        for ui, um in enumerate(unit_modules):
            for n, p in um.named_parameters():
                if p.requires_grad and id(p) not in seen:
                    seen.add(id(p))
                    owner[id(p)] = ui + 1
                    named_by_unit[ui + 1].append((n, p))
        for n, p in module.named_parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                owner[id(p)] = 0
                named_by_unit[0].append((n, p))
        self.units: List[_Unit] = []
        names = ["root"] + [f"unit{i}" for i in range(len(unit_modules))]
        for i, named in enumerate(named_by_unit):
            if named:
                self.units.append(_Unit(len(self.units), names[i], named, self.world, self.rank))
        self.root = self.units[0] if owner and named_by_unit[0] else None
        self.param_unit: Dict[int, _Unit] = {}
        for u in self.units:
            for p in u.params:
                self.param_unit[id(p)] = u
        # ---- local shard buffers (weights in model dtype, gradients in the reduce dtype)
        lo = 0
        for u in self.units:
            u.local_off = lo
            lo += u.shard
        self.local_numel = lo
        self.local_data = torch.zeros(lo, dtype=self.dtype, device=self.device)
        self.local_grad = torch.zeros(lo, dtype=self.reduce_dtype if self.world > 1 else self.dtype,
                                      device=self.device)
        src = dist.get_global_rank(process_group, 0) if (process_group is not None and self.world > 1) else 0
        for u in self.units:
            u.local = self.local_data[u.local_off: u.local_off + u.shard]
            u.local_grad = self.local_grad[u.local_off: u.local_off + u.shard]
            self._init_unit(u, sync_module_states, src)
        for b in module.buffers():
            if b.device != self.device:
                b.data = b.data.to(self.device)
            if self.world > 1 and sync_module_states:
                dist.broadcast(b, src=src, group=process_group)
        # ---- hooks
        self._hooks = []
        self._hooks += register_grad_ready([p for u in self.units for p in u.params], self._on_grad)
        self._module_unit: Dict[int, _Unit] = {}
        for m in module.modules():
            own = [p for p in m.parameters(recurse=False) if id(p) in self.param_unit]
            if not own:
                continue
            us = {self.param_unit[id(p)].index for p in own}
            if len(us) != 1:
                raise ValueError(f"module {type(m).__name__} owns parameters of several units")
            self._module_unit[id(m)] = self.units[us.pop()]
            self._hooks.append(m.register_forward_pre_hook(self._pre_forward))
            self._hooks.append(m.register_forward_hook(self._post_forward))
        self._fwd_order: List[int] = []
        self._recording = True
        self._current: Optional[_Unit] = None
        self._rs_inflight: List[tuple] = []
        self._sync = True

    # ------------------------------------------------------------------ setup
    @torch.no_grad()
    def _init_unit(self, u: _Unit, sync: bool, src: int):
        full = torch.zeros(u.numel, dtype=self.dtype, device=self.device)
        for p, off in zip(u.params, u.offsets):
            full[off: off + p.numel()].copy_(p.data.reshape(-1))
        if self.world > 1 and sync:
            dist.broadcast(full, src=src, group=self.pg)
        s, e = u.shard_range
        u.local.copy_(full[s:e])
        if self.world == 1:
            # unsharded: the full buffers ARE the local shards (no gathers, no copies)
            u.full = u.local
            u.full_grad = u.local_grad
            u.state = _READY
        else:
            u.full = full
            u.full_grad = torch.empty(u.numel, dtype=self.dtype, device=self.device)
            _storage_resize(u.full_grad, 0)
        for p, off in zip(u.params, u.offsets):
            p.data = u.full[off: off + p.numel()].view(p.shape)
            p.grad = None
            if getattr(p, "_rca_fused_wgrad", False) and self.world == 1:
                p._rca_flat_grad = True
        if self.world > 1:
            for p in u.params:
                if getattr(p, "_rca_fused_wgrad", False):
                    p._rca_flat_grad = True
            u.state = _READY
            if u is not self.root or self.root is None:
                self._free(u)

    # ------------------------------------------------------------------ gather / free
    def _gather(self, u: _Unit, wait: bool):
        if self.world == 1:
            return
        if u.state == _READY and u.stale:
            u.state = _FREE  # storage still allocated: just refill it
        if u.state == _FREE:
            _storage_resize(u.full, u.numel * u.full.element_size())
            # ``.data``: its own version counter, so parameters autograd saved stay valid
            u.work = dist.all_gather_into_tensor(u.full.data, u.local.data, group=self.pg, async_op=True)
            u.state = _GATHERING
            u.stale = False
        if wait and u.state == _GATHERING:
            with self.comm_timer.region():
                u.work.wait()
            u.work = None
            u.state = _READY

    def _free(self, u: _Unit):
        if self.world == 1 or u.state == _FREE:
            return
        if u.state == _GATHERING:
            u.work.wait()
            u.work = None
        _storage_resize(u.full, 0)
        u.state = _FREE

    def _next_in_order(self, u: _Unit, step: int) -> Optional[_Unit]:
        if u.index not in self._fwd_order:
            return None
        k = self._fwd_order.index(u.index) + step
        while 0 <= k < len(self._fwd_order):
            nxt = self.units[self._fwd_order[k]]
            if nxt is not self.root:
                return nxt
            k += step
        return None

    # ------------------------------------------------------------------ forward hooks
    def _pre_forward(self, m, args):
        u = self._module_unit[id(m)]
        if self._recording and u.index not in self._fwd_order:
            self._fwd_order.append(u.index)
        if u is not self._current:
            prev = self._current
            self._current = u
            self._gather(u, wait=True)
            if self.prefetch and not self._recording:
                nxt = self._next_in_order(u, +1)
                if nxt is not None:
                    self._gather(nxt, wait=False)
            # the previous block is finished once another block starts (keep it when the root
            # takes over at the end of forward: backward needs the last block first)
            if (prev is not None and prev is not self.root and u is not self.root and self.reshard_after_forward
                    and prev.index in self._fwd_order):
                self._free(prev)
        else:
            self._gather(u, wait=True)

    def _post_forward(self, m, args, out):
        if not torch.is_grad_enabled():
            return
        u = self._module_unit[id(m)]
        if u is self.root:
            return  # root grads are prepared before the forward starts
        ts = out if isinstance(out, (tuple, list)) else (out,)
        for t in ts:
            if isinstance(t, torch.Tensor) and t.requires_grad:
                t.register_hook(lambda g, u=u: self._pre_backward(u))

    # ------------------------------------------------------------------ backward
    def _prepare_grads(self, u: _Unit):
        if u.bwd_ready:
            return
        if self.world > 1:
            _storage_resize(u.full_grad, u.numel * u.full_grad.element_size())
        fresh = self.world > 1 or u.grad_fresh  # full grad buffer starts empty
        for p, off in zip(u.params, u.offsets):
            p.grad = u.full_grad[off: off + p.numel()].view(p.shape)
            if getattr(p, "_rca_fused_wgrad", False) and p.grad.dtype == p.dtype:
                p._rca_flat_grad = True
                p._rca_grad_fresh = fresh
        if fresh:
            # everything except fused-wgrad weights (which overwrite their region) starts at zero
            self._zero_unfused(u)
        u.bwd_ready = True

    def _zero_unfused(self, u: _Unit):
        """Zero the full gradient buffer except the regions fused-wgrad GEMMs will overwrite."""
        runs = []
        o = 0
        for p, off in zip(u.params, u.offsets):
            if getattr(p, "_rca_flat_grad", False) and getattr(p, "_rca_grad_fresh", False):
                if off > o:
                    runs.append((o, off))
                o = off + p.numel()
        if u.numel > o:
            runs.append((o, u.numel))
        for s, e in runs:
            u.full_grad[s:e].zero_()

    def _pre_backward(self, u: _Unit):
        if not self._sync or u.bwd_done or u.bwd_ready:
            return
        self._gather(u, wait=True)
        self._prepare_grads(u)
        if self.prefetch:
            prv = self._next_in_order(u, -1)
            if prv is not None and not prv.bwd_done:
                self._gather(prv, wait=False)

    def _on_grad(self, p):
        if not self._sync:
            return
        u = self.param_unit[id(p)]
        u.pending -= 1
        if u.pending == 0:
            self._reduce(u)

    def _finalize_fused(self, u: _Unit):
        for p, off in zip(u.params, u.offsets):
            if getattr(p, "_rca_flat_grad", False) and getattr(p, "_rca_grad_fresh", False):
                u.full_grad[off: off + p.numel()].zero_()
                p._rca_grad_fresh = False

    def _reduce(self, u: _Unit):
        if u.bwd_done:
            return
        if not u.bwd_ready:  # no gradient reached this unit (all of its params unused)
            u.bwd_done = True
            return
        self._finalize_fused(u)
        u.bwd_done = True
        if self.world == 1:
            u.grad_fresh = False
            return
        src = u.full_grad
        if self.reduce_dtype != src.dtype:
            src = src.to(self.reduce_dtype)
        if u.grad_fresh:
            out, tmp = u.local_grad, None
        else:
            tmp = torch.empty_like(u.local_grad)
            out = tmp
        work = dist.reduce_scatter_tensor(out, src, group=self.pg, async_op=True)
        u.grad_fresh = False
        for p in u.params:
            p.grad = None
        self._rs_inflight.append((u, work, src, tmp))
        if u is not self.root:
            self._free(u)
        while len(self._rs_inflight) > 2:
            self._retire(self._rs_inflight.pop(0))

    def _retire(self, item):
        u, work, src, tmp = item
        with self.comm_timer.region():
            work.wait()
        if tmp is not None:
            u.local_grad.add_(tmp)
        _storage_resize(u.full_grad, 0)

    def finish_gradient_sync(self):
        """Reduce-scatter units whose gradients never all arrived and wait for every collective."""
        for u in self.units:
            if u.bwd_ready and not u.bwd_done:
                self._reduce(u)
        while self._rs_inflight:
            self._retire(self._rs_inflight.pop(0))
        for u in self.units:
            if u.grad_fresh:  # never reduced since zero_grad: its shard holds no gradient
                u.local_grad.zero_()
                u.grad_fresh = False
            u.pending = len(u.params)
            u.bwd_ready = u.bwd_done = False
            if self.world > 1 and u is not self.root:
                self._free(u)
        self._current = None

    # ------------------------------------------------------------------ module API
    def forward(self, *args, **kwargs):
        self._current = None
        if self._fwd_order:
            self._recording = False
        for u in self.units:
            u.pending = len(u.params)
            u.bwd_ready = u.bwd_done = False
        if self.root is not None:
            self._gather(self.root, wait=True)
            if torch.is_grad_enabled() and self._sync:
                self._prepare_grads(self.root)
        if self.prefetch and not self._recording:
            first = next((self.units[i] for i in self._fwd_order if self.units[i] is not self.root), None)
            if first is not None:
                self._gather(first, wait=False)
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        """ZeRO-3 keeps no full gradients between micro-batches: every micro-batch reduce-scatters
        and accumulates into the local shard, so this context is a no-op kept for API parity."""
        yield

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world if self.world > 1 else 1.0

    def zero_grad(self, set_to_none: bool = False):
        # lazy: a fresh unit's first reduce-scatter (world > 1) or its fused-wgrad GEMMs plus the
        # zeroing of the other regions in _prepare_grads (world == 1) overwrite its shard, and
        # finish_gradient_sync zeroes shards that received nothing
        for u in self.units:
            u.grad_fresh = True

    def mark_stale(self):
        """Called by the optimizer after the local shards changed."""
        for u in self.units:
            if self.world > 1:
                u.stale = True
        if self.root is not None and self.world > 1:
            self._gather(self.root, wait=False)

    @contextlib.contextmanager
    def summon_full_params(self):
        """All units gathered (full model views) inside the context."""
        for u in self.units:
            self._gather(u, wait=True)
        try:
            yield self.module
        finally:
            for u in self.units:
                if u is not self.root:
                    self._free(u)

    def state_dict(self, *a, **k):
        """Full (unsharded) state dict, gathered unit by unit onto the host."""
        out = {}
        id_name = {}
        for n, p in self.module.named_parameters():
            id_name.setdefault(id(p), n)
        for u in self.units:
            self._gather(u, wait=True)
            for p in u.params:
                out[id_name[id(p)]] = p.detach().to("cpu", copy=True)
            if u is not self.root:
                self._free(u)
        for n, b in self.module.named_buffers():
            out[n] = b.detach().to("cpu", copy=True)
        return out

    @torch.no_grad()
    def load_state_dict(self, sd, strict=True):
        id_name = {}
        for n, p in self.module.named_parameters():
            id_name.setdefault(id(p), n)
        missing = []
        for u in self.units:
            full = torch.zeros(u.numel, dtype=self.dtype, device=self.device)
            for p, off in zip(u.params, u.offsets):
                name = id_name[id(p)]
                if name not in sd:
                    missing.append(name)
                    continue
                full[off: off + p.numel()].copy_(sd[name].reshape(-1))
            s, e = u.shard_range
            u.local.copy_(full[s:e])
            u.stale = self.world > 1
        for n, b in self.module.named_buffers():
            if n in sd:
                b.copy_(sd[n])
        if strict and missing:
            raise KeyError(f"missing keys in state dict: {missing}")
        if self.root is not None and self.world > 1:
            self._gather(self.root, wait=True)


class FullyShardedAdamW:
    """AdamW over the local shards of a ``FullyShardedDataParallel`` model: fp32 master weights
    and moments for this rank's chunks only; one fused HIP launch per contiguous weight-decay
    segment of the local buffer; global-norm clipping via a scalar all-reduce (no host sync).
    Same update rule as ``FlatAdamW`` / ``torch.optim.AdamW``."""

    def __init__(self, fsdp: FullyShardedDataParallel, lr: float = 3e-4, betas=(0.9, 0.95), eps: float = 1e-8,
                 weight_decay: float = 0.1, max_grad_norm: Optional[float] = 1.0, lr_schedule=None):
        self.fsdp = fsdp
        self.lr, (self.b1, self.b2), self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.lr_schedule = lr_schedule
        self.step_count = 0
        self.master_weights = fsdp.dtype != torch.float32
        dev = fsdp.device
        self.master = fsdp.local_data.float() if self.master_weights else fsdp.local_data
        self.m = torch.zeros(fsdp.local_numel, dtype=torch.float32, device=dev)
        self.v = torch.zeros(fsdp.local_numel, dtype=torch.float32, device=dev)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._grad_scale = 1.0
        # local segments (start, end, weight decay), adjacent equal-decay runs merged
        segs = []
        for u in fsdp.units:
            s, e = u.shard_range
            cut = min(max(u.decay_end, s), e)
            for a, b, wd in ((s, cut, weight_decay), (cut, e, 0.0)):
                if b > a:
                    ls, le = u.local_off + a - s, u.local_off + b - s
                    if segs and segs[-1][1] == ls and segs[-1][2] == wd:
                        segs[-1][1] = le
                    else:
                        segs.append([ls, le, wd])
        self.segments = [tuple(x) for x in segs]

    @property
    def param_groups(self):
        return [{"lr": self.lr, "weight_decay": self.wd}]

    def current_lr(self) -> float:
        return self.lr_schedule(self.step_count) if self.lr_schedule else self.lr

    def sync_master(self):
        if self.master_weights:
            self.master.copy_(self.fsdp.local_data.float())

    @torch.no_grad()
    def step(self, grad_scale: Optional[float] = None):
        f = self.fsdp
        grad_scale = f.grad_scale if grad_scale is None else grad_scale
        self._grad_scale = grad_scale
        self.step_count += 1
        t = self.step_count
        lr = self.current_lr()
        bc1, bc2 = 1.0 - self.b1 ** t, 1.0 - self.b2 ** t
        g = f.local_grad
        clip = self.max_grad_norm if self.max_grad_norm and self.max_grad_norm > 0 else 0.0
        if clip:
            ops.grad_sumsq([g], out=self._sumsq)
            if f.world > 1:
                dist.all_reduce(self._sumsq, group=f.pg)
        if g.is_cuda:
            from ..ops._lib import check, lib, stream_ptr

            if g.dtype not in (torch.bfloat16, torch.float32):
                raise TypeError(f"unsupported grad dtype {g.dtype}")
            gdt = 0 if g.dtype == torch.bfloat16 else 1
            st = stream_ptr(g.device)
            for s, e, wd in self.segments:
                p16 = f.local_data.data_ptr() + s * f.local_data.element_size() if self.master_weights else 0
                check(lib().rca_adamw(self.master.data_ptr() + s * 4, p16, g.data_ptr() + s * g.element_size(), gdt,
                                      self.m.data_ptr() + s * 4, self.v.data_ptr() + s * 4, e - s, lr, self.b1,
                                      self.b2, self.eps, wd, bc1, bc2, grad_scale,
                                      self._sumsq.data_ptr() if clip else 0, float(clip), st), "adamw")
        else:
            coef = 1.0
            if clip:
                nrm = math.sqrt(float(self._sumsq)) * abs(grad_scale)
                coef = min(1.0, clip / (nrm + 1e-6))
            for s, e, wd in self.segments:
                ops.reference.adamw_ref(self.master[s:e], g[s:e], self.m[s:e], self.v[s:e], lr, self.b1, self.b2,
                                        self.eps, wd, t, grad_mul=grad_scale, clip=coef)
            if self.master_weights:
                f.local_data.copy_(self.master.to(f.dtype))
        f.mark_stale()

    def grad_norm(self) -> float:
        return math.sqrt(float(self._sumsq.item())) * abs(self._grad_scale)

    def zero_grad(self, set_to_none: bool = False):
        self.fsdp.zero_grad()

    def state_dict(self):
        """This rank's shard of the optimizer state (save one file per rank)."""
        return {"step": self.step_count, "m": self.m, "v": self.v, "master": self.master if self.master_weights else None,
                "rank": self.fsdp.rank, "world": self.fsdp.world, "lr": self.lr, "betas": (self.b1, self.b2),
                "eps": self.eps, "wd": self.wd}

    def load_state_dict(self, sd):
        if sd.get("world", self.fsdp.world) != self.fsdp.world:
            raise ValueError("sharded optimizer state was saved with a different world size")
        self.step_count = sd["step"]
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        if self.master_weights and sd.get("master") is not None:
            self.master.copy_(sd["master"])
            with torch.no_grad():
                self.fsdp.local_data.copy_(self.master.to(self.fsdp.dtype))
            self.fsdp.mark_stale()


def estimate_memory_gb(cfg, world: int, micro_batch: int = 1, seq_len: int = 4096, reduce_bytes: int = 2,
                       activation_bytes_per_token_layer: Optional[float] = None) -> Dict[str, float]:
    """Per-GPU HBM model of ZeRO-3 training of a ``LlamaConfig`` (no activation recomputation).

    Sharded state: bf16 weights (2) + reduced grads (``reduce_bytes``) + fp32 master, m, v (12)
    per param / world. Transient: two gathered block units (weights + grads, bf16) and the
    resident root unit (embedding + lm_head + norm, weights + grads). Activations saved for
    backward per token per layer (bf16): the block input/residual, normed input, fused qkv,
    attention output + logsumexp, second residual + norm, gate|up, SwiGLU output -> about
    ``2 * (5H + (Hq + 2Hkv)D + 3I) + 4Hq`` bytes; plus the fp32/bf16 logits of one micro-batch.
    """
    P = cfg.num_params()
    H, I, L, V = cfg.hidden_size, cfg.intermediate_size, cfg.num_layers, cfg.vocab_size
    D = cfg.head_dim
    kv = cfg.num_kv_heads * D
    per_layer = H * (H + 2 * kv) + H * H + 2 * H * I + I * H + 2 * H
    root = V * H * (1 if cfg.tie_embeddings else 2) + H
    sharded = P * (2 + reduce_bytes + 12) / world / 1e9
    transient = (2 * per_layer * 2 * 2 + root * 2 * 2) / 1e9
    if activation_bytes_per_token_layer is None:
        activation_bytes_per_token_layer = 2 * (5 * H + (cfg.num_heads * D + 2 * kv) + 3 * I) + 4 * cfg.num_heads + 8
    T = micro_batch * seq_len
    acts = activation_bytes_per_token_layer * T * L / 1e9
    logits = T * V * 2 / 1e9
    total = sharded + transient + acts + logits
    return {"sharded_state": sharded, "transient_units": transient, "activations": acts, "logits": logits,
            "total": total}
