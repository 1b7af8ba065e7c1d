"""MI355X (gfx950) fused ops with autograd.

Every op has two paths:
  * CUDA/HIP tensors -> the hand-written gfx950 kernels in ``ops/csrc`` (mandatory on GPU:
    a missing kernel library raises, there is no silent eager fallback);
  * CPU tensors -> the plain PyTorch fp32 reference in ``ops/reference.py``.

Reference parity notes: RMSNorm/SwiGLU/RoPE follow the HF Llama numerics (normalise in fp32,
round to bf16 before the weight multiply). GAE follows
``rllib/evaluation/postprocessing.py:compute_advantages`` (/root/reference) generalised to
per-step terminated/done flags.
"""
from __future__ import annotations

import os

import torch

from . import reference as ref
from ._lib import check, lib, stream_ptr

__all__ = [
    "rms_norm",
    "swiglu",
    "apply_rope_",
    "rope_cos_sin",
    "cross_entropy",
    "grad_sumsq",
    "compute_gae",
    "vtrace",
    "standardize_", "gbdt_histogram",
    "batched_concat",
    "image_normalize",
    "crop_resize_normalize",
    "batch_norm_act",
    "flash_attention",
    "flash_attention_qkv",
    "flash_attention_supported",
    "kernels_available",
]

rope_cos_sin = ref.rope_cos_sin


def kernels_available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def _p(t):
    return 0 if t is None else t.data_ptr()


# ----------------------------------------------------------------------------------- RMSNorm
class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps, residual):
        H = x.shape[-1]
        x2 = x.contiguous().view(-1, H)
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
        s = None
        r2 = None
        if residual is not None:
            r2 = residual.contiguous().view(-1, H)
            s = torch.empty_like(x2)
        L = lib()
        check(L.rca_rmsnorm_fwd(x2.data_ptr(), _p(r2), w.data_ptr(), y.data_ptr(), _p(s), rstd.data_ptr(), rows, H,
                                float(eps), stream_ptr(x.device)), "rmsnorm_fwd")
        saved = s if s is not None else x2
        ctx.save_for_backward(saved, w, rstd)
        ctx.weight = w
        ctx.has_res = residual is not None
        ctx.shape = x.shape
        if s is None:
            return y.view(x.shape)
        return y.view(x.shape), s.view(x.shape)

    @staticmethod
    def backward(ctx, dy, ds=None):
        s, w, rstd = ctx.saved_tensors
        H = s.shape[-1]
        rows = s.shape[0]
        dy2 = dy.contiguous().view(-1, H)
        ds2 = ds.contiguous().view(-1, H) if ds is not None else None
        dx = torch.empty_like(s)
        L = lib()
        nb = L.rca_rmsnorm_bwd_blocks(rows, H)
        part = torch.empty(nb, H, device=s.device, dtype=torch.float32)
        # flat-buffer gradients (parallel/flat.py, DDP grad-ready hooks registered): the column sum
        # accumulates dw straight into the weight's bf16 grad view -- no dw tensor, no separate
        # AccumulateGrad add kernel (two per layer in the 8B step)
        wp = ctx.weight
        view = wp.grad
        into = (ctx.needs_input_grad[1] and view is not None and view.dtype == torch.bfloat16 and view.is_cuda
                and view.is_contiguous() and getattr(wp, "_rca_grad_ready", None) is not None)
        dw = None if into else torch.empty_like(w)
        check(L.rca_rmsnorm_bwd(s.data_ptr(), dy2.data_ptr(), w.data_ptr(), rstd.data_ptr(), _p(ds2), dx.data_ptr(),
                                part.data_ptr(), (view if into else dw).data_ptr(), 0, 1 if into else 0, rows, H,
                                stream_ptr(s.device)), "rmsnorm_bwd")
        dx = dx.view(ctx.shape)
        if into:
            wp._rca_grad_ready(wp)
        return dx, dw, None, (dx if ctx.has_res else None)


def rms_norm(x, weight, eps: float = 1e-5, residual=None):
    """RMSNorm(x [+ residual]) * weight. With ``residual`` returns ``(y, x + residual)``."""
    if x.is_cuda:
        assert x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16, "HIP RMSNorm expects bf16"
        return _RMSNorm.apply(x, weight, eps, residual)
    y, s = ref.rms_norm_ref(x, weight, eps, residual)
    return y if residual is None else (y, s)


# ----------------------------------------------------------------------------------- SwiGLU
# Transposed gradient side channel: a backward kernel that already has a gradient tile in
# registers can also emit its transpose (one extra write instead of a later read + write
# transpose pass). The consumer -- the weight GEMM of the linear that produced the forward input
# (parallel/fused_linear.py) -- looks the transposed copy up by the gradient's storage pointer.
_GRAD_T = {}


def put_grad_transposed(g, gT):
    import weakref

    for k in [k for k, (r, _) in _GRAD_T.items() if r() is None]:  # producers' grads already freed
        del _GRAD_T[k]
    _GRAD_T[(g.data_ptr(), tuple(g.shape))] = (weakref.ref(g), gT)


def pop_grad_transposed(g):
    """The transposed copy a producer registered for gradient ``g`` (None if there is none). A
    match needs the registered gradient to be alive (then its storage cannot have been reused)."""
    if not _GRAD_T:
        return None
    hit = _GRAD_T.pop((g.data_ptr(), tuple(g.shape)), None)
    if hit is None or hit[0]() is None:
        return None
    return hit[1]


def _swiglu_tr_ok(gu) -> bool:
    return gu.dim() == 2 and gu.shape[0] % 64 == 0 and (gu.shape[1] // 2) % 64 == 0 and gu.is_contiguous()


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, with_t):
        gu = gu.contiguous()
        F2 = gu.shape[-1]
        F = F2 // 2
        T = gu.numel() // F2
        out = torch.empty(*gu.shape[:-1], F, device=gu.device, dtype=gu.dtype)
        ctx.tr = bool(with_t) and _swiglu_tr_ok(gu)
        ctx.save_for_backward(gu)
        ctx.set_materialize_grads(False)  # out^T gets no gradient: no [F, T] zero tensor per layer
        if ctx.tr:
            out_t = torch.empty(F, T, device=gu.device, dtype=gu.dtype)
            check(lib().rca_swiglu_fwd_tr(gu.data_ptr(), out.data_ptr(), out_t.data_ptr(), T, F,
                                          stream_ptr(gu.device)), "swiglu_fwd_tr")
            ctx.mark_non_differentiable(out_t)
            return out, out_t
        check(lib().rca_swiglu_fwd(gu.data_ptr(), out.data_ptr(), T, F, stream_ptr(gu.device)), "swiglu_fwd")
        return out, None

    @staticmethod
    def backward(ctx, dout, _dout_t=None):
        (gu,) = ctx.saved_tensors
        if dout is None:
            return None, None
        return swiglu_backward(gu, dout, ctx.tr), None


def swiglu_backward(gu, dout, with_transposed: bool = False):
    """d(gate|up) of ``swiglu(gu)`` (GPU kernels). ``with_transposed`` (the ``_swiglu_tr_ok``
    shapes) also writes its transpose and registers it for the producing linear's weight GEMM."""
    gu = gu.contiguous()
    F2 = gu.shape[-1]
    T = gu.numel() // F2
    dgu = torch.empty_like(gu)
    dout = dout.contiguous()
    if with_transposed and _swiglu_tr_ok(gu):
        dgu_t = torch.empty(F2, T, device=gu.device, dtype=gu.dtype)
        check(lib().rca_swiglu_bwd_tr(gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), dgu_t.data_ptr(), T,
                                      F2 // 2, stream_ptr(gu.device)), "swiglu_bwd_tr")
        put_grad_transposed(dgu, dgu_t)
    else:
        check(lib().rca_swiglu_bwd(gu.data_ptr(), dout.data_ptr(), dgu.data_ptr(), T, F2 // 2,
                                   stream_ptr(gu.device)), "swiglu_bwd")
    return dgu


def swiglu(gu, with_transposed: bool = False):
    """silu(gu[..., :F]) * gu[..., F:] for the fused gate|up projection output.

    ``with_transposed=True`` (2-D, T and F multiples of 64, GPU) returns ``(out, out^T)``: the
    transposed copy feeds the next linear's weight gradient, and the backward registers the
    transposed input gradient for the producing linear (``pop_grad_transposed``). Otherwise
    ``(out, None)`` is returned in that mode."""
    if gu.is_cuda:
        out, out_t = _SwiGLU.apply(gu, with_transposed)
        return (out, out_t) if with_transposed else out
    out = ref.swiglu_ref(gu)
    return (out, None) if with_transposed else out


def gemm_swiglu_bwd_supported(dy, w_t, gu) -> bool:
    """Shapes of the fused down-projection dgrad + SwiGLU backward (ops/csrc/gemm4.hip variant 7,
    EPI 1): T, F multiples of 256, H of 128, bf16 CUDA, unit inner strides, contiguous gu."""
    if not (dy.is_cuda and dy.dim() == 2 and w_t.dim() == 2 and gu.dim() == 2):
        return False
    T, H = dy.shape
    F = w_t.shape[0]
    return (T % 256 == 0 and F % 256 == 0 and H % 128 == 0 and w_t.shape[1] == H and tuple(gu.shape) == (T, 2 * F)
            and gu.is_contiguous() and all(_gemm_operand_ok(t) for t in (dy, w_t, gu)))


def gemm_swiglu_bwd(dy, w_t, gu):
    """``(dgu, dgu^T)`` for ``y = swiglu(gu) @ W^T`` given ``dy``: the input gradient of the down
    projection, ``dh = dy @ W`` (``w_t`` = ``W^T``, ``[F, H]``), stays in the GEMM's registers and
    its epilogue applies the SwiGLU backward (``dgu = [dh * u * s(g)(1 + g(1 - s(g))), dh * silu(g)]``)
    and writes ``dgu`` and its transpose; no ``dh`` tensor, no separate SwiGLU pass."""
    if not gemm_swiglu_bwd_supported(dy, w_t, gu):
        raise ValueError("gemm_swiglu_bwd: unsupported operands")
    T, H = dy.shape
    F = w_t.shape[0]
    dgu = torch.empty_like(gu)
    dgu_t = torch.empty(2 * F, T, device=gu.device, dtype=gu.dtype)
    check(lib().rca_gemm_swiglu_bwd(dy.data_ptr(), w_t.data_ptr(), gu.data_ptr(), dgu.data_ptr(), dgu_t.data_ptr(),
                                    T, F, H, dy.stride(0), w_t.stride(0), stream_ptr(dy.device)), "gemm_swiglu_bwd")
    return dgu, dgu_t


def transpose_supported(x) -> bool:
    """2-D bf16 CUDA tensor, unit inner stride, both dims multiples of 64, 16-B aligned rows."""
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.bfloat16 and x.stride(1) == 1 and x.shape[0] % 64 == 0
            and x.shape[1] % 64 == 0 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0)


def transpose(x, out=None):
    """``x.t().contiguous()`` for a 2-D bf16 tensor: one LDS-tiled pass at HBM rate on the GPU
    (torch's generic permute copy runs at a fraction of it). CPU / unsupported shapes: torch."""
    if not transpose_supported(x):
        return x.t().contiguous() if out is None else out.copy_(x.t())
    R, C = x.shape
    if out is None:
        out = torch.empty((C, R), device=x.device, dtype=x.dtype)
    check(lib().rca_transpose_bf16(x.data_ptr(), out.data_ptr(), R, C, x.stride(0), stream_ptr(x.device)),
          "transpose_bf16")
    return out


# ----------------------------------------------------------------------------------- GEMM
def _gemm_operand_ok(t) -> bool:
    return (t.is_cuda and t.dim() == 2 and t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0)


def gemm_supported(M: int, N: int, K: int, *tensors) -> bool:
    """Shapes the hand-written gfx950 GEMM (ops/csrc/gemm.hip) takes: M, N multiples of 256, K of
    64, bf16 CUDA operands with unit inner stride and 16-B aligned rows."""
    return M % 256 == 0 and N % 256 == 0 and K % 64 == 0 and M > 0 and N > 0 and K > 0 and all(
        _gemm_operand_ok(t) for t in tensors)


def gemm(a, b, a_kmajor: bool = False, b_kmajor: bool = False, out=None, accumulate: bool = False):
    """``C[M][N] (+)= sum_k A(m,k) B(n,k)`` on the gfx950 MFMA GEMM.

    ``a`` is ``[M][K]`` (``a_kmajor=False``) or ``[K][M]`` (True); ``b`` is ``[N][K]`` or ``[K][N]``.
    So ``gemm(x, w)`` = ``x @ w.T`` (linear forward), ``gemm(dy, w, b_kmajor=True)`` = ``dy @ w``
    (dgrad) and ``gemm(dy, x, True, True)`` = ``dy.T @ x`` (wgrad), all without transposed copies.
    """
    M, K = (a.shape[1], a.shape[0]) if a_kmajor else a.shape
    N, Kb = (b.shape[1], b.shape[0]) if b_kmajor else b.shape
    if K != Kb:
        raise ValueError(f"gemm: reduction dims differ ({K} vs {Kb})")
    if out is None:
        if accumulate:
            raise ValueError("gemm: accumulate needs out")
        out = torch.empty((M, N), device=a.device, dtype=torch.bfloat16)
    if not gemm_supported(M, N, K, a, b, out) or tuple(out.shape) != (M, N):
        raise ValueError(f"gemm: unsupported operands M={M} N={N} K={K}")
    check(lib().rca_gemm_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0), b.stride(0),
                              out.stride(0), int(a_kmajor), int(b_kmajor), int(accumulate), stream_ptr(a.device)),
          "gemm_bf16")
    return out


# ----------------------------------------------------------------------------------- RoPE
class _RoPE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cs, seq_len, n_rot_heads, head_dim, positions):
        T = qkv.shape[0]
        row_stride = qkv.stride(0)
        check(lib().rca_rope(qkv.data_ptr(), cs.data_ptr(), _p(positions), T, seq_len, n_rot_heads, row_stride, head_dim,
                             0, stream_ptr(qkv.device)), "rope_fwd")
        ctx.mark_dirty(qkv)
        ctx.save_for_backward(cs, positions) if positions is not None else ctx.save_for_backward(cs)
        ctx.meta = (seq_len, n_rot_heads, head_dim, positions is not None)
        return qkv

    @staticmethod
    def backward(ctx, g):
        seq_len, n_rot, D, has_pos = ctx.meta
        saved = ctx.saved_tensors
        cs = saved[0]
        pos = saved[1] if has_pos else None
        if not getattr(g, "_rca_owned_grad", False) or not g.is_contiguous():
            g = g.contiguous().clone()  # never rotate a gradient buffer someone else may still read
        T, Wd = g.shape
        if _ROPE_BWD_TR and D == 128 and T % 128 == 0 and Wd % 128 == 0:
            # rotate back AND write g^T for the qkv weight gradient in one pass (the linear's
            # backward picks the transposed copy up by the gradient's storage: no transpose pass)
            g_t = torch.empty(Wd, T, device=g.device, dtype=g.dtype)
            check(lib().rca_rope_bwd_tr(g.data_ptr(), cs.data_ptr(), _p(pos), g_t.data_ptr(), T, seq_len, Wd, n_rot,
                                        stream_ptr(g.device)), "rope_bwd_tr")
            put_grad_transposed(g, g_t)
            return g, None, None, None, None, None
        check(lib().rca_rope(g.data_ptr(), cs.data_ptr(), _p(pos), g.shape[0], seq_len, n_rot, g.stride(0), D, 1,
                             stream_ptr(g.device)), "rope_bwd")
        return g, None, None, None, None, None


# RCA_ROPE_BWD_TR=0: the separate in-place RoPE backward (+ the consumer's own transpose), for A/B
_ROPE_BWD_TR = os.environ.get("RCA_ROPE_BWD_TR", "1") != "0"


def apply_rope_(qkv, cs, seq_len: int, n_q_heads: int, n_kv_heads: int, head_dim: int, positions=None):
    """Rotate the q and k heads of a fused ``qkv`` [T, (Hq + 2*Hkv) * D] tensor in place.

    Position of token t is ``positions[t]`` if given else ``t % seq_len``. ``cs`` comes from
    :func:`rope_cos_sin`.
    """
    n_rot = n_q_heads + n_kv_heads
    if qkv.is_cuda:
        assert qkv.dim() == 2 and qkv.stride(1) == 1
        pos = positions.to(torch.int32).contiguous() if positions is not None else None
        return _RoPE.apply(qkv, cs, seq_len, n_rot, head_dim, pos)
    T = qkv.shape[0]
    pos = positions if positions is not None else torch.arange(T, device=qkv.device) % seq_len
    x = qkv[:, : n_rot * head_dim].reshape(T, n_rot, head_dim)
    rot = ref.rope_ref(x, cs, pos).reshape(T, n_rot * head_dim)
    return torch.cat([rot, qkv[:, n_rot * head_dim:]], dim=1)


# ----------------------------------------------------------------------------------- cross-entropy
class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, inplace_backward):
        logits = logits.contiguous()
        T, V = logits.shape
        labels = labels.contiguous().to(torch.int64)
        loss = torch.empty(T, device=logits.device, dtype=torch.float32)
        lse = torch.empty(T, device=logits.device, dtype=torch.float32)
        check(lib().rca_ce_fwd(logits.data_ptr(), labels.data_ptr(), loss.data_ptr(), lse.data_ptr(), T, V, ignore_index,
                               stream_ptr(logits.device)), "ce_fwd")
        ctx.save_for_backward(logits, labels, lse)
        ctx.ignore_index = ignore_index
        ctx.inplace = inplace_backward
        return loss

    @staticmethod
    def backward(ctx, gloss):
        logits, labels, lse = ctx.saved_tensors
        T, V = logits.shape
        gl = gloss.contiguous().float()
        d = logits if ctx.inplace else torch.empty_like(logits)
        check(lib().rca_ce_bwd(logits.data_ptr(), labels.data_ptr(), lse.data_ptr(), gl.data_ptr(), 0.0, d.data_ptr(), T, V,
                               ctx.ignore_index, stream_ptr(logits.device)), "ce_bwd")
        return d, None, None, None


def cross_entropy(logits, labels, ignore_index: int = -100, reduction: str = "mean", inplace_backward: bool = False):
    """Softmax cross-entropy over the last dim of 2-D ``logits`` (bf16 on GPU).

    ``inplace_backward=True`` writes dlogits over the logits buffer (only safe when nothing else
    reads the logits after the loss).
    """
    if not logits.is_cuda:
        return ref.cross_entropy_ref(logits, labels, ignore_index, reduction)
    rows = _CrossEntropy.apply(logits, labels, ignore_index, inplace_backward)
    if reduction == "none":
        return rows
    if reduction == "sum":
        return rows.sum()
    n = (labels != ignore_index).sum().clamp_min(1)
    return rows.sum() / n


def ce_fused_(logits, labels, gscale, ignore_index: int = -100):
    """One-pass HIP cross-entropy over 2-D bf16 ``logits``: returns per-row losses (fp32) and
    overwrites ``logits`` with ``gscale * (softmax - onehot)`` (ignored rows -> 0). ``gscale`` is
    a 1-element fp32 device tensor. Needs V % 8 == 0 and V <= 131072."""
    T, V = logits.shape
    assert logits.is_contiguous() and logits.dtype == torch.bfloat16
    labels = labels.contiguous().to(torch.int64)
    loss = torch.empty(T, device=logits.device, dtype=torch.float32)
    lse = torch.empty(T, device=logits.device, dtype=torch.float32)
    check(lib().rca_ce_fused(logits.data_ptr(), labels.data_ptr(), gscale.data_ptr(), loss.data_ptr(), lse.data_ptr(),
                             T, V, ignore_index, stream_ptr(logits.device)), "ce_fused")
    return loss


def ce_fused_supported(V: int) -> bool:
    return V % 8 == 0 and 0 < V <= 131072


# ----------------------------------------------------------------------------------- grad norm
_WS = {}


def _workspace(device, key, numel, dtype=torch.float32, zero=False):
    k = (str(device), key)
    t = _WS.get(k)
    if t is None or t.numel() < numel:
        t = (torch.zeros if zero else torch.empty)(numel, device=device, dtype=dtype)
        _WS[k] = t
    return t


# floats of the rca_sumsq workspace: 1024 block partials + the last-block ticket word (zeroed once;
# every launch leaves it zero again)
SUMSQ_WS = 1028


def grad_sumsq(tensors, out=None):
    """Device scalar sum of squares over a list of bf16/f32 tensors (no host sync)."""
    tensors = [t for t in tensors if t is not None]
    if not tensors:
        return torch.zeros((), dtype=torch.float32)
    dev = tensors[0].device
    if not tensors[0].is_cuda:
        s = sum(t.float().pow(2).sum() for t in tensors)
        if out is None:
            return s
        out.reshape(-1)[0] = s
        return out
    out = torch.zeros(1, device=dev, dtype=torch.float32) if out is None else out
    part = _workspace(dev, "sumsq", SUMSQ_WS, zero=True)
    L = lib()
    st = stream_ptr(dev)
    for i, t in enumerate(tensors):
        t = t.contiguous()
        dt = 0 if t.dtype == torch.bfloat16 else 1
        if t.dtype not in (torch.bfloat16, torch.float32):
            t = t.float()
            dt = 1
        check(L.rca_sumsq(t.data_ptr(), t.numel(), dt, part.data_ptr(), out.data_ptr(), 1 if i else 0, st), "sumsq")
    return out


# ----------------------------------------------------------------------------------- RL ops
def compute_gae(rewards, values, terminateds, dones=None, gamma=0.99, lam=0.95, last_values=None, next_values=None,
                standardize=False, eps=1e-4):
    """GAE over [B, T] trajectories. Returns ``(advantages, value_targets)`` (float32).

    ``dones`` (terminated or truncated) cuts the recurrence, ``terminateds`` zeroes the bootstrap.
    ``next_values[b, t]`` = V(s_{t+1}) if available (exact under auto-reset/truncation); else
    V(s_{t+1}) = values[b, t+1] and ``last_values[b]`` at the fragment end.
    """
    if dones is None:
        dones = terminateds
    squeeze = rewards.dim() == 1
    if squeeze:
        rewards, values, terminateds, dones = (x.unsqueeze(0) for x in (rewards, values, terminateds, dones))
        if next_values is not None:
            next_values = next_values.unsqueeze(0)
        if last_values is not None:
            last_values = torch.as_tensor(last_values).reshape(1)
    B, T = rewards.shape
    if rewards.is_cuda:
        dev = rewards.device
        f = lambda x: x.to(device=dev, dtype=torch.float32).contiguous() if x is not None else None  # noqa: E731
        u8 = lambda x: _as_u8(x, dev)  # noqa: E731
        r, v, nv, lv = f(rewards), f(values), f(next_values), f(last_values)
        te, do = u8(terminateds), u8(dones)
        adv = torch.empty(B, T, device=dev, dtype=torch.float32)
        tgt = torch.empty_like(adv)
        part = _workspace(dev, "gae_part", 2 * ((B + 3) // 4))
        stats = _workspace(dev, "gae_stats", 2)
        check(lib().rca_gae(r.data_ptr(), v.data_ptr(), _p(nv), _p(lv), te.data_ptr(), do.data_ptr(), adv.data_ptr(),
                            tgt.data_ptr(), B, T, float(gamma), float(lam), 1 if standardize else 0, part.data_ptr(),
                            stats.data_ptr(), float(eps), stream_ptr(dev)), "gae")
    else:
        adv, tgt = _gae_cpu(rewards, values, terminateds, dones, gamma, lam, last_values, next_values)
        if standardize:
            adv = (adv - adv.mean()) / (adv.std(unbiased=False) + eps)
    if squeeze:
        adv, tgt = adv[0], tgt[0]
    return adv, tgt


def vtrace(log_rhos, rewards, values, next_values, terminateds, dones=None, gamma=0.99, clip_rho_threshold=1.0,
           clip_c_threshold=1.0, clip_pg_rho_threshold=1.0):
    """V-trace targets over ``[B, T]`` fragments. Returns ``(vs, pg_advantages)`` (float32).

    ``log_rhos`` = log pi(a|s) - log mu(a|s); ``next_values[b, t]`` = V(s_{t+1}) (used at episode
    cuts and the fragment end); ``dones`` cuts the trace, ``terminateds`` zeroes the bootstrap.
    """
    if dones is None:
        dones = terminateds
    B, T = rewards.shape
    if rewards.is_cuda:
        dev = rewards.device
        f = lambda x: x.to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
        u8 = lambda x: _as_u8(x, dev)  # noqa: E731
        lr, r, v, nv, te, do = f(log_rhos), f(rewards), f(values), f(next_values), u8(terminateds), u8(dones)
        vs = torch.empty(B, T, device=dev, dtype=torch.float32)
        pg = torch.empty_like(vs)
        check(lib().rca_vtrace(lr.data_ptr(), r.data_ptr(), v.data_ptr(), nv.data_ptr(), te.data_ptr(), do.data_ptr(),
                               vs.data_ptr(), pg.data_ptr(), B, T, float(gamma), float(clip_rho_threshold),
                               float(clip_c_threshold), float(clip_pg_rho_threshold), stream_ptr(dev)), "vtrace")
        return vs, pg
    return ref.vtrace_ref(log_rhos, rewards, values, next_values, terminateds, dones, gamma, clip_rho_threshold,
                          clip_c_threshold, clip_pg_rho_threshold)


def _as_u8(x, dev):
    """Flags as uint8 for the RL kernels: a contiguous bool tensor on the device is reinterpreted
    in place (same 1-byte storage) instead of converted by an extra elementwise kernel."""
    x = torch.as_tensor(x)
    if x.dtype == torch.bool and x.device == torch.device(dev) and x.is_contiguous():
        return x.view(torch.uint8)
    return x.to(device=dev, dtype=torch.uint8).contiguous()


def _gae_cpu(rewards, values, terminateds, dones, gamma, lam, last_values, next_values):
    r = torch.as_tensor(rewards, dtype=torch.float32)
    v = torch.as_tensor(values, dtype=torch.float32)
    te = torch.as_tensor(terminateds).bool()
    do = torch.as_tensor(dones).bool()
    B, T = r.shape
    if next_values is not None:
        nv = torch.as_tensor(next_values, dtype=torch.float32)
    else:
        lv = torch.zeros(B) if last_values is None else torch.as_tensor(last_values, dtype=torch.float32).reshape(B)
        nv = torch.cat([v[:, 1:], lv[:, None]], dim=1)
    delta = r + gamma * torch.where(te, torch.zeros_like(nv), nv) - v
    c = gamma * lam * (~do).float()
    adv = torch.empty_like(r)
    A = torch.zeros(B)
    for t in range(T - 1, -1, -1):  # vectorised over B
        A = delta[:, t] + c[:, t] * A
        adv[:, t] = A
    return adv, adv + v


def standardize_(x, eps=1e-4):
    """In-place (x - mean) / (std + eps) over all elements (float32)."""
    if x.is_cuda:
        assert x.dtype == torch.float32 and x.is_contiguous()
        part = _workspace(x.device, "std_part", 2048)
        stats = _workspace(x.device, "std_stats", 2)
        check(lib().rca_standardize(x.data_ptr(), x.numel(), part.data_ptr(), stats.data_ptr(), float(eps),
                                    stream_ptr(x.device)), "standardize")
        return x
    m, s = x.mean(), x.std(unbiased=False)
    return x.sub_(m).div_(s + eps)


# ----------------------------------------------------------------------------------- GBDT
_GBDT_Q = {}


def gbdt_quantize(gh):
    """(grad, hess[, count]) float32 [ld, C] -> one packed fixed-point int64 per row (signed
    grad * sg in the high 32 bits, hess * sh >= 0 in the low 32) + device scales [1/sg, 1/sh],
    the operand of the GPU histogram kernel (``ops/csrc/gbdt.hip``: one ds_add_u64 per (row,
    feature); the kernel's <= 32768 rows per workgroup bound the per-row magnitudes to 2^16 / 2^17).
    Cached per (tensor, version) so the levels of one tree quantise once."""
    hit = _GBDT_Q.get(gh.device)
    if hit is not None and hit[0] is gh and hit[3] == gh._version:
        return hit[1], hit[2]
    g, h = gh[:, 0], gh[:, 1]
    gmax = g.abs().max().clamp_min(1e-30)
    hmax = h.max().clamp_min(1e-30)
    sg, sh = 65535.0 / gmax, 131071.0 / hmax
    gq = torch.round(g * sg).to(torch.int64)
    hq = torch.round(h.clamp_min(0) * sh).to(torch.int64)
    packed = (gq << 32) + hq
    inv = torch.stack([1.0 / sg, 1.0 / sh]).to(torch.float32)
    _GBDT_Q[gh.device] = (gh, packed, inv, gh._version)
    return packed, inv


# Fixed-point histograms keep the hessian sums to ~1e-5 of the LARGEST per-row hessian; when the
# hessians span more than this ratio (e.g. confident logistic rows next to uncertain ones) the
# smallest would keep fewer than ~128 quantisation steps, biasing min_child_weight checks and
# leaf values, so "auto" switches to the exact (fp64-accumulated) kernel.
GBDT_EXACT_HESS_RATIO = 2.0 ** 10


def _gbdt_needs_exact(gh) -> bool:
    hit = _GBDT_Q.get(("exact", gh.device))
    if hit is not None and hit[0] is gh and hit[2] == gh._version:
        return hit[1]
    h = gh[:, 1]
    pos = h[h > 0]
    need = bool(pos.numel() and (pos.max() / pos.min()).item() > GBDT_EXACT_HESS_RATIO)
    _GBDT_Q[("exact", gh.device)] = (gh, need, gh._version)
    return need


def gbdt_histogram(bins, node, gh, num_nodes, out=None, precision: str = "auto"):
    """Per-node gradient histograms for histogram GBDT (``train/gbdt``).

    bins: uint8 [F, ld] feature-major quantised matrix (bin 255 = missing), node: int32 [ld] node
    slot of every row (-1 = skip), gh: float32 [ld, C] (grad, hess[, count: 1 per row]).
    Returns float32 [num_nodes, F, 256, C].

    ``precision``: "fixed" -- GPU ``gbdt_hist_kernel`` over the fixed-point packed (grad, hess) of
    :func:`gbdt_quantize` (error ~1e-5 of the largest |grad| / hess per row; the count is exact;
    CPU: one fp32 ``index_add_``); "exact" -- fp64 accumulation rounded to fp32 once, the SAME
    numbers on GPU (``gbdt_hist_exact_kernel``, fp64 LDS atomics) and CPU (fp64 ``index_add_``)
    up to the last bit of the fp64 sum, for parity checks; "auto" (default) -- "fixed" unless the
    positive hessians span more than ``GBDT_EXACT_HESS_RATIO``. ld % 4 == 0 on GPU."""
    if precision not in ("auto", "fixed", "exact"):
        raise ValueError(f"precision must be auto|fixed|exact, got {precision!r}")
    exact = precision == "exact" or (precision == "auto" and bins.is_cuda and _gbdt_needs_exact(gh))
    F, ld = bins.shape
    C = gh.shape[1]
    if out is None:  # the GPU path writes every entry
        out = (torch.empty if bins.is_cuda else torch.zeros)(num_nodes, F, 256, C, dtype=torch.float32,
                                                              device=bins.device)
    elif not bins.is_cuda:
        out.zero_()
    if bins.is_cuda:
        assert bins.dtype == torch.uint8 and node.dtype == torch.int32 and gh.dtype == torch.float32
        assert bins.is_contiguous() and node.is_contiguous() and gh.is_contiguous()
        assert ld % 4 == 0 and node.numel() == ld and gh.shape[0] == ld and C in (2, 3)
        assert out.shape == (num_nodes, F, 256, C) and out.is_contiguous()
        if exact:
            nbytes = int(lib().rca_gbdt_hist_exact_workspace(F, ld, int(num_nodes), C))
            work = _workspace(bins.device, "gbdt_hist_exact", (nbytes + 3) // 4)
            check(lib().rca_gbdt_hist_exact(bins.data_ptr(), node.data_ptr(), gh.data_ptr(), out.data_ptr(),
                                            work.data_ptr(), F, ld, int(num_nodes), C, stream_ptr(bins.device)),
                  "gbdt_hist_exact")
            return out
        packed, inv = gbdt_quantize(gh)
        nbytes = int(lib().rca_gbdt_hist_workspace(F, ld, int(num_nodes), C))
        work = _workspace(bins.device, "gbdt_hist", (nbytes + 3) // 4)
        check(lib().rca_gbdt_hist(bins.data_ptr(), node.data_ptr(), packed.data_ptr(), inv.data_ptr(),
                                  out.data_ptr(), work.data_ptr(), F, ld, int(num_nodes), C,
                                  stream_ptr(bins.device)), "gbdt_hist")
        return out
    keep = (node >= 0) & (node < num_nodes)
    rows = keep.nonzero().squeeze(1)
    if rows.numel() == 0:
        return out
    nd = node[rows].long()
    idx = (nd[None, :] * F + torch.arange(F, device=bins.device)[:, None]) * 256 + bins[:, rows].long()
    if exact:
        vals = gh[rows].double().unsqueeze(0).expand(F, -1, -1)
        acc = torch.zeros(out.numel() // C, C, dtype=torch.float64, device=bins.device)
        acc.index_add_(0, idx.reshape(-1), vals.reshape(-1, C))
        out.view(-1, C).copy_(acc)
        return out
    vals = gh[rows].unsqueeze(0).expand(F, -1, -1)
    out.view(-1, C).index_add_(0, idx.reshape(-1), vals.reshape(-1, C))
    return out


# ----------------------------------------------------------------------------------- data ops
def batched_concat(tensors, dim=0):
    """torch.cat along dim 0 of same-trailing-shape tensors in ONE kernel launch on GPU."""
    if not tensors:
        raise ValueError("empty list")
    if not tensors[0].is_cuda or dim != 0 or len(tensors) == 1:
        return torch.cat(tensors, dim=dim)
    dev, dt = tensors[0].device, tensors[0].dtype
    tail = tensors[0].shape[1:]
    ts = [t.contiguous() for t in tensors]
    for t in ts:
        if t.shape[1:] != tail or t.dtype != dt or t.device != dev:
            return torch.cat(tensors, dim=0)
    out = torch.empty(sum(t.shape[0] for t in ts), *tail, device=dev, dtype=dt)
    esz = out.element_size()
    descs = []
    off = 0
    maxb = 0
    for t in ts:
        nb = t.numel() * esz
        descs += [t.data_ptr(), off, nb]
        off += nb
        maxb = max(maxb, nb)
    d = torch.tensor(descs, dtype=torch.int64).to(dev, non_blocking=True)
    check(lib().rca_batched_copy(d.data_ptr(), len(ts), out.data_ptr(), maxb, stream_ptr(dev)), "batched_copy")
    # keep sources + descriptor alive until the copy retires on this stream
    for t in ts:
        t.record_stream(torch.cuda.current_stream(dev))
    d.record_stream(torch.cuda.current_stream(dev))
    return out


def image_normalize(u8, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), dtype=torch.bfloat16,
                    channels_last: bool = False):
    """uint8 [N, H, W, C] -> normalised [N, C, H, W] (bf16 or f32) on the device of ``u8``.

    ``channels_last=True`` returns the same logical NCHW tensor in NHWC memory (what MIOpen's
    NHWC convolutions consume), written by a 16-byte-vectorised streaming kernel."""
    if not u8.is_cuda:
        out = ref.image_normalize_ref(u8, mean, std, dtype)
        return out.contiguous(memory_format=torch.channels_last) if channels_last else out
    import ctypes

    u8 = u8.contiguous()
    N, H, W, C = u8.shape
    if channels_last:
        out = torch.empty(N, H, W, C, device=u8.device, dtype=dtype).permute(0, 3, 1, 2)
    else:
        out = torch.empty(N, C, H, W, device=u8.device, dtype=dtype)
    ma = (ctypes.c_float * 4)(*[float(m) for m in mean])
    sa = (ctypes.c_float * 4)(*[float(s) for s in std])
    check(lib().rca_image_normalize(u8.data_ptr(), out.data_ptr(), N, H, W, C, ctypes.cast(ma, ctypes.c_void_p),
                                    ctypes.cast(sa, ctypes.c_void_p), 0 if dtype == torch.bfloat16 else 1,
                                    1 if channels_last else 0, stream_ptr(u8.device)), "image_normalize")
    return out


def crop_resize_normalize(u8, boxes, size, flips=None, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                          dtype=torch.bfloat16, channels_last: bool = False):
    """Fused per-image crop -> bilinear resize -> optional h-flip -> normalise (one HIP pass).

    ``u8``: uint8 [N, H, W, C]; ``boxes``: int [N, 4] = (y0, x0, h, w); ``flips``: bool/uint8 [N]
    or None; ``size``: (Ho, Wo). Returns [N, C, Ho, Wo] (channels_last: same logical shape in
    NHWC memory) on ``u8``'s device."""
    Ho, Wo = (size, size) if isinstance(size, int) else tuple(size)
    N, H, W, C = u8.shape
    bx = torch.as_tensor(boxes, dtype=torch.int32).reshape(N, 4)
    if ((bx[:, 0] < 0) | (bx[:, 1] < 0) | (bx[:, 2] < 1) | (bx[:, 3] < 1) | (bx[:, 0] + bx[:, 2] > H)
            | (bx[:, 1] + bx[:, 3] > W)).any():
        raise ValueError("crop boxes must lie inside the images")
    if not u8.is_cuda:
        out = ref.crop_resize_normalize_ref(u8, bx, flips, (Ho, Wo), mean, std, dtype)
        return out.contiguous(memory_format=torch.channels_last) if channels_last else out
    import ctypes

    u8 = u8.contiguous()
    bxd = bx.to(u8.device)
    fl = None if flips is None else torch.as_tensor(flips).to(device=u8.device, dtype=torch.uint8).contiguous()
    if channels_last:
        out = torch.empty(N, Ho, Wo, C, device=u8.device, dtype=dtype).permute(0, 3, 1, 2)
    else:
        out = torch.empty(N, C, Ho, Wo, device=u8.device, dtype=dtype)
    ma = (ctypes.c_float * 4)(*[float(m) for m in mean])
    sa = (ctypes.c_float * 4)(*[float(s) for s in std])
    check(lib().rca_crop_resize_normalize(u8.data_ptr(), out.data_ptr(), bxd.data_ptr(), _p(fl), N, H, W, C, Ho, Wo,
                                          ctypes.cast(ma, ctypes.c_void_p), ctypes.cast(sa, ctypes.c_void_p),
                                          0 if dtype == torch.bfloat16 else 1, 1 if channels_last else 0,
                                          stream_ptr(u8.device)), "crop_resize_normalize")
    return out


# --------------------------------------------------------------------------------- batch norm
def bn_supported(x) -> bool:
    """Shapes/layouts the fused NHWC BatchNorm kernels cover."""
    if x.dim() != 4 or x.dtype != torch.bfloat16 or not x.is_cuda:
        return False
    C = x.shape[1]
    return (C % 8 == 0 and 8 <= C <= 2048 and 256 % (C // 8) == 0
            and x.is_contiguous(memory_format=torch.channels_last))


def _rows(t):
    N, C, H, W = t.shape
    return N * H * W, C


class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, running_mean, running_var, momentum, eps, relu):
        R, C = _rows(x)
        L = lib()
        dev = x.device
        out = torch.empty_like(x, memory_format=torch.channels_last)
        stats = torch.empty(4, C, device=dev, dtype=torch.float32)
        ws = _workspace(dev, "bn", int(L.rca_bn_workspace(R, C)))
        res = residual.contiguous(memory_format=torch.channels_last) if residual is not None else None
        check(L.rca_bn_fwd(x.data_ptr(), res.data_ptr() if res is not None else 0, _p(weight), _p(bias),
                           _p(running_mean), _p(running_var), stats.data_ptr(), ws.data_ptr(), out.data_ptr(), R, C,
                           float(eps), float(momentum), 1 if relu else 0, stream_ptr(dev)), "bn_fwd")
        ctx.save_for_backward(x, out, stats, weight)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.has_w = weight is not None
        ctx.has_b = bias is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        x, out, stats, weight = ctx.saved_tensors
        R, C = _rows(x)
        L = lib()
        dev = x.device
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res else None
        dw = torch.empty(C, device=dev, dtype=torch.float32) if ctx.has_w else None
        db = torch.empty(C, device=dev, dtype=torch.float32) if ctx.has_b else None
        coef = torch.empty(3, C, device=dev, dtype=torch.float32)
        ws = _workspace(dev, "bn", int(L.rca_bn_workspace(R, C)))
        check(L.rca_bn_bwd(dy.data_ptr(), out.data_ptr(), x.data_ptr(), stats.data_ptr(), _p(weight), _p(dw), _p(db),
                           coef.data_ptr(), ws.data_ptr(), dx.data_ptr(), dres.data_ptr() if dres is not None else 0,
                           R, C, 1 if ctx.relu else 0, stream_ptr(dev)), "bn_bwd")
        return dx, dw, db, dres, None, None, None, None, None


def batch_norm_act(x, weight, bias, running_mean=None, running_var=None, training: bool = True,
                   momentum: float = 0.1, eps: float = 1e-5, residual=None, relu: bool = True):
    """``act(batch_norm(x) [+ residual])`` for NCHW-logical tensors.

    channels_last bf16 CUDA tensors in training mode run the fused gfx950 kernels
    (``ops/csrc/batchnorm.hip``); everything else (CPU, eval mode, other layouts) uses the
    PyTorch composition with identical semantics (batch statistics, biased variance for
    normalisation, unbiased variance in the running estimate)."""
    use_kernel = training and bn_supported(x) and (residual is None or residual.shape == x.shape)
    if use_kernel and weight is not None and weight.dtype != torch.float32:
        use_kernel = False
    if not use_kernel:
        y = torch.nn.functional.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
        if residual is not None:
            y = y + residual
        return torch.relu(y) if relu else y
    if residual is not None and residual.dtype != x.dtype:
        residual = residual.to(x.dtype)
    return _BatchNormAct.apply(x, weight, bias, residual, running_mean, running_var, momentum, eps, relu)


def affine_act_(x, stats, residual=None, relu: bool = True):
    """In place: ``x = act(x * stats[2] + stats[3] [+ residual])`` per channel, for a channels_last
    bf16 CUDA tensor (the folded-BatchNorm inference epilogue: bias, residual add and ReLU of a
    convolution's output in ONE NHWC pass, ``rca_bn_apply``). ``stats`` is a float32 [4, C]
    tensor (rows 2 / 3: scale / shift; rows 0 / 1 unused). Other inputs: the torch composition."""
    C = x.shape[1] if x.dim() == 4 else 0
    if bn_supported(x) and stats.is_cuda and (residual is None or (residual.shape == x.shape and residual.dtype ==
                                                                   x.dtype and residual.is_contiguous(
                                                                       memory_format=torch.channels_last))):
        R = x.numel() // C
        check(lib().rca_bn_apply(x.data_ptr(), residual.data_ptr() if residual is not None else None,
                                 stats.data_ptr(), x.data_ptr(), R, C, int(relu), stream_ptr(x.device)),
              "bn_apply")
        return x
    y = x.float() * stats[2].view(1, -1, 1, 1) + stats[3].view(1, -1, 1, 1)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return x.copy_(y.to(x.dtype))


def conv1x1_affine_act_supported(x, weight) -> bool:
    """1x1 / stride-1 NHWC convolutions the in-tree GEMM runs with the affine epilogue:
    M = N*H*W % 256, Cout % 256, Cin % 128 (``rca_gemm_affine_act``)."""
    if not (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last) and weight.dim() == 4
            and tuple(weight.shape[2:]) == (1, 1)):
        return False
    n, c, h, w = x.shape
    return (n * h * w) % 256 == 0 and weight.shape[0] % 256 == 0 and c % 128 == 0 and c == weight.shape[1] and \
        n * h * w * c * 2 < 2 ** 32


def conv1x1_affine_act(x, weight, shift, residual=None, relu: bool = True):
    """``act(conv1x1(x, weight) + shift [+ residual])`` for a channels_last bf16 CUDA tensor: ONE
    kernel, the convolution as a GEMM [N*H*W, Cin] x [Cout, Cin]^T with the shift / residual /
    ReLU applied to the fp32 accumulators (``ops/csrc/gemm4.hip`` EPI 2). ``shift``: fp32 [Cout]
    (the folded BatchNorm shift). Unsupported shapes raise (check ``conv1x1_affine_act_supported``)."""
    if not conv1x1_affine_act_supported(x, weight):
        raise ValueError("conv1x1_affine_act: unsupported shape / layout")
    n, c, h, w = x.shape
    co = weight.shape[0]
    wm = weight.reshape(co, c)
    if not wm.is_contiguous():
        wm = wm.contiguous()
    out = torch.empty((n, co, h, w), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
    sh = shift.contiguous().float()
    if residual is not None and (residual.shape != out.shape or residual.dtype != out.dtype
                                 or not residual.is_contiguous(memory_format=torch.channels_last)):
        residual = residual.to(out.dtype).contiguous(memory_format=torch.channels_last)
    M = n * h * w
    check(lib().rca_gemm_affine_act(x.data_ptr(), wm.data_ptr(), sh.data_ptr(),
                                    residual.data_ptr() if residual is not None else None, out.data_ptr(), M, co, c,
                                    c, c, co, co, int(relu), stream_ptr(x.device)), "gemm_affine_act")
    return out


# --------------------------------------------------------------------------------- attention
def flash_attention_supported(seq_len: int, head_dim: int, n_q_heads: int, n_kv_heads: int) -> bool:
    """Shapes the gfx950 flash-attention kernels cover (others use torch SDPA)."""
    return seq_len % 128 == 0 and head_dim in (64, 128) and n_kv_heads > 0 and n_q_heads % n_kv_heads == 0


def _attn_fwd(q, k, v, o, lse, B, S, Hq, Hk, D, sq, sk, sv, so, scale, causal):
    check(lib().rca_attn_fwd(q, k, v, o, lse, B, S, Hq, Hk, D, sq, sk, sv, so, scale, int(causal), stream_ptr()),
          "rca_attn_fwd")


def _attn_bwd(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, Hq, Hk, D, strides, scale, causal, device=None):
    """Attention backward. With a dS workspace (D = 128, default mode) the dK/dV kernel stores the
    bf16 dS tiles and dQ = dS.K is read back from them (no S/P/dP recomputation for dQ); the
    workspace is a transient caching-allocator block (1.08 GB at the Llama-3-8B shape, reused by
    every layer's backward).

    The workspace grows as B*Hq*S^2 (34 GB at S = 32k, B*Hq = 32), so it is only taken when it fits
    ``attn_ds_workspace_cap(device)`` -- an absolute cap (``RCA_ATTN_DS_WS_MAX_GB``, default 8) and
    a fraction of the device's free memory -- and when the allocation itself succeeds; otherwise the
    O(S)-memory recompute path (dQ kernel recomputing S, P, dP) runs, with the same gradients up to
    rounding (``tests/test_attention_gpu.py::test_ds_workspace_cap_falls_back_to_recompute``)."""
    L = lib()
    nbytes = L.rca_attn_bwd_ws_bytes(B, S, Hq, Hk, D, int(causal))
    ws = None
    if nbytes > 0 and nbytes <= attn_ds_workspace_cap(device):
        try:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        except torch.OutOfMemoryError:
            ws = None
    if ws is None:
        nbytes = 0
    check(L.rca_attn_bwd2(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, Hq, Hk, D, *strides, scale, int(causal),
                          ws.data_ptr() if ws is not None else None, nbytes, stream_ptr()), "rca_attn_bwd2")
    del ws  # stream-ordered: the caching allocator reuses the block only for later work on this stream


_DS_WS_CAP_OVERRIDE = None


def attn_ds_workspace_cap(device=None) -> int:
    """Largest dS workspace (bytes) the attention backward may allocate: min of the absolute cap
    (``RCA_ATTN_DS_WS_MAX_GB``, default 8 GB: 7x the Llama-3-8B bench's 1.08 GB) and half of the
    memory the caching allocator could still hand out (free device memory + its reserved-unused
    blocks). ``set_attn_ds_workspace_cap(n)`` overrides it (tests, memory-tight jobs)."""
    if _DS_WS_CAP_OVERRIDE is not None:
        return int(_DS_WS_CAP_OVERRIDE)
    cap = int(float(os.environ.get("RCA_ATTN_DS_WS_MAX_GB", "8")) * (1 << 30))
    try:
        free, _ = torch.cuda.mem_get_info(device)
        idx = torch.device(device).index if device is not None else None
        spare = torch.cuda.memory_reserved(idx) - torch.cuda.memory_allocated(idx)
        cap = min(cap, (free + max(spare, 0)) // 2)
    except (RuntimeError, AssertionError, ValueError):
        pass
    return cap


def set_attn_ds_workspace_cap(nbytes):
    """Override the dS workspace cap (``None`` restores the default policy); returns the old override."""
    global _DS_WS_CAP_OVERRIDE
    old, _DS_WS_CAP_OVERRIDE = _DS_WS_CAP_OVERRIDE, nbytes
    return old


class _FlashAttnQKV(torch.autograd.Function):
    """Attention straight off the fused qkv projection ``[B*S, (Hq+2Hk)*D]``; output ``[B*S, Hq*D]``.
    The backward writes dQ/dK/dV into one fused ``dqkv`` gradient (no slicing copies)."""

    @staticmethod
    def forward(ctx, qkv, B, S, Hq, Hk, D, causal, scale):
        W = (Hq + 2 * Hk) * D
        o = torch.empty(B * S, Hq * D, device=qkv.device, dtype=qkv.dtype)
        lse = torch.empty(B, Hq, S, device=qkv.device, dtype=torch.float32)
        base, es = qkv.data_ptr(), qkv.element_size()
        _attn_fwd(base, base + es * Hq * D, base + es * (Hq + Hk) * D, o.data_ptr(), lse.data_ptr(), B, S, Hq, Hk, D,
                  W, W, W, Hq * D, scale, causal)
        ctx.save_for_backward(qkv, o, lse)
        ctx.cfg = (B, S, Hq, Hk, D, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        B, S, Hq, Hk, D, causal, scale = ctx.cfg
        do = do.contiguous()
        W = (Hq + 2 * Hk) * D
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(B, Hq, S, device=qkv.device, dtype=torch.float32)
        base, gb, es = qkv.data_ptr(), dqkv.data_ptr(), qkv.element_size()
        _attn_bwd(base, base + es * Hq * D, base + es * (Hq + Hk) * D, o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                  delta.data_ptr(), gb, gb + es * Hq * D, gb + es * (Hq + Hk) * D, B, S, Hq, Hk, D,
                  (W, W, W, Hq * D, Hq * D, W, W, W), scale, causal, qkv.device)
        dqkv._rca_owned_grad = True  # fresh buffer: the RoPE backward may rotate it in place
        return dqkv, None, None, None, None, None, None, None


def flash_attention_qkv(qkv, B: int, S: int, Hq: int, Hk: int, D: int, causal: bool = True, scale=None):
    """Fused-qkv attention: ``qkv`` is ``[B*S, (Hq+2Hk)*D]`` (token-major, heads contiguous)."""
    scale = float(D ** -0.5 if scale is None else scale)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and flash_attention_supported(S, D, Hq, Hk):
        return _FlashAttnQKV.apply(qkv.contiguous(), B, S, Hq, Hk, D, causal, scale)
    q = qkv[:, : Hq * D].view(B, S, Hq, D)
    k = qkv[:, Hq * D: (Hq + Hk) * D].view(B, S, Hk, D)
    v = qkv[:, (Hq + Hk) * D:].view(B, S, Hk, D)
    return ref.attention_ref(q, k, v, causal, scale).reshape(B * S, Hq * D)


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        B, S, Hq, D = q.shape
        Hk = k.shape[2]
        o = torch.empty(B, S, Hq, D, device=q.device, dtype=q.dtype)
        lse = torch.empty(B, Hq, S, device=q.device, dtype=torch.float32)
        _attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, Hq, Hk, D,
                  q.stride(1), k.stride(1), v.stride(1), o.stride(1), scale, causal)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        causal, scale = ctx.cfg
        B, S, Hq, D = q.shape
        Hk = k.shape[2]
        do = do.contiguous()
        dq = torch.empty(B, S, Hq, D, device=q.device, dtype=q.dtype)
        dk = torch.empty(B, S, Hk, D, device=q.device, dtype=q.dtype)
        dv = torch.empty(B, S, Hk, D, device=q.device, dtype=q.dtype)
        delta = torch.empty(B, Hq, S, device=q.device, dtype=torch.float32)
        _attn_bwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                  delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), B, S, Hq, Hk, D,
                  (q.stride(1), k.stride(1), v.stride(1), o.stride(1), do.stride(1), dq.stride(1), dk.stride(1),
                   dv.stride(1)), scale, causal, q.device)
        return dq, dk, dv, None, None


def _token_major_ok(t):
    B, S, H, D = t.shape
    return t.stride(3) == 1 and t.stride(2) == D and t.stride(0) == S * t.stride(1)


def flash_attention(q, k, v, causal: bool = True, scale=None):
    """Attention on ``[B, S, H, D]`` tensors (GQA when k/v have fewer heads). Returns ``[B, S, Hq, D]``."""
    B, S, Hq, D = q.shape
    Hk = k.shape[2]
    scale = float(D ** -0.5 if scale is None else scale)
    if (q.is_cuda and q.dtype == torch.bfloat16 and flash_attention_supported(S, D, Hq, Hk)
            and all(_token_major_ok(t) for t in (q, k, v))):
        return _FlashAttn.apply(q, k, v, causal, scale)
    return ref.attention_ref(q, k, v, causal, scale)
