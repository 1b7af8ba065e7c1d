"""Plain PyTorch fp32 references of every HIP op (numerics oracle for tests, CPU execution path)."""
from __future__ import annotations

import torch


def rms_norm_ref(x, w, eps=1e-5, residual=None):
    s = x if residual is None else (x.float() + residual.float()).to(x.dtype)
    sf = s.float()
    r = torch.rsqrt(sf.pow(2).mean(-1, keepdim=True) + eps)
    y = (sf * r).to(x.dtype).float() * w.float()
    return y.to(x.dtype), s


def swiglu_ref(gu):
    F = gu.shape[-1] // 2
    g, u = gu[..., :F].float(), gu[..., F:].float()
    return (torch.nn.functional.silu(g).to(gu.dtype).float() * u).to(gu.dtype)


def rope_cos_sin(max_pos: int, head_dim: int, theta: float = 500000.0, device=None):
    """[max_pos, head_dim/2, 2] float32 table of (cos, sin) for the rotate-half convention."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    cs = torch.stack([f.cos(), f.sin()], dim=-1).float()
    return cs.to(device) if device is not None else cs


def rope_ref(x, cs, positions):
    """x: [T, H, D] ; cs [max_pos, D/2, 2]; positions [T] -> rotated x (rotate-half convention)."""
    D = x.shape[-1]
    half = D // 2
    c = cs[positions, :, 0][:, None, :]
    s = cs[positions, :, 1][:, None, :]
    xf = x.float()
    a, b = xf[..., :half], xf[..., half:]
    return torch.cat([a * c - b * s, b * c + a * s], dim=-1).to(x.dtype)


def cross_entropy_ref(logits, labels, ignore_index=-100, reduction="mean"):
    return torch.nn.functional.cross_entropy(logits.float(), labels, ignore_index=ignore_index, reduction=reduction)


def adamw_ref(p, g, m, v, lr, b1, b2, eps, wd, step, grad_mul=1.0, clip=1.0):
    g = g.float() * grad_mul * clip
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    p.sub_(lr * ((m / bc1) / ((v / bc2).sqrt() + eps) + wd * p))
    return p


def split_master(master):
    """fp32 master -> (hi, lo): hi = the bit pattern rounded half-up in magnitude to 16 bits (a bf16
    tensor: the model weight; equal to RNE except at exact ties), lo = the low 16 bits (int16
    storage). ``join_master(hi, lo)`` reconstructs ``master`` bit-exactly (loss_optim.hip)."""
    M = master.float().contiguous().view(torch.int32)
    hi = ((M + 0x8000) >> 16) & 0xFFFF
    lo = M & 0xFFFF
    to16 = lambda x: (x - ((x >> 15) << 16)).to(torch.int16)  # 0..65535 -> same 16 bits as int16
    return to16(hi).view(torch.bfloat16), to16(lo)


def join_master(hi, lo):
    """Inverse of ``split_master``: the fp32 master from the bf16 weight and its low halves."""
    h = hi.contiguous().view(torch.int16).to(torch.int32) & 0xFFFF
    l_ = lo.contiguous().to(torch.int32) & 0xFFFF
    up = h - (l_ >> 15)
    return ((up << 16) | l_).view(torch.float32)


def gae_ref(rewards, values, terminateds, dones, gamma, lam, last_values=None, next_values=None):
    """rewards/values/...: [B, T] -> (advantages, value_targets) in fp64-accurate float32."""
    B, T = rewards.shape
    r = rewards.double()
    v = values.double()
    adv = torch.zeros_like(r)
    for b in range(B):
        A = 0.0
        for t in range(T - 1, -1, -1):
            if next_values is not None:
                nv = float(next_values[b, t])
            elif t + 1 < T:
                nv = float(v[b, t + 1])
            else:
                nv = float(last_values[b]) if last_values is not None else 0.0
            d = float(r[b, t]) + gamma * (0.0 if terminateds[b, t] else nv) - float(v[b, t])
            c = gamma * lam * (0.0 if dones[b, t] else 1.0)
            A = d + c * A
            adv[b, t] = A
    return adv.float(), (adv + v).float()


def image_normalize_ref(u8, mean, std, dtype=torch.bfloat16):
    x = u8.float() / 255.0
    m = torch.tensor(mean, dtype=torch.float32).view(1, 1, 1, -1)
    s = torch.tensor(std, dtype=torch.float32).view(1, 1, 1, -1)
    return ((x - m) / s).permute(0, 3, 1, 2).contiguous().to(dtype)


def crop_resize_normalize_ref(u8, boxes, flips, size, mean, std, dtype=torch.float32):
    """Per image: crop box (y0, x0, h, w) -> bilinear resize (align_corners=False) -> optional
    horizontal flip -> /255, mean/std. uint8 [N, H, W, C] -> [N, C, Ho, Wo]."""
    import torch.nn.functional as F

    outs = []
    m = torch.tensor(mean, dtype=torch.float32).view(-1, 1, 1)
    s = torch.tensor(std, dtype=torch.float32).view(-1, 1, 1)
    for n in range(u8.shape[0]):
        y0, x0, h, w = (int(v) for v in boxes[n])
        crop = u8[n, y0:y0 + h, x0:x0 + w, :].float().permute(2, 0, 1)[None]
        r = F.interpolate(crop, size=tuple(size), mode="bilinear", align_corners=False, antialias=False)[0]
        if flips is not None and bool(flips[n]):
            r = r.flip(-1)
        outs.append((r / 255.0 - m) / s)
    return torch.stack(outs).to(dtype)


def attention_ref(q, k, v, causal: bool = True, scale=None):
    """fp32 attention on ``[B, S, H, D]`` tensors (GQA by head repetition); returns q's dtype."""
    B, S, Hq, D = q.shape
    Hk = k.shape[2]
    scale = D ** -0.5 if scale is None else scale
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if Hk != Hq:
        kf = kf.repeat_interleave(Hq // Hk, dim=1)
        vf = vf.repeat_interleave(Hq // Hk, dim=1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        m = torch.ones(S, k.shape[1], dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    o = torch.matmul(torch.softmax(s, dim=-1), vf)
    return o.transpose(1, 2).to(q.dtype)


def vtrace_ref(log_rhos, rewards, values, next_values, terminateds, dones, gamma=0.99, clip_rho=1.0, clip_c=1.0,
               clip_pg=1.0):
    """Sequential fp32 V-trace (see ops/csrc/rl_data.hip vtrace_kernel for the recurrences)."""
    lr, r, v, nv = (torch.as_tensor(x, dtype=torch.float32) for x in (log_rhos, rewards, values, next_values))
    term = torch.as_tensor(terminateds).bool()
    done = torch.as_tensor(dones).bool()
    B, T = r.shape
    ir = lr.exp()
    rho, c, rpg = ir.clamp(max=clip_rho), ir.clamp(max=clip_c), ir.clamp(max=clip_pg)
    disc = gamma * (~term).float()
    vs = torch.zeros(B, T)
    pg = torch.zeros(B, T)
    acc = torch.zeros(B)
    for t in range(T - 1, -1, -1):
        cut = done[:, t] | (t + 1 >= T)
        vnext_in = v[:, t + 1] + acc if t + 1 < T else nv[:, t]
        vs_next = torch.where(cut, nv[:, t], vnext_in)
        d = rho[:, t] * (r[:, t] + disc[:, t] * nv[:, t] - v[:, t])
        k = gamma * c[:, t] * (~done[:, t]).float()
        acc = d + k * acc
        vs[:, t] = v[:, t] + acc
        pg[:, t] = rpg[:, t] * (r[:, t] + disc[:, t] * vs_next - v[:, t])
    return vs, pg
