"""Diagnose the recompute-free attention backward: decode the dS tiles the dK/dV kernel wrote and
compare them with an fp32 reference dS = P * (dP - delta), and the dQ kernel's output with
scale * dS . K computed from the decoded tiles.

    python scripts/diag/attn_ds_diag.py [S] [causal]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from ray_community_amd import ops  # noqa: E402
from ray_community_amd.ops._lib import stream_ptr  # noqa: E402


def decode_tiles(ws, B, Hq, S, causal):
    nb = S // 32
    tiles = nb * (nb + 1) // 2 if causal else nb * nb
    raw = ws[: B * Hq * tiles * 2048].view(torch.bfloat16).view(B * Hq, tiles, 2, 64, 8).float().cpu()
    # flat position (inside a tile's 1024 bf16) of element (query row, key column)
    pos = torch.zeros(32, 32, dtype=torch.long)
    for s in range(2):
        for lane in range(64):
            h = lane >> 5
            slot = lane ^ (4 * h + 8 * s)
            for j in range(8):
                r = 8 * s + j
                pos[(r & 3) + 8 * (r >> 2) + 4 * h, lane & 31] = (s * 64 + slot) * 8 + j
    flat = raw.reshape(B * Hq, tiles, 1024)
    out = torch.zeros(B * Hq, S, S)
    for qb in range(nb):
        for kb in range(nb):
            if causal and kb > qb:
                continue
            idx = qb * (qb + 1) // 2 + kb if causal else qb * nb + kb
            out[:, 32 * qb:32 * qb + 32, 32 * kb:32 * kb + 32] = flat[:, idx][:, pos]
    return out.view(B, Hq, S, S)


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    causal = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
    B, Hq, Hk, D = 1, 2, 1, 128
    scale = D ** -0.5
    g = torch.Generator(device="cuda").manual_seed(0)
    mk = lambda h: torch.randn(B, S, h, D, device="cuda", dtype=torch.bfloat16, generator=g)  # noqa: E731
    q, k, v, do = mk(Hq), mk(Hk), mk(Hk), mk(Hq)
    lib = ops._lib.lib()
    o = torch.empty(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, Hq, S, device="cuda", dtype=torch.float32)
    ops._attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, Hq, Hk, D,
                  q.stride(1), k.stride(1), v.stride(1), o.stride(1), scale, causal)
    nbytes = lib.rca_attn_bwd_ws_bytes(B, S, Hq, Hk, D, int(causal))
    ws = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    delta = torch.empty(B, Hq, S, device="cuda", dtype=torch.float32)
    st = (q.stride(1), k.stride(1), v.stride(1), o.stride(1), do.stride(1), dq.stride(1), dk.stride(1), dv.stride(1))
    rc = lib.rca_attn_bwd2(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), do.data_ptr(), lse.data_ptr(),
                           delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), B, S, Hq, Hk, D, *st, scale,
                           int(causal), ws.data_ptr(), nbytes, stream_ptr())
    torch.cuda.synchronize()
    print("rc", rc, "ws MB", nbytes / 1e6)
    # fp32 reference
    qf, kf, vf, dof = (t.float().permute(0, 2, 1, 3) for t in (q, k, v, do))  # [B, H, S, D]
    kf = kf.repeat_interleave(Hq // Hk, 1)
    vf = vf.repeat_interleave(Hq // Hk, 1)
    s_ = qf @ kf.transpose(-1, -2) * scale
    if causal:
        s_ = s_.masked_fill(torch.triu(torch.ones(S, S, device="cuda", dtype=torch.bool), 1), float("-inf"))
    p = torch.softmax(s_, -1)
    of = p @ vf
    dp = dof @ vf.transpose(-1, -2)
    dlt = (dof * of).sum(-1, keepdim=True)
    ds_ref = p * (dp - dlt)
    print("delta err", (delta - dlt.squeeze(-1)).abs().max().item(), "delta max", dlt.abs().max().item())
    ds_k = decode_tiles(ws, B, Hq, S, causal).cuda()
    err = (ds_k - ds_ref).abs()
    print("dS max err", err.max().item(), "dS max", ds_ref.abs().max().item())
    bad = (err > 0.02 * ds_ref.abs().max()).nonzero()
    print("bad elements", bad.shape[0])
    if bad.shape[0]:
        qs = sorted(set((bad[:, 2] // 32).tolist()))
        ks = sorted(set((bad[:, 3] // 32).tolist()))
        print("bad q blocks", qs[:20], "bad k blocks", ks[:20])
        print("first bad", bad[:8].tolist())
    dq_from_tiles = (ds_k @ kf) * scale  # [B, H, S, D]
    dq_k = dq.float().permute(0, 2, 1, 3)
    print("dQ vs dS_tiles.K", (dq_k - dq_from_tiles).abs().max().item(), "dQ max", dq_from_tiles.abs().max().item())
    dq_ref = (ds_ref @ kf) * scale
    print("dQ vs ref", (dq_k - dq_ref).abs().max().item())
    dk_ref = (ds_ref.transpose(-1, -2) @ qf * scale).view(B, Hk, Hq // Hk, S, D).sum(2)
    print("dK vs ref", (dk.float().permute(0, 2, 1, 3) - dk_ref).abs().max().item(), "dK max", dk_ref.abs().max().item())


if __name__ == "__main__":
    main()
