"""gfx950 flash attention (ops/csrc/attention.hip) vs a plain fp32 PyTorch reference."""
import pytest
import torch

from ray_community_amd import ops
from ray_community_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _mk(B, S, H, D, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)


def _err(a, b):
    return ((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6)).item()


@pytest.mark.parametrize("B,S,Hq,Hk,D,causal", [
    (2, 256, 4, 2, 128, True),
    (1, 384, 4, 4, 128, False),
    (1, 256, 8, 2, 64, True),
    (2, 128, 2, 1, 64, False),
])
def test_flash_attention_fwd_bwd(B, S, Hq, Hk, D, causal):
    q, k, v = _mk(B, S, Hq, D, 1), _mk(B, S, Hk, D, 2), _mk(B, S, Hk, D, 3)
    do = _mk(B, S, Hq, D, 4)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    o_ref = ref.attention_ref(qr, kr, vr, causal)
    o_ref.backward(do.float())
    q.requires_grad_(True)
    k.requires_grad_(True)
    v.requires_grad_(True)
    o = ops.flash_attention(q, k, v, causal)
    o.backward(do)
    torch.cuda.synchronize()
    assert _err(o, o_ref) < 2e-2
    assert _err(q.grad, qr.grad) < 3e-2
    assert _err(k.grad, kr.grad) < 3e-2
    assert _err(v.grad, vr.grad) < 3e-2


def test_flash_attention_qkv_matches_split():
    B, S, Hq, Hk, D = 2, 256, 8, 2, 128
    g = torch.Generator(device="cuda").manual_seed(7)
    qkv = torch.randn(B * S, (Hq + 2 * Hk) * D, device="cuda", dtype=torch.bfloat16, generator=g, requires_grad=True)
    o = ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D, causal=True)
    do = torch.randn_like(o)
    o.backward(do)
    x = qkv.detach().float().requires_grad_(True)
    q = x[:, : Hq * D].view(B, S, Hq, D)
    k = x[:, Hq * D: (Hq + Hk) * D].view(B, S, Hk, D)
    v = x[:, (Hq + Hk) * D:].view(B, S, Hk, D)
    o_ref = ref.attention_ref(q, k, v, True).reshape(B * S, Hq * D)
    o_ref.backward(do.float())
    assert _err(o, o_ref) < 2e-2
    assert _err(qkv.grad, x.grad) < 3e-2


def test_flash_attention_long_causal_rows():
    # a 4096-token causal row exercises the online-softmax rescale over 64 key tiles
    B, S, Hq, Hk, D = 1, 4096, 2, 1, 128
    q, k, v = _mk(B, S, Hq, D, 11), _mk(B, S, Hk, D, 12), _mk(B, S, Hk, D, 13)
    o = ops.flash_attention(q, k, v, True)
    o_ref = ref.attention_ref(q, k, v, True)
    assert _err(o, o_ref) < 2e-2


# Shapes of the production path: B*Hk a multiple of 8 takes the XCD-grouped workgroup order of
# xcd_group_map (ops/csrc/common.h) in the fwd, dQ and dK/dV kernels -- the Llama-3-8B bench
# shape is (B=2, S=4096, Hq=32, Hk=8, D=128), B*Hk = 16. dK/dV runs its default 64-row
# pipelined-slice variant (RCA_ATTN_DKDV_NH unset).
@pytest.mark.parametrize("B,S,Hq,Hk,D,causal", [
    (2, 1024, 32, 8, 128, True),
    (2, 1024, 32, 8, 128, False),
    (1, 4096, 32, 8, 128, True),
    (2, 512, 16, 8, 64, True),
    (1, 1024, 32, 8, 64, False),
])
def test_flash_attention_xcd_grouped_fwd_bwd(B, S, Hq, Hk, D, causal):
    assert (B * Hk) % 8 == 0
    q, k, v = _mk(B, S, Hq, D, 21), _mk(B, S, Hk, D, 22), _mk(B, S, Hk, D, 23)
    do = _mk(B, S, Hq, D, 24)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    o_ref = ref.attention_ref(qr, kr, vr, causal)
    o_ref.backward(do.float())
    o_ref = o_ref.detach()
    q.requires_grad_(True)
    k.requires_grad_(True)
    v.requires_grad_(True)
    o = ops.flash_attention(q, k, v, causal)
    o.backward(do)
    torch.cuda.synchronize()
    assert _err(o, o_ref) < 2e-2
    assert _err(q.grad, qr.grad) < 3e-2
    assert _err(k.grad, kr.grad) < 3e-2
    assert _err(v.grad, vr.grad) < 3e-2
    # every (batch, kv-head) group is covered: no head left unwritten
    assert torch.isfinite(q.grad).all() and k.grad.float().abs().amax(dim=(1, 3)).min() > 0


@pytest.mark.parametrize("B,S,Hq,Hk,D", [(2, 128, 4, 2, 64), (2, 1024, 32, 8, 128), (1, 512, 16, 8, 64)])
def test_flash_attention_bitwise_deterministic(B, S, Hq, Hk, D):
    """Forward and backward are bitwise reproducible run to run (no float atomics, no hazards):
    an inline-asm v_max3 that read the S^T MFMA accumulators without the MFMA->VALU wait states
    once made the forward's row max (and so the output rounding) timing dependent."""
    q, k, v = _mk(B, S, Hq, D, 31), _mk(B, S, Hk, D, 32), _mk(B, S, Hk, D, 33)
    do = _mk(B, S, Hq, D, 34)
    runs = []
    for _ in range(4):
        qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
        o = ops.flash_attention(qq, kk, vv, True)
        o.backward(do)
        runs.append((o.detach(), qq.grad, kk.grad, vv.grad))
    torch.cuda.synchronize()
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("B,S,Hq,Hk,causal", [(2, 256, 4, 2, True), (1, 384, 4, 4, False), (1, 512, 8, 2, True),
                                              (2, 256, 8, 1, False)])
def test_dkdv_hand_scheduled_matches_compiler_scheduled(B, S, Hq, Hk, causal, mode):
    """The hand-scheduled dK/dV kernel (RCA_ATTN_DKDV=hs) computes the same products in the same
    order as the compiler-scheduled one: dK and dV agree to bf16 rounding, dQ is untouched."""
    D = 128
    q, k, v = _mk(B, S, Hq, D, 11), _mk(B, S, Hk, D, 12), _mk(B, S, Hk, D, 13)
    do = _mk(B, S, Hq, D, 14)
    lib = ops._lib.lib()
    grads = []
    prev_bwd = lib.rca_attn_set_bwd_mode(0)  # the recompute path: the dkdv selector applies there
    try:
        for hs in (0, mode):
            prev = lib.rca_attn_set_dkdv_hs(hs)
            try:
                qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
                ops.flash_attention(qq, kk, vv, causal).backward(do)
                torch.cuda.synchronize()
            finally:
                lib.rca_attn_set_dkdv_hs(prev)
            grads.append((qq.grad, kk.grad, vv.grad))
    finally:
        lib.rca_attn_set_bwd_mode(prev_bwd)
    (q0, k0, v0), (q1, k1, v1) = grads
    assert torch.equal(q0, q1)
    assert _err(k1, k0) < 1e-2 and _err(v1, v0) < 1e-2, (_err(k1, k0), _err(v1, v0))


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("B,S,Hq,Hk,causal", [(2, 256, 4, 2, True), (1, 512, 4, 4, False), (1, 1024, 8, 2, True),
                                              (2, 768, 8, 1, False), (1, 4096, 2, 1, True)])
def test_fwd_variants_match_reference_and_default(B, S, Hq, Hk, causal, mode):
    """The opt-in forward variants (1: 64 rows per wave, attention_fwd_wide.hip; 2: the hand-scheduled
    64-row kernel, attention_fwd_hs.hip) against the fp32 reference and the default kernel; the backward runs from
    their O and LSE, so the grads are checked too."""
    D = 128
    q, k, v = _mk(B, S, Hq, D, 41), _mk(B, S, Hk, D, 42), _mk(B, S, Hk, D, 43)
    do = _mk(B, S, Hq, D, 44)
    lib = ops._lib.lib()
    outs = []
    for m in (0, mode):
        prev = lib.rca_attn_set_fwd_mode(m)
        try:
            qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
            o = ops.flash_attention(qq, kk, vv, causal)
            o.backward(do)
            torch.cuda.synchronize()
        finally:
            lib.rca_attn_set_fwd_mode(prev)
        outs.append((o.detach(), qq.grad, kk.grad, vv.grad))
    o_ref = ref.attention_ref(q.float(), k.float(), v.float(), causal)
    assert _err(outs[1][0], o_ref) < 2e-2
    for a, b in zip(outs[1], outs[0]):
        assert _err(a, b) < 1e-2, _err(a, b)


@pytest.mark.parametrize("mode", [0, 2])
@pytest.mark.parametrize("causal", [True, False])
def test_fwd_large_logits_rescale(causal, mode):
    """Scores spanning hundreds of log2 units: every deferred-rescale branch fires and a wrong row
    max would overflow exp2 (inf / NaN) -- checked for the default and the hand-scheduled forward."""
    B, S, Hq, Hk, D = 1, 1024, 4, 2, 128
    q, k, v = _mk(B, S, Hq, D, 51) * 6, _mk(B, S, Hk, D, 52) * 6, _mk(B, S, Hk, D, 53)
    lib = ops._lib.lib()
    prev = lib.rca_attn_set_fwd_mode(mode)
    try:
        o = ops.flash_attention(q, k, v, causal)
        torch.cuda.synchronize()
    finally:
        lib.rca_attn_set_fwd_mode(prev)
    o_ref = ref.attention_ref(q.float(), k.float(), v.float(), causal)
    assert torch.isfinite(o.float()).all()
    assert _err(o, o_ref) < 2e-2


def _bwd(q, k, v, do, causal, mode):
    lib = ops._lib.lib()
    prev = lib.rca_attn_set_bwd_mode(mode)
    try:
        qq, kk, vv = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
        o = ops.flash_attention(qq, kk, vv, causal)
        o.backward(do)
        torch.cuda.synchronize()
    finally:
        lib.rca_attn_set_bwd_mode(prev)
    return o.detach(), qq.grad, kk.grad, vv.grad


@pytest.mark.parametrize("B,S,Hq,Hk,causal", [(2, 256, 4, 2, True), (1, 384, 4, 4, False), (1, 1024, 8, 2, True),
                                              (2, 1024, 32, 8, True), (2, 512, 32, 8, False), (1, 4096, 8, 8, True)])
def test_recompute_free_dq_matches_reference_and_recompute_path(B, S, Hq, Hk, causal):
    """Backward mode 1 (default, D = 128): the dK/dV kernel stores the bf16 dS tiles and dQ = dS.K is
    read back from them (attention_dq.hip). Against the fp32 reference, and against mode 0 (the dQ
    kernel that recomputes S, P and dP) to bf16 rounding: dK and dV come from the same hand-scheduled
    products, but delta = rowsum(dO * O) is summed in a different order by the two paths."""
    D = 128
    q, k, v = _mk(B, S, Hq, D, 61), _mk(B, S, Hk, D, 62), _mk(B, S, Hk, D, 63)
    do = _mk(B, S, Hq, D, 64)
    assert ops._lib.lib().rca_attn_bwd_ws_bytes(B, S, Hq, Hk, D, int(causal)) > 0
    o1, dq1, dk1, dv1 = _bwd(q, k, v, do, causal, 1)
    o0, dq0, dk0, dv0 = _bwd(q, k, v, do, causal, 0)
    assert torch.equal(o1, o0)
    assert _err(dk1, dk0) < 1e-2 and _err(dv1, dv0) < 1e-2, (_err(dk1, dk0), _err(dv1, dv0))
    assert _err(dq1, dq0) < 1e-2, _err(dq1, dq0)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref.attention_ref(qr, kr, vr, causal).backward(do.float())
    assert _err(dq1, qr.grad) < 3e-2 and _err(dk1, kr.grad) < 3e-2 and _err(dv1, vr.grad) < 3e-2
    assert torch.isfinite(dq1).all() and dq1.float().abs().amax(dim=(1, 3)).min() > 0


def test_ds_workspace_cap_falls_back_to_recompute():
    """A dS workspace over the cap is never allocated: the backward runs the O(S) recompute path
    and its gradients match mode 0's exactly (same kernels) and the workspace path's to rounding."""
    B, S, Hq, Hk, D = 1, 2048, 16, 4, 128
    need = ops._lib.lib().rca_attn_bwd_ws_bytes(B, S, Hq, Hk, D, 1)
    assert need > 0
    q, k, v = _mk(B, S, Hq, D, 81), _mk(B, S, Hk, D, 82), _mk(B, S, Hk, D, 83)
    do = _mk(B, S, Hq, D, 84)
    ws_run = _bwd(q, k, v, do, True, 1)
    old = ops.set_attn_ds_workspace_cap(need - 1)
    try:
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        capped = _bwd(q, k, v, do, True, 1)
        peak = torch.cuda.max_memory_allocated() - base
    finally:
        ops.set_attn_ds_workspace_cap(old)
    recompute = _bwd(q, k, v, do, True, 0)
    for a, b in zip(capped, recompute):
        assert torch.equal(a, b)
    assert peak < need  # the workspace was not taken
    for a, b in zip(capped[1:], ws_run[1:]):
        assert _err(a, b) < 1e-2
    assert ops.attn_ds_workspace_cap() >= 1 << 30  # default policy: GBs on a 288 GB device


def test_recompute_free_dq_large_logits_and_determinism():
    """Scores spanning hundreds of log2 units (P saturates to 0/1 across tiles) through the dS-tile
    path, and bitwise run-to-run reproducibility of dQ (each element summed by one wave, in key order)."""
    B, S, Hq, Hk, D = 1, 2048, 8, 2, 128
    q, k, v = _mk(B, S, Hq, D, 71) * 6, _mk(B, S, Hk, D, 72) * 6, _mk(B, S, Hk, D, 73)
    do = _mk(B, S, Hq, D, 74)
    runs = [_bwd(q, k, v, do, True, 1) for _ in range(3)]
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)
    qr, kr, vr = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ref.attention_ref(qr, kr, vr, True).backward(do.float())
    _, dq, dk, dv = runs[0]
    assert torch.isfinite(dq).all()
    assert _err(dq, qr.grad) < 3e-2 and _err(dk, kr.grad) < 3e-2 and _err(dv, vr.grad) < 3e-2


@pytest.mark.parametrize("D", [128, 64])
@pytest.mark.parametrize("S,causal", [(256, True), (1024, True), (768, False), (4096, True)])
def test_forward_eight_wave_workgroup_is_bitwise_equal(S, causal, D):
    """The 8-wave forward (256 query rows per workgroup, K/V staged once for all 8 waves) runs the
    same per-wave schedule over the same tiles as the 4-wave form: bitwise equal O and LSE."""
    B, Hq, Hk = 1, 8, 2
    q, k, v = _mk(B, S, Hq, D, 91), _mk(B, S, Hk, D, 92), _mk(B, S, Hk, D, 93)
    lib = ops._lib.lib()
    prev = lib.rca_attn_set_fwd_nw(4)
    try:
        o4 = ops.flash_attention(q, k, v, causal)
        lib.rca_attn_set_fwd_nw(8)
        o8 = ops.flash_attention(q, k, v, causal)
    finally:
        lib.rca_attn_set_fwd_nw(prev)
    torch.cuda.synchronize()
    assert torch.equal(o4, o8)  # (S % 256 != 0 runs the 4-wave kernel in both)
    qr, kr, vr = (t.detach().float() for t in (q, k, v))
    assert _err(o8, ref.attention_ref(qr, kr, vr, causal)) < 2e-2


@pytest.mark.parametrize("S,causal", [(256, True), (1024, True), (2048, False), (4096, True)])
def test_dq_from_ds_two_blocks_per_wave_is_bitwise_equal(S, causal):
    """The dQ-from-dS kernel with 2 query blocks per wave (the K tile staged once for 256 query
    rows) sums every dQ element over the same tiles in the same key order as the 1-block variant:
    bitwise equal gradients, causal and not."""
    B, Hq, Hk, D = 1, 8, 2, 128
    q, k, v = _mk(B, S, Hq, D, 81), _mk(B, S, Hk, D, 82), _mk(B, S, Hk, D, 83)
    do = _mk(B, S, Hq, D, 84)
    lib = ops._lib.lib()
    prev = lib.rca_attn_set_dq_qw(1)
    try:
        a = _bwd(q, k, v, do, causal, 1)
        lib.rca_attn_set_dq_qw(2)
        b2 = _bwd(q, k, v, do, causal, 1)
    finally:
        lib.rca_attn_set_dq_qw(prev)
    for x, y in zip(a, b2):
        assert torch.equal(x, y)


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("B,S,Hq,Hk", [(2, 1024, 8, 2), (1, 512, 8, 8), (1, 768, 8, 1), (2, 2048, 32, 8)])
def test_ds_kernel_wait_state_variants_agree_bitwise(causal, B, S, Hq, Hk):
    """The dS-storing dK/dV kernel with 2 (s_nop 1) and 4 (s_nop 3) wait states ahead of each asm MFMA
    computes bit-identical gradients (a missing wait state shows up as stale MFMA operands), on the
    causal and full masks and MHA / GQA group sizes 1, 4 and 8 (the 8B bench's 32 q / 8 kv heads)."""
    D = 128
    q, k, v = _mk(B, S, Hq, D, 81), _mk(B, S, Hk, D, 82), _mk(B, S, Hk, D, 83)
    do = _mk(B, S, Hq, D, 84)
    lib = ops._lib.lib()
    outs = []
    for n in (3, 1):
        prev = lib.rca_attn_set_hs_nops(n)
        try:
            outs.append(_bwd(q, k, v, do, causal, 1))
        finally:
            lib.rca_attn_set_hs_nops(prev)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
