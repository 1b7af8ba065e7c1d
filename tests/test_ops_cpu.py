"""CPU-path tests of the ops / model / flat optimizer (reference math)."""
import torch

from ray_community_amd import ops
from ray_community_amd.ops import reference as ref


def test_gae_cpu_matches_reference():
    torch.manual_seed(0)
    B, T = 4, 50
    rew, val = torch.randn(B, T), torch.randn(B, T)
    term = torch.rand(B, T) < 0.1
    done = term | (torch.rand(B, T) < 0.05)
    last = torch.randn(B)
    a, t = ops.compute_gae(rew, val, term, done, 0.9, 0.8, last_values=last)
    ar, tr = ref.gae_ref(rew, val, term, done, 0.9, 0.8, last_values=last)
    assert torch.allclose(a, ar, atol=1e-5) and torch.allclose(t, tr, atol=1e-5)


def test_flat_adamw_matches_torch_adamw():
    from ray_community_amd.parallel import FlatAdamW, FlatParameters

    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 2))
    m2 = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Linear(16, 2))
    m2.load_state_dict(m1.state_dict())
    flat = FlatParameters(m1)
    opt = FlatAdamW(flat, lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None)
    topt = torch.optim.AdamW(m2.parameters(), lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0)
    x = torch.randn(32, 8)
    for _ in range(5):
        m1(x).pow(2).mean().backward()
        opt.step()
        opt.zero_grad()
        topt.zero_grad()
        m2(x).pow(2).mean().backward()
        topt.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.allclose(a, b, atol=1e-5)


def test_llama_tiny_cpu_forward_backward():
    from ray_community_amd.models import build_llama

    net = build_llama("llama3-tiny", dtype=torch.float32)
    toks = torch.randint(0, 1024, (2, 17))
    loss = net(toks[:, :-1], toks[:, 1:])
    assert torch.isfinite(loss) and 5.0 < loss.item() < 9.0
    loss.backward()
    assert all(p.grad is not None for p in net.parameters())
    logits = net(toks[:, :-1])
    assert logits.shape == (2, 16, 1024)


def test_swiglu_rope_cpu_shapes():
    gu = torch.randn(5, 16)
    assert ops.swiglu(gu).shape == (5, 8)
    cs = ops.rope_cos_sin(32, 16)
    qkv = torch.randn(8, (2 + 2) * 16)
    out = ops.apply_rope_(qkv, cs, 8, 2, 1, 16)
    assert out.shape == qkv.shape
    # v heads untouched, position-0 rows unchanged
    assert torch.equal(out[:, 3 * 16:], qkv[:, 3 * 16:])
    assert torch.allclose(out[0], qkv[0])


def test_attention_reference_matches_sdpa():
    import torch.nn.functional as F

    from ray_community_amd import ops
    from ray_community_amd.ops import reference as ref

    B, S, Hq, Hk, D = 2, 64, 4, 2, 32
    q = torch.randn(B, S, Hq, D)
    k = torch.randn(B, S, Hk, D)
    v = torch.randn(B, S, Hk, D)
    o = ref.attention_ref(q, k, v, True)
    kk = k.repeat_interleave(2, dim=2)
    vv = v.repeat_interleave(2, dim=2)
    o2 = F.scaled_dot_product_attention(q.transpose(1, 2), kk.transpose(1, 2), vv.transpose(1, 2), is_causal=True)
    assert torch.allclose(o, o2.transpose(1, 2), atol=1e-5)
    # CPU tensors take the reference path of the public op
    assert torch.allclose(ops.flash_attention(q, k, v, True), o)
    qkv = torch.cat([q.reshape(B * S, -1), k.reshape(B * S, -1), v.reshape(B * S, -1)], dim=1)
    assert torch.allclose(ops.flash_attention_qkv(qkv, B, S, Hq, Hk, D), o.reshape(B * S, -1), atol=1e-6)


def test_fused_wgrad_linear_matches_autograd_with_accumulation():
    import contextlib

    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    def run(fused):
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", device="cpu", dtype=torch.float32)
        if not fused:
            for m in net.modules():
                if getattr(getattr(m, "weight", None), "_rca_fused_wgrad", False):
                    m.weight._rca_fused_wgrad = False
        ddp = DistributedDataParallel(net)
        assert (len(ddp.flat.fused) > 0) == fused
        opt = FlatAdamW(ddp.flat, lr=1e-3)
        torch.manual_seed(1)
        tok = torch.randint(0, net.cfg.vocab_size, (2, 33))
        losses = []
        for i in range(4):
            with ddp.no_sync() if i == 0 else contextlib.nullcontext():
                loss = ddp(tok[:, :-1], tok[:, 1:])
                loss.backward()
            if i == 0:
                continue
            ddp.finish_gradient_sync()
            opt.step()
            opt.zero_grad()
            losses.append(loss.item())
        return losses, ddp.flat.data.clone()

    (la, da), (lb, db) = run(True), run(False)
    assert la == lb
    assert torch.equal(da, db)


def test_flat_sgd_matches_torch_sgd():
    import copy

    import torch.nn.functional as F

    from ray_community_amd.models.resnet import ResNet
    from ray_community_amd.parallel import DistributedDataParallel, FlatSGD

    torch.manual_seed(0)
    a = ResNet((1, 1, 1, 1), num_classes=5)
    b = copy.deepcopy(a)
    ddp = DistributedDataParallel(a)
    fopt = FlatSGD(ddp.flat, lr=0.05, momentum=0.9)
    topt = torch.optim.SGD(b.parameters(), lr=0.05, momentum=0.9)
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 5, (4,))
    for _ in range(3):
        F.cross_entropy(ddp(x), y).backward()
        fopt.step(ddp.grad_scale)
        fopt.zero_grad()
        F.cross_entropy(b(x), y).backward()
        topt.step()
        topt.zero_grad()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-5, rtol=1e-4), n


def test_flat_sgd_state_dict_roundtrip():
    """Resume: a fresh FlatSGD restored from a state_dict continues exactly like the original."""
    import copy

    import torch.nn.functional as F

    from ray_community_amd.models.resnet import ResNet
    from ray_community_amd.parallel import DistributedDataParallel, FlatSGD

    torch.manual_seed(0)
    a = ResNet((1, 1, 1, 1), num_classes=5)
    b = copy.deepcopy(a)
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 5, (4,))
    da = DistributedDataParallel(a)
    oa = FlatSGD(da.flat, lr=0.05, momentum=0.9, nesterov=True)
    for _ in range(2):
        F.cross_entropy(da(x), y).backward()
        oa.step(da.grad_scale)
        oa.zero_grad()
    sd = copy.deepcopy(oa.state_dict())
    b.load_state_dict(a.state_dict())
    db = DistributedDataParallel(b)
    ob = FlatSGD(db.flat, lr=0.05, momentum=0.9, nesterov=True)
    ob.load_state_dict(sd)
    assert ob.step_count == 2 and torch.equal(ob.buf, oa.buf)
    for d, o in ((da, oa), (db, ob)):
        F.cross_entropy(d(x), y).backward()
        o.step(d.grad_scale)
        o.zero_grad()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(pa, pb), n


def test_split_master_roundtrip_is_exact():
    """fp32 master <-> (bf16 high half, low 16 bits): bit-exact, including exact rounding ties,
    negatives, zeros and subnormals; the high half is the RNE bf16 except at ties (<= 1 ulp)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1 << 16, generator=g) * torch.logspace(-30, 30, 1 << 16)
    bits = x.view(torch.int32)
    ties = (bits & ~0xFFFF) | 0x8000  # exact half-way cases
    specials = torch.tensor([0.0, -0.0, 1e-40, -1e-40, 1.0, -1.0, 3.0e38, -3.0e38])
    for t in (x, ties.view(torch.float32), specials):
        hi, lo = ref.split_master(t)
        assert hi.dtype == torch.bfloat16 and lo.dtype == torch.int16
        back = ref.join_master(hi, lo)
        assert torch.equal(back.view(torch.int32), t.contiguous().view(torch.int32))
        d = (hi.view(torch.int16).to(torch.int32) - t.to(torch.bfloat16).view(torch.int16).to(torch.int32)).abs()
        assert int(d.max()) <= 1


def test_flat_adamw_split_master_matches_fp32_master():
    """The split master format (GPU default for bf16 models) follows the fp32-master trajectory
    bit-exactly (reference math on CPU; the HIP kernel is checked on the GPU)."""
    from ray_community_amd.parallel import FlatAdamW
    from ray_community_amd.parallel.flat import FlatParameters

    outs = []
    for fmt in ("fp32", "split"):
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(33, 17), torch.nn.Linear(17, 5)).to(torch.bfloat16)
        flat = FlatParameters(net)
        opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5, master_format=fmt)
        assert opt.split_master == (fmt == "split")
        g = torch.Generator().manual_seed(1)
        for _ in range(4):
            flat.grad.copy_(torch.randn(flat.numel, generator=g).to(torch.bfloat16))
            opt.step(0.5)
        outs.append((opt.master.clone(), opt.m.clone(), flat.data.clone()))
        sd = opt.state_dict()
        opt.load_state_dict(sd)
        assert torch.equal(opt.master, outs[-1][0])
    (m32, mm32, w32), (ms, mms, ws) = outs
    assert torch.equal(m32, ms) and torch.equal(mm32, mms)
    dw = (w32.view(torch.int16).to(torch.int32) - ws.view(torch.int16).to(torch.int32)).abs()
    assert int(dw.max()) <= 1  # model weights: RNE vs half-up only at exact ties
