"""Numerics of the gfx950 HIP kernels against plain PyTorch fp32 references."""
import pytest
import torch

from ray_community_amd import ops
from ray_community_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=0.0, msg=""):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    assert bool((err <= tol).all()), f"{msg} max err {err.max().item():.4g}"


def test_kernel_library_loads():
    L = ops.lib()
    assert L.rca_rmsnorm_bwd_blocks(100, 4096) >= 1


@pytest.mark.parametrize("H,rows", [(512, 300), (1024, 300), (2048, 301), (4096, 300), (4096, 8203), (640, 300),
                                    (8192, 300)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_fwd_bwd(H, rows, with_res):
    torch.manual_seed(0)
    x = torch.randn(rows, H, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(rows, H, device=DEV, dtype=torch.bfloat16, requires_grad=True) if with_res else None
    out = ops.rms_norm(x, w, 1e-5, r)
    y, s = out if with_res else (out, None)
    # fp32 reference with autograd
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if with_res else None
    sr = xr + rr if with_res else xr
    yr = sr * torch.rsqrt(sr.pow(2).mean(-1, keepdim=True) + 1e-5) * wr
    _close(y, yr, atol=3e-2, rtol=2e-2, msg="y")
    if with_res:
        _close(s, sr, atol=2e-2, rtol=1e-2, msg="sum")
    gy = torch.randn_like(y)
    gs = torch.randn_like(y) if with_res else None
    if with_res:
        torch.autograd.backward([y, s], [gy, gs])
        torch.autograd.backward([yr, sr], [gy.float(), gs.float()])
    else:
        y.backward(gy)
        yr.backward(gy.float())
    _close(x.grad, xr.grad, atol=5e-2, rtol=3e-2, msg="dx")
    # dw sums `rows` terms whose bf16 roundings (s, s*rstd) the fp32 reference skips: that error
    # grows like sqrt(rows); the rounding-matched fp64 sum below pins the reduction itself
    _close(w.grad, wr.grad, atol=0.5 * max(1.0, (rows / 300) ** 0.5), rtol=3e-2, msg="dw")
    s16 = (x.detach().float() + r.detach().float()).bfloat16().float() if with_res else x.detach().float()
    rs = torch.rsqrt(s16.pow(2).mean(-1, keepdim=True) + 1e-5)
    dw_m = (gy.double() * (s16 * rs).bfloat16().double()).sum(0)
    _close(w.grad, dw_m.float(), atol=0.05, rtol=1e-2, msg="dw (rounding-matched)")
    if with_res:
        _close(r.grad, rr.grad, atol=5e-2, rtol=3e-2, msg="dres")


def test_swiglu():
    torch.manual_seed(0)
    T, F = 257, 1024
    gu = torch.randn(T, 2 * F, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    out = ops.swiglu(gu)
    gur = gu.detach().float().requires_grad_(True)
    outr = torch.nn.functional.silu(gur[:, :F]) * gur[:, F:]
    _close(out, outr, atol=3e-2, rtol=2e-2)
    g = torch.randn_like(out)
    out.backward(g)
    outr.backward(g.float())
    _close(gu.grad, gur.grad, atol=5e-2, rtol=3e-2)


def test_rope_inplace_fwd_bwd():
    torch.manual_seed(0)
    B, S, Hq, Hk, D = 2, 64, 4, 2, 128
    T = B * S
    cs = ops.rope_cos_sin(256, D, 500000.0).to(DEV)
    base = torch.randn(T, (Hq + 2 * Hk) * D, device=DEV, dtype=torch.bfloat16)
    x = base.clone().requires_grad_(True)
    y = x * 1.0  # non-leaf so the in-place op is legal
    out = ops.apply_rope_(y, cs, S, Hq, Hk, D)
    pos = torch.arange(T, device=DEV) % S
    xr = base.float().requires_grad_(True)
    n_rot = Hq + Hk
    rot = ref.rope_ref(xr[:, : n_rot * D].reshape(T, n_rot, D), cs, pos).reshape(T, -1)
    outr = torch.cat([rot, xr[:, n_rot * D:]], dim=1)
    _close(out, outr, atol=3e-2, rtol=2e-2)
    g = torch.randn_like(out)
    out.backward(g)
    outr.backward(g.float())
    _close(x.grad, xr.grad, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("T,S,Hq,Hk,with_pos", [(256, 128, 4, 2, False), (8192, 4096, 32, 8, False),
                                                (384, 384, 8, 8, True), (128, 64, 2, 1, False)])
def test_rope_backward_fused_with_transpose(T, S, Hq, Hk, with_pos):
    """rca_rope_bwd_tr: the RoPE backward (rotation by -theta of the q / k heads) and the transpose
    of the whole dqkv gradient in one pass, against the fp32 reference and the separate in-place
    kernel (within one bf16 rounding: the two may contract the mul/adds differently)."""
    from ray_community_amd.ops._lib import stream_ptr

    torch.manual_seed(3)
    D, n_rot = 128, Hq + Hk
    W = (Hq + 2 * Hk) * D
    cs = ops.rope_cos_sin(8192, D, 500000.0).to(DEV)
    g = torch.randn(T, W, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 8192, (T,), device=DEV, dtype=torch.int32) if with_pos else None
    L = ops.lib()
    g1, g1t = g.clone(), torch.empty(W, T, device=DEV, dtype=torch.bfloat16)
    assert L.rca_rope_bwd_tr(g1.data_ptr(), cs.data_ptr(), pos.data_ptr() if pos is not None else None,
                             g1t.data_ptr(), T, S, W, n_rot, stream_ptr(g.device)) == 0
    g2 = g.clone()
    assert L.rca_rope(g2.data_ptr(), cs.data_ptr(), pos.data_ptr() if pos is not None else None, T, S, n_rot, W,
                      D, 1, stream_ptr(g.device)) == 0
    torch.cuda.synchronize()
    assert torch.equal(g1t, g1.t())  # the transposed copy is exactly the rotated gradient
    assert torch.equal(g1[:, n_rot * D:], g[:, n_rot * D:])  # v heads untouched
    ulps = (g1.view(torch.int16).int() - g2.view(torch.int16).int()).abs()
    assert int(ulps.max()) <= 1
    # fp32 reference: rotation by -theta = rotation with sin negated
    p = pos.long() if pos is not None else torch.arange(T, device=DEV) % S
    csn = cs.clone()
    csn[..., 1] = -csn[..., 1]
    rot = ref.rope_ref(g[:, : n_rot * D].float().reshape(T, n_rot, D), csn, p).reshape(T, -1)
    _close(g1[:, : n_rot * D], rot, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("V", [128256, 1000, 1003])
def test_cross_entropy(V):
    torch.manual_seed(0)
    T = 67
    logits = (3 * torch.randn(T, V, device=DEV)).to(torch.bfloat16).requires_grad_(True)
    labels = torch.randint(0, V, (T,), device=DEV)
    labels[3] = -100
    loss = ops.cross_entropy(logits, labels)
    lr = logits.detach().float().requires_grad_(True)
    lossr = torch.nn.functional.cross_entropy(lr, labels, ignore_index=-100)
    assert abs(loss.item() - lossr.item()) < 2e-3 * max(1.0, abs(lossr.item()))
    loss.backward()
    lossr.backward()
    _close(logits.grad, lr.grad, atol=2e-4, rtol=2e-2)


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_adamw_flat(gdt):
    from ray_community_amd.parallel import FlatAdamW, FlatParameters

    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(64, 129), torch.nn.LayerNorm(129), torch.nn.Linear(129, 3)).to(DEV)
    m = m.to(torch.bfloat16)
    flat = FlatParameters(m, grad_dtype=gdt)
    opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
    master0 = opt.master.clone()
    for _ in range(3):
        flat.grad.copy_(torch.randn_like(flat.grad, dtype=torch.float32).to(gdt))
        g = flat.grad.clone()
        # reference on a CPU copy
        opt_ref_master = opt.master.detach().cpu().clone()
        mr, vr = opt.m.cpu().clone(), opt.v.cpu().clone()
        opt.step(grad_scale=0.5)
        nrm = g.float().pow(2).sum().sqrt().item() * 0.5
        coef = min(1.0, 0.5 / (nrm + 1e-6))
        t = opt.step_count
        for s, e, wd in [(0, flat.decay_end, 0.1), (flat.decay_end, flat.numel, 0.0)]:
            ref.adamw_ref(opt_ref_master[s:e], g[s:e].cpu(), mr[s:e], vr[s:e], 1e-2, 0.9, 0.95, 1e-8, wd, t,
                          grad_mul=0.5, clip=coef)
        _close(opt.master, opt_ref_master, atol=1e-5, rtol=1e-5)
        # the bf16 model weights are the rounded fp32 master weights (split master: half-up at
        # exact ties instead of RNE, <= 1 ulp)
        d = flat.data.view(torch.int16).int() - opt.master.to(torch.bfloat16).view(torch.int16).int()
        assert int(d.abs().max()) <= 1
    assert not torch.equal(master0, opt.master)


def test_grad_sumsq():
    xs = [torch.randn(1000, device=DEV, dtype=torch.bfloat16), torch.randn(77, device=DEV)]
    s = ops.grad_sumsq(xs)
    r = sum(x.float().pow(2).sum() for x in xs)
    assert abs(s.item() - r.item()) < 1e-3 * r.item()


def test_grad_sumsq_last_block_finalize_many_launches():
    """The last-block-done finalize (no separate reduce launch): sizes from one block to the
    1024-block cap, bf16 and fp32, accumulate chains, and bitwise run-to-run determinism over
    repeated launches on the same workspace (the ticket word must come back to zero)."""
    torch.manual_seed(1)
    sizes = [1, 7, 2048, 2049, 262_144 * 8 + 3, 64 << 20]
    xs = [torch.randn(n, device=DEV, dtype=torch.bfloat16 if i % 2 == 0 else torch.float32)
          for i, n in enumerate(sizes)]
    ref_ = sum(x.double().pow(2).sum() for x in xs).item()
    first = ops.grad_sumsq(xs).clone()
    assert abs(first.item() - ref_) < 1e-4 * ref_
    for _ in range(20):
        again = ops.grad_sumsq(xs)
        assert torch.equal(again, first)
    ws = ops._workspace(xs[0].device, "sumsq", ops.SUMSQ_WS)
    torch.cuda.synchronize()
    assert int(ws[1024:1025].view(torch.int32).item()) == 0


@pytest.mark.parametrize("B,T", [(1, 1000), (64, 128), (5, 63), (3, 1)])
def test_gae(B, T):
    torch.manual_seed(0)
    rew = torch.randn(B, T)
    val = torch.randn(B, T)
    term = torch.rand(B, T) < 0.05
    done = term | (torch.rand(B, T) < 0.03)
    last = torch.randn(B)
    adv_r, tgt_r = ref.gae_ref(rew, val, term, done, 0.99, 0.95, last_values=last)
    adv, tgt = ops.compute_gae(rew.to(DEV), val.to(DEV), term.to(DEV), done.to(DEV), 0.99, 0.95, last_values=last.to(DEV))
    _close(adv, adv_r, atol=1e-4, rtol=1e-4)
    _close(tgt, tgt_r, atol=1e-4, rtol=1e-4)
    adv_s, _ = ops.compute_gae(rew.to(DEV), val.to(DEV), term.to(DEV), done.to(DEV), 0.99, 0.95,
                               last_values=last.to(DEV), standardize=True)
    if B * T > 1:
        expect = (adv_r - adv_r.mean()) / (adv_r.std(unbiased=False) + 1e-4)
        _close(adv_s, expect, atol=1e-3, rtol=1e-3)


def test_standardize():
    x = torch.randn(100003, device=DEV) * 3 + 2
    e = (x - x.mean()) / (x.std(unbiased=False) + 1e-4)
    ops.standardize_(x)
    _close(x, e, atol=1e-4, rtol=1e-4)


def test_batched_concat():
    ts = [torch.randn(n, 33, device=DEV) for n in (1, 7, 1000, 0, 5)]
    out = ops.batched_concat(ts)
    assert torch.equal(out, torch.cat(ts))
    ts8 = [torch.randint(0, 255, (n, 3), device=DEV, dtype=torch.uint8) for n in (3, 5)]
    assert torch.equal(ops.batched_concat(ts8), torch.cat(ts8))


def test_image_normalize():
    u8 = torch.randint(0, 256, (4, 17, 19, 3), dtype=torch.uint8)
    out = ops.image_normalize(u8.to(DEV), dtype=torch.float32)
    r = ref.image_normalize_ref(u8, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), torch.float32)
    _close(out, r, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("shape", [(4, 17, 19, 3), (2, 224, 224, 3), (3, 5, 7, 4), (1, 3, 3, 1)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_image_normalize_channels_last(shape, dtype):
    u8 = torch.randint(0, 256, shape, dtype=torch.uint8)
    out = ops.image_normalize(u8.to(DEV), dtype=dtype, channels_last=True, mean=(0.4, 0.5, 0.6, 0.3)[: shape[3]],
                              std=(0.2, 0.25, 0.3, 0.5)[: shape[3]])
    assert out.shape == (shape[0], shape[3], shape[1], shape[2])
    assert out.is_contiguous(memory_format=torch.channels_last) or shape[3] == 1
    r = ref.image_normalize_ref(u8, (0.4, 0.5, 0.6, 0.3)[: shape[3]], (0.2, 0.25, 0.3, 0.5)[: shape[3]], torch.float32)
    _close(out, r, atol=1e-5 if dtype == torch.float32 else 2e-2, rtol=1e-5 if dtype == torch.float32 else 1e-2)


@pytest.mark.parametrize("relu,with_res", [(True, False), (False, False), (True, True)])
def test_affine_act_inplace_matches_fp32(relu, with_res):
    torch.manual_seed(0)
    for C in (64, 256, 2048):
        x = torch.randn(3, C, 7, 9, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        res = torch.randn_like(x) if with_res else None
        stats = torch.zeros(4, C, device=DEV)
        stats[2] = torch.rand(C, device=DEV) + 0.5
        stats[3] = torch.randn(C, device=DEV)
        want = x.float() * stats[2].view(1, -1, 1, 1) + stats[3].view(1, -1, 1, 1)
        if with_res:
            want = want + res.float()
        if relu:
            want = torch.relu(want)
        ptr = x.data_ptr()
        out = ops.affine_act_(x, stats, res, relu)
        assert out.data_ptr() == ptr  # in place
        _close(out, want, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("N,Cin,Cout,HW", [(2, 128, 256, 16), (4, 512, 2048, 7), (1, 1024, 256, 16)])
@pytest.mark.parametrize("with_res,relu", [(False, True), (True, True), (False, False)])
def test_conv1x1_affine_act_matches_fp32(N, Cin, Cout, HW, with_res, relu):
    torch.manual_seed(0)
    x = torch.randn(N, Cin, HW, HW, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, Cin, 1, 1, device=DEV) / Cin ** 0.5).to(torch.bfloat16)
    shift = torch.randn(Cout, device=DEV)
    res = torch.randn(N, Cout, HW, HW, device=DEV).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last) if with_res else None
    if not ops.conv1x1_affine_act_supported(x, w):
        pytest.skip("M = N*H*W not a multiple of 256")
    out = ops.conv1x1_affine_act(x, w, shift, res, relu)
    assert out.is_contiguous(memory_format=torch.channels_last) and out.shape == (N, Cout, HW, HW)
    want = torch.nn.functional.conv2d(x.float(), w.float()) + shift.view(1, -1, 1, 1)
    if with_res:
        want = want + res.float()
    if relu:
        want = torch.relu(want)
    _close(out, want, atol=3e-2, rtol=2e-2)


def test_folded_resnet50_inference_matches_fp32():
    """Serving graph (BN folded, shift + residual + ReLU in one NHWC pass per conv) in bf16 against
    the unfolded fp32 eval-mode network."""
    from ray_community_amd.models.resnet import BiasAct, fold_batchnorm, resnet50

    torch.manual_seed(0)
    ref = resnet50(num_classes=10).to(DEV).eval()
    for m in ref.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 1.5)
            m.weight.data.uniform_(0.5, 1.2)
            m.bias.data.uniform_(-0.1, 0.1)
    x = torch.randn(4, 3, 96, 96, device=DEV).contiguous(memory_format=torch.channels_last)
    with torch.no_grad():
        want = ref(x)
        import copy

        net = fold_batchnorm(copy.deepcopy(ref)).to(torch.bfloat16)
        assert isinstance(net.blocks[0].bn3, BiasAct) and net.blocks[0].bn3.stats.dtype == torch.float32
        from ray_community_amd.models import resnet as R

        got = net(x.to(torch.bfloat16)).float()  # MIOpen convolutions + the BiasAct pass (default)
        R.GEMM_1X1[0] = True
        try:
            got_gemm = net(x.to(torch.bfloat16)).float()  # 1x1 convolutions on the GEMM epilogue where covered
        finally:
            R.GEMM_1X1[0] = False
    for g in (got, got_gemm):
        err = (g - want).abs().max() / want.abs().max()
        assert err < 5e-2, float(err)


def test_resnet50_train_step_gpu():
    from ray_community_amd.train.vision import build_resnet_training

    net, ddp, opt, batch, step = build_resnet_training(batch_size=32, image_size=64, num_classes=10, lr=1e-3)
    data = batch()
    w0 = net.fc.weight.detach().clone()
    losses = [float(step(*data)) for _ in range(4)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert not torch.equal(w0, net.fc.weight)


def test_llama_tiny_train_step_gpu():
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    torch.manual_seed(0)
    net = build_llama("llama3-tiny", device=DEV)
    ddp = DistributedDataParallel(net)
    opt = FlatAdamW(ddp.flat, lr=1e-3)
    toks = torch.randint(0, 1024, (2, 65), device=DEV)
    losses = []
    for _ in range(8):
        loss = ddp(toks[:, :-1], toks[:, 1:])
        loss.backward()
        ddp.finish_gradient_sync()
        opt.step(ddp.grad_scale)
        opt.zero_grad()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


def test_llama_hip_matches_reference_path():
    """Same weights: GPU (HIP kernels) loss/grads vs the CPU fp32 reference path."""
    from ray_community_amd.models import build_llama

    torch.manual_seed(0)
    net = build_llama("llama3-tiny", device="cpu", dtype=torch.float32)
    toks = torch.randint(0, 1024, (2, 33))
    loss_cpu = net(toks[:, :-1], toks[:, 1:])
    loss_cpu.backward()
    g_cpu = {n: p.grad.clone() for n, p in net.named_parameters()}
    net.zero_grad()
    gnet = net.to(DEV, torch.bfloat16)
    loss_gpu = gnet(toks[:, :-1].to(DEV), toks[:, 1:].to(DEV))
    loss_gpu.backward()
    assert abs(loss_gpu.item() - loss_cpu.item()) < 2e-2 * abs(loss_cpu.item())
    for n, p in gnet.named_parameters():
        a, b = p.grad.float().cpu(), g_cpu[n]
        rel = (a - b).norm() / (b.norm() + 1e-8)
        assert rel < 0.1, (n, rel.item())


def test_vtrace_kernel_matches_reference():
    from ray_community_amd.ops import reference as ref

    torch.manual_seed(3)
    B, T = 37, 203
    lr = 0.5 * torch.randn(B, T)
    r, v, nv = torch.randn(B, T), torch.randn(B, T), torch.randn(B, T)
    term = torch.rand(B, T) < 0.03
    done = term | (torch.rand(B, T) < 0.02)
    vs_r, pg_r = ref.vtrace_ref(lr, r, v, nv, term, done, 0.97, 1.0, 0.9, 1.0)
    vs, pg = ops.vtrace(lr.cuda(), r.cuda(), v.cuda(), nv.cuda(), term.cuda(), done.cuda(), 0.97, 1.0, 0.9, 1.0)
    assert torch.allclose(vs.cpu(), vs_r, atol=1e-4, rtol=1e-4)
    assert torch.allclose(pg.cpu(), pg_r, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("clip", [None, 0.5])
def test_sharded_adamw_matches_flat_adamw_gpu(clip):
    """world=1 ZeRO optimizer path (per-bucket chunks, HIP AdamW per chunk) == the flat AdamW path,
    fed identical gradients (the model's backward has atomics, so grads are fed, not recomputed)."""
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW, ShardedAdamW, ShardedDataParallel

    torch.manual_seed(0)
    w1 = DistributedDataParallel(build_llama("llama3-tiny", device=DEV), bucket_cap_mb=0.2)
    torch.manual_seed(0)
    w2 = ShardedDataParallel(build_llama("llama3-tiny", device=DEV), bucket_cap_mb=0.2)
    assert w1.flat.offsets == w2.flat.offsets and len(w2.flat.buckets) > 2
    o1 = FlatAdamW(w1.flat, lr=1e-3, max_grad_norm=clip)
    o2 = ShardedAdamW(w2, lr=1e-3, max_grad_norm=clip)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    for _ in range(3):
        grad = torch.randn(w1.flat.numel, device=DEV, generator=g).to(torch.bfloat16) * 0.01
        w1.flat.grad.copy_(grad)
        w2.flat.grad.copy_(grad)
        o1.step(1.0)
        o2.step(1.0)
    torch.cuda.synchronize()
    a, b = w1.flat.data.float(), w2.flat.data.float()
    if clip is None:
        assert torch.equal(a, b)
    else:  # only the grad-norm reduction order differs (chunk list vs whole buffer)
        assert torch.allclose(a, b, atol=1e-5, rtol=8e-3), (a - b).abs().max()


def test_zero_side_stream_weight_transposes_track_updates():
    """ZeRO's W^T copies (transposed on a side stream by the forward pre-hook) equal W^T after every
    optimizer update, and the gradients match the in-line-transpose path (``_module_wt`` cleared)."""
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import ShardedAdamW, ShardedDataParallel

    runs = []
    for side in (True, False):
        torch.manual_seed(0)
        m = ShardedDataParallel(build_llama("llama3-tiny", device=DEV), bucket_cap_mb=0.2)
        wts = [p for p in m.flat.fused if getattr(p, "_rca_wt", None) is not None]
        assert len(wts) >= 4 * 2  # qkv, o, gate_up, down per layer
        if not side:
            m._module_wt = {}
        opt = ShardedAdamW(m, lr=1e-2)
        g = torch.Generator(device=DEV)
        g.manual_seed(1)
        grads = []
        for step in range(3):
            tok = torch.randint(0, 1024, (2, 128), device=DEV, generator=g)
            loss = m(tok, labels=tok)
            if side:
                torch.cuda.synchronize()
                for p in wts:  # refreshed before the backward needs it, from the updated weights
                    assert p._rca_wt_ev is not None
                    assert torch.equal(p._rca_wt, p.detach().t())
            loss.backward()
            m.finish_gradient_sync()
            if side:
                assert all(p._rca_wt_ev is None for p in wts)  # every dgrad waited on its event
            grads.append(m.flat.grad.float().clone())
            opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        runs.append((grads, m.flat.data.float().clone()))
    for a, b in zip(runs[0][0], runs[1][0]):
        assert torch.allclose(a, b, atol=2e-3, rtol=2e-2), (a - b).abs().max()
    assert torch.allclose(runs[0][1], runs[1][1], atol=1e-3, rtol=1e-2)


@pytest.mark.parametrize("N,C,H,W", [(4, 64, 12, 10), (2, 256, 7, 7), (3, 2048, 3, 3), (2, 8, 5, 5), (1, 128, 1, 33)])
@pytest.mark.parametrize("relu,with_res", [(True, False), (True, True), (False, False), (False, True)])
def test_batch_norm_act_matches_fp32(N, C, H, W, relu, with_res):
    torch.manual_seed(0)
    x = (torch.randn(N, C, H, W, device=DEV) * 3 + 5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn(N, C, H, W, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last) \
        if with_res else None
    w = (torch.rand(C, device=DEV) + 0.5).requires_grad_()
    b = torch.randn(C, device=DEV).requires_grad_()
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    xk = x.clone().requires_grad_()
    rk = res.clone().requires_grad_() if with_res else None
    out = ops.batch_norm_act(xk, w, b, rm, rv, training=True, momentum=0.1, eps=1e-5, residual=rk, relu=relu)
    assert out.dtype == torch.bfloat16 and out.is_contiguous(memory_format=torch.channels_last)
    # fp32 reference
    xr = x.float().requires_grad_()
    wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rmr, rvr = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    rr = res.float().requires_grad_() if with_res else None
    # plain-op reference (MIOpen's own fp32 NHWC batch_norm is not the thing under test)
    mu = xr.mean(dim=(0, 2, 3))
    var = xr.var(dim=(0, 2, 3), unbiased=False)
    z = (xr - mu.view(1, -1, 1, 1)) * torch.rsqrt(var.view(1, -1, 1, 1) + 1e-5) * wr.view(1, -1, 1, 1) \
        + br.view(1, -1, 1, 1)
    n = N * H * W
    rmr = 0.9 * rmr + 0.1 * mu.detach()
    rvr = 0.9 * rvr + 0.1 * var.detach() * (n / max(n - 1, 1))
    if with_res:
        z = z + rr
    _close(out, torch.relu(z) if relu else z, atol=3e-2, rtol=2e-2, msg="fwd")
    _close(rm, rmr, atol=1e-4, rtol=1e-4, msg="running_mean")
    _close(rv, rvr, atol=1e-3, rtol=1e-3, msg="running_var")
    gy = torch.randn(N, C, H, W, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out.backward(gy)
    # the reference backward uses the kernel's ReLU mask (taken from the bf16 output, as the kernel does)
    mask = (out.detach().float() > 0).float() if relu else 1.0
    (z * mask).backward(gy.float())
    _close(xk.grad, xr.grad, atol=3e-2, rtol=3e-2, msg="dx")
    _close(w.grad, wr.grad, atol=5e-2 * (N * H * W) ** 0.5, rtol=2e-2, msg="dgamma")
    _close(b.grad, br.grad, atol=5e-2 * (N * H * W) ** 0.5, rtol=2e-2, msg="dbeta")
    if with_res:
        _close(rk.grad, rr.grad, atol=3e-2, rtol=3e-2, msg="dres")


@pytest.mark.parametrize("R,C,pad", [(64, 64, 0), (256, 192, 0), (8192, 448, 64), (128, 4096, 8)])
def test_transpose_bf16(R, C, pad):
    torch.manual_seed(0)
    base = torch.randn(R, C + pad, device=DEV, dtype=torch.bfloat16)
    x = base[:, :C]
    out = ops.transpose(x)
    assert out.shape == (C, R) and out.is_contiguous()
    assert torch.equal(out, x.t().contiguous())


def test_fused_wgrad_linear_transposed_backward_matches_fp32():
    """dgrad/wgrad through the transposed-operand GEMMs vs an fp32 autograd reference."""
    from ray_community_amd.parallel.fused_linear import FusedWgradLinear

    torch.manual_seed(0)
    lin = FusedWgradLinear(256, 384, device=DEV, dtype=torch.bfloat16)
    x = torch.randn(2, 64, 256, device=DEV, dtype=torch.bfloat16, requires_grad=True)
    gy = torch.randn(2, 64, 384, device=DEV, dtype=torch.bfloat16)
    lin.weight._rca_flat_grad = True
    lin.weight.grad = torch.zeros_like(lin.weight)
    lin.weight._rca_grad_fresh = True
    lin(x).backward(gy)
    xr = x.detach().float().requires_grad_(True)
    wr = lin.weight.detach().float().requires_grad_(True)
    torch.nn.functional.linear(xr, wr).backward(gy.float())
    _close(x.grad, xr.grad, atol=0.15, rtol=2e-2, msg="dgrad")
    _close(lin.weight.grad, wr.grad, atol=0.15, rtol=2e-2, msg="wgrad")


def test_llama_8b_width_two_layers_matches_fp32_cpu():
    """Two decoder layers at Llama-3-8B width (H=4096, 32 q / 8 kv heads, FFN 14336, RoPE 5e5):
    the bf16 GPU path (HIP attention on its XCD-grouped branch, B*Hk=16; HIP RMSNorm/RoPE/SwiGLU/CE;
    fused-wgrad linears) vs the fp32 CPU reference path with the same weights."""
    from ray_community_amd.models import build_llama

    torch.manual_seed(0)
    net = build_llama("llama3-8b", device="cpu", dtype=torch.float32, num_layers=2, vocab_size=8192)
    assert net.cfg.hidden_size == 4096 and net.cfg.num_heads == 32 and net.cfg.num_kv_heads == 8
    toks = torch.randint(0, 8192, (2, 257))
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    loss_cpu = net(toks[:, :-1], toks[:, 1:])
    loss_cpu.backward()
    g_cpu = {n: p.grad.clone() for n, p in net.named_parameters()}
    net.zero_grad()
    gnet = net.to(DEV, torch.bfloat16)
    loss_gpu = gnet(toks[:, :-1].to(DEV), toks[:, 1:].to(DEV))
    loss_gpu.backward()
    torch.cuda.synchronize()
    assert abs(loss_gpu.item() - loss_cpu.item()) < 1e-2 * abs(loss_cpu.item())
    for n, p in gnet.named_parameters():
        a, b = p.grad.float().cpu(), g_cpu[n]
        rel = (a - b).norm() / (b.norm() + 1e-8)
        assert rel < 0.1, (n, rel.item())


def test_flat_adamw_overlapped_with_forward_matches_serial():
    """AdamW issued per bucket on a side stream, waited for by forward pre-hooks, gives exactly
    the serial update (fed identical gradients; forwards interleaved as in training). The forward
    outputs are compared with a tolerance: hipBLASLt's stream-K GEMMs are not bitwise
    reproducible run to run, while a forward that read pre-update weights (lr=5e-2) would be off
    by far more."""
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    nets, opts = [], []
    for overlap in (False, True):
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", device=DEV)
        ddp = DistributedDataParallel(net, bucket_cap_mb=0.2)
        opt = FlatAdamW(ddp.flat, lr=5e-2, max_grad_norm=0.5)
        if overlap:
            opt.overlap_with_forward(net)
            assert len(ddp.flat.buckets) > 2
        nets.append((net, ddp))
        opts.append(opt)
    g = torch.Generator(device=DEV)
    g.manual_seed(1)
    toks = torch.randint(0, 1024, (2, 128), device=DEV)
    for _ in range(3):
        grad = torch.randn(nets[0][1].flat.numel, device=DEV, generator=g).to(torch.bfloat16) * 0.01
        outs = []
        for (net, ddp), opt in zip(nets, opts):
            ddp.flat.grad.copy_(grad)
            opt.step(1.0)
            opt.zero_grad()
            with torch.no_grad():
                outs.append(net(toks).float())
        assert (outs[0] - outs[1]).abs().max().item() < 3e-2
    torch.cuda.synchronize()
    assert torch.equal(nets[0][1].flat.data, nets[1][1].flat.data)
    assert torch.equal(opts[0].m, opts[1].m) and torch.equal(opts[0].v, opts[1].v)
    fl = nets[1][1].flat
    assert fl.grad[fl.zero_start:].abs().max().item() == 0  # zeroed behind the update


def _gemm_excess(out, ref, absprod, K, base=None):
    """Largest ratio |out - ref| / bound over all elements (> 1 = outside the rounding model).
    Per element: the bf16 rounding of the stored result (<= 2^-9 relative, bound taken as 2^-8)
    plus fp32 accumulation over K (<= K * 2^-24 * sum_k |a||b|), plus the bf16 base it was added
    to in an accumulating epilogue; a wrong or missing K-slice moves an element by a whole
    slice's contribution, far above this."""
    exact = ref if base is None else ref + base
    bound = 2.0 ** -8 * exact.abs() + K * 2.0 ** -24 * absprod + 1e-6
    return ((out.float() - exact).abs() / bound).max().item()


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 512, 128), (512, 256, 192), (512, 768, 320),
                                   (1024, 512, 1024)])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(False, False), (False, True), (True, True), (True, False)])
@pytest.mark.parametrize("variant", [7, 6, 5, 3, 2, 0])
def test_gemm_bf16_all_layouts_match_fp32(M, N, K, a_kmaj, b_kmaj, variant):
    """ops.gemm (hand-written gfx950 MFMA GEMM, LDS-DMA staging, swizzled row / transposed-read
    operand images, XCD-grouped tile order) vs an fp32 torch reference, all four operand
    layouts, plain and accumulating epilogues; asymmetric operands (integer-valued rows/cols
    mixed with noise) so a transposed output or operand cannot pass."""
    torch.manual_seed(M + N + K)
    a = torch.randn(K, M, device=DEV) if a_kmaj else torch.randn(M, K, device=DEV)
    b = torch.randn(K, N, device=DEV) if b_kmaj else torch.randn(N, K, device=DEV)
    a = (a + torch.arange(a.shape[1], device=DEV) * 0.01).to(torch.bfloat16)
    b = (b - torch.arange(b.shape[0], device=DEV)[:, None] * 0.003).to(torch.bfloat16)
    af = a.float().t() if a_kmaj else a.float()
    bf = b.float() if b_kmaj else b.float().t()
    ref = af @ bf
    lib = ops._lib.lib()
    prev = lib.rca_gemm_set_variant(variant)
    try:
        out = ops.gemm(a, b, a_kmaj, b_kmaj)
        base = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        acc = base.clone()
        ops.gemm(a, b, a_kmaj, b_kmaj, out=acc, accumulate=True)
    finally:
        lib.rca_gemm_set_variant(prev)
    torch.cuda.synchronize()
    absprod = af.abs() @ bf.abs()
    assert _gemm_excess(out, ref, absprod, K) <= 1.0
    assert _gemm_excess(acc, ref, absprod, K, base.float()) <= 1.0


@pytest.mark.parametrize("M,N,K", [(1280, 768, 2048), (2048, 2304, 4096), (512, 256, 128)])
@pytest.mark.parametrize("variant", [6, 7])
def test_gemm_buffer_dma_tn_variants(M, N, K, variant):
    """Variants 6 (buffer-descriptor LDS-DMA, immediate-offset fragment reads, 4 slices per loop
    iteration) and 7 (64-deep tiles, full-cache-line DMA, buffer refilled two tiles ahead) on
    multi-tile k-contiguous shapes with many ring wraps (and the 2-tile minimum), plain and
    accumulating."""
    torch.manual_seed(M + K)
    a = (torch.randn(M, K, device=DEV) + torch.arange(K, device=DEV) * 1e-3).to(torch.bfloat16)
    b = (torch.randn(N, K, device=DEV) - torch.arange(N, device=DEV)[:, None] * 1e-3).to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    absprod = a.float().abs() @ b.float().abs().t()
    lib = ops._lib.lib()
    prev = lib.rca_gemm_set_variant(variant)
    try:
        out = ops.gemm(a, b)
        base = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        acc = base.clone()
        ops.gemm(a, b, out=acc, accumulate=True)
    finally:
        lib.rca_gemm_set_variant(prev)
    torch.cuda.synchronize()
    assert _gemm_excess(out, ref, absprod, K) <= 1.0
    assert _gemm_excess(acc, ref, absprod, K, base.float()) <= 1.0


@pytest.mark.parametrize("M,N,K", [(8192, 4096, 28672), (8192, 4096, 14336), (8192, 6144, 4096)])
def test_gemm_variant7_at_llama8b_shapes(M, N, K):
    """Variant 7 at the production shapes of the 8B step: the gate_up input gradient it runs in
    the step (8192 x 4096 x 28672, K = 2 x FFN), the down-projection reduction (K = 14336) and the
    qkv width, against fp32 with the per-element bound above (plain and accumulating)."""
    torch.manual_seed(K)
    a = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    b = (torch.randn(N, K, device=DEV) * 0.5 + torch.arange(N, device=DEV)[:, None] * 1e-4).to(torch.bfloat16)
    lib = ops._lib.lib()
    prev = lib.rca_gemm_set_variant(7)
    try:
        out = ops.gemm(a, b)
        base = torch.randn(M, N, device=DEV).to(torch.bfloat16)
        acc = base.clone()
        ops.gemm(a, b, out=acc, accumulate=True)
    finally:
        lib.rca_gemm_set_variant(prev)
    torch.cuda.synchronize()
    # reference in row blocks (fp32 operands of this size are 0.5-1 GB each)
    af, bf = a.float(), b.float()
    worst = 0.0
    for r in range(0, M, 2048):
        ref = af[r:r + 2048] @ bf.t()
        absprod = af[r:r + 2048].abs() @ bf.abs().t()
        worst = max(worst, _gemm_excess(out[r:r + 2048], ref, absprod, K),
                    _gemm_excess(acc[r:r + 2048], ref, absprod, K, base[r:r + 2048].float()))
    assert worst <= 1.0, worst


def test_gemm_check_catches_a_corrupted_k_slice():
    """The per-element bound above is tight enough to fail a kernel that drops K-tiles: variant 91
    (timing diagnostic: no LDS-DMA inside the K loop, so every tile after the first two re-reads
    stale LDS) is rejected on a shape where only a few of 16 K-tiles go wrong."""
    M, N, K = 512, 512, 1024
    torch.manual_seed(3)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    b = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    ref = a.float() @ b.float().t()
    absprod = a.float().abs() @ b.float().abs().t()
    lib = ops._lib.lib()
    prev = lib.rca_gemm_set_variant(3)
    try:
        assert _gemm_excess(ops.gemm(a, b), ref, absprod, K) <= 1.0
        lib.rca_gemm_set_variant(91)
        bad = ops.gemm(a, b)
    finally:
        lib.rca_gemm_set_variant(prev)
    torch.cuda.synchronize()
    assert _gemm_excess(bad, ref, absprod, K) > 10.0


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [8 * 4096 + 5, 1 << 20])
def test_adamw_split_master_kernel_matches_fp32_master(gdt, n):
    """rca_adamw_split (bf16 high half + 16 low bits) == rca_adamw with an fp32 master, bit for bit
    on master / m / v (the split format changes nothing in the math); the bf16 weights differ from
    RNE only at exact ties (<= 1 ulp); each step agrees with the fp32 PyTorch reference step
    (ops.reference.adamw_ref) to rounding."""
    from ray_community_amd.parallel import FlatAdamW
    from ray_community_amd.parallel.flat import FlatParameters

    res = []
    worst = 0
    for fmt in ("fp32", "split"):
        torch.manual_seed(0)
        net = torch.nn.Linear(n, 1, bias=False).to(device=DEV, dtype=torch.bfloat16)
        flat = FlatParameters(net, grad_dtype=gdt)
        opt = FlatAdamW(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=0.5, master_format=fmt)
        assert opt.split_master == (fmt == "split")
        g = torch.Generator(device=DEV).manual_seed(1)
        for _ in range(3):
            flat.grad.copy_(torch.randn(flat.numel, device=DEV, generator=g).to(gdt))
            p, mr, vr, gr = opt.master.clone(), opt.m.clone(), opt.v.clone(), flat.grad.float().clone()
            p_old = p.clone()
            opt.step(0.5)
            c = min(1.0, 0.5 / (float(gr.norm()) * 0.5 + 1e-6))
            for s, e, wd in ((0, flat.decay_end, 0.1), (flat.decay_end, flat.numel, 0.0)):
                if e > s:
                    ref.adamw_ref(p[s:e], gr[s:e], mr[s:e], vr[s:e], 1e-3, 0.9, 0.95, 1e-8, wd, opt.step_count,
                                  grad_mul=0.5, clip=c)
            # vs the fp32 PyTorch reference: same math, different rounding (fma contraction, the
            # grad-norm reduction order: ~1e-7 relative in the clip coefficient) -- amplified where
            # m's EMA cancels, so the bound is on the update's scale (lr), not on |p|'s ulp
            worst = max(worst, float(((opt.master - p).abs() - 1e-5 * p.abs()).max() / 1e-3))
        torch.cuda.synchronize()
        res.append((opt.master.clone(), opt.m.clone(), opt.v.clone(), flat.data.clone()))
    (p0, m0, v0, w0), (p1, m1, v1, w1) = res
    assert torch.equal(p0.view(torch.int32), p1.view(torch.int32))
    assert torch.equal(m0, m1) and torch.equal(v0, v1)
    dw = (w0.view(torch.int16).to(torch.int32) - w1.view(torch.int16).to(torch.int32)).abs()
    assert int(dw.max()) <= 1
    assert worst <= 1e-6, worst  # |err| <= 1e-5 |p| + 1e-9 (lr = 1e-3)


@pytest.mark.parametrize("gdt", [torch.bfloat16, torch.float32])
def test_adamw_segmented_with_transposed_weights_bitwise(gdt):
    """The segmented split-master AdamW (rca_adamw_split_seg: 64x64 matrix tiles that also write
    W^T, 1-D blocks for everything else) is bit-identical to the flat kernel on weights, low
    halves, m and v, across decay / no-decay params and odd-length tails; every fused-wgrad
    weight's W^T equals W.t() exactly after each step and the backward's weight_t() uses it."""
    from ray_community_amd.parallel import FlatAdamW
    from ray_community_amd.parallel.flat import FlatParameters
    from ray_community_amd.parallel.fused_linear import FusedWgradLinear, weight_t

    def build():
        torch.manual_seed(0)
        # (never run forward: only the parameter layout matters) a plain Linear first, so every
        # fused weight precedes it in the flat layout; FusedWgradLinear(37, 256) is a fused weight
        # whose shape is no 128-multiple (updated by 1-D tiles, no W^T; so is the 64 x 128 one)
        m = torch.nn.ModuleList([torch.nn.Linear(64, 37), torch.nn.LayerNorm(37), FusedWgradLinear(37, 256),
                                 FusedWgradLinear(256, 384), torch.nn.LayerNorm(384), FusedWgradLinear(384, 128),
                                 FusedWgradLinear(128, 256), FusedWgradLinear(128, 64)])
        return m.to(device=DEV, dtype=torch.bfloat16)

    runs = []
    for wt_on in (False, True):
        net = build()
        flat = FlatParameters(net, grad_dtype=gdt)
        opt = FlatAdamW(flat, lr=1e-2, weight_decay=0.1, max_grad_norm=0.5)
        opt.transposed_weights = wt_on
        g = torch.Generator(device=DEV).manual_seed(3)
        for _ in range(3):
            flat.grad.copy_(torch.randn(flat.numel, device=DEV, generator=g).to(gdt))
            opt.step(0.5)
            if wt_on:
                mats = [p for p in net.parameters() if getattr(p, "_rca_wt", None) is not None]
                # fp32 gradients: no flat-grad fused weights, so no W^T (all 1-D segments)
                assert len(mats) == (3 if gdt == torch.bfloat16 else 0)
                for p in mats:
                    assert torch.equal(p._rca_wt, p.detach().t())
                    assert weight_t(p).data_ptr() == p._rca_wt.data_ptr()
        torch.cuda.synchronize()
        runs.append((flat.data.clone(), opt.lo.clone(), opt.m.clone(), opt.v.clone()))
    for a, b in zip(*runs):
        assert torch.equal(a, b)
    # an in-place edit of a weight invalidates its W^T: weight_t() re-transposes
    net = build()
    flat = FlatParameters(net, grad_dtype=gdt)
    opt = FlatAdamW(flat, lr=1e-2)
    flat.grad.normal_()
    opt.step()
    w = net[3].weight
    with torch.no_grad():
        w.mul_(2.0)
    assert torch.equal(weight_t(w), w.detach().t())


@pytest.mark.parametrize("plan_shape", [(4096, 4096, 8192), (128256, 4096, 8192)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_plans_match_fp32(plan_shape, accumulate):
    """The measured per-shape weight-gradient plans (hand GEMM on natural layouts for o_proj,
    activation-only transpose for lm_head) vs an fp32 reference of dW = g^T x."""
    from ray_community_amd.parallel import fused_linear as fl

    N, K, T = plan_shape
    torch.manual_seed(N)
    g2 = torch.randn(T, N, device=DEV).to(torch.bfloat16)
    x2 = (torch.randn(T, K, device=DEV) + torch.arange(K, device=DEV) * 1e-3).to(torch.bfloat16)
    out = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    base = out.float().clone()
    assert fl._wgrad_plan(g2, x2, None, None, out) in ("hand", "trB")
    fl._wgrad(g2, x2, True, out=out, accumulate=accumulate)
    ref = g2.float().t() @ x2.float()
    absprod = g2.float().abs().t() @ x2.float().abs()
    assert _gemm_excess(out, ref, absprod, T, base if accumulate else None) <= 1.0


def test_rmsnorm_weight_grads_accumulated_into_flat_buffer_match_plain_autograd():
    """With flat gradient buffers + DDP grad-ready hooks the RMSNorm backward accumulates dw
    straight into the bf16 grad view (no dw tensor, no AccumulateGrad add); the result equals the
    plain-autograd gradient bit for bit and the bucket bookkeeping still counts the weight once."""
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel

    def run(use_ddp):
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", device=DEV)
        mod = DistributedDataParallel(net, precompute_grad_norm=True) if use_ddp else net
        toks = torch.randint(0, net.cfg.vocab_size, (2, 129), device=DEV, generator=torch.Generator(DEV).manual_seed(1))
        loss = mod(toks[:, :-1], toks[:, 1:])
        loss.backward()
        if use_ddp:
            mod.finish_gradient_sync()
            assert mod.flat.precomputed_sumsq is not None  # every bucket was counted
        return {n: p.grad.detach().clone() for n, p in net.named_parameters() if "norm" in n}

    plain, flat = run(False), run(True)
    assert plain.keys() == flat.keys() and len(plain) >= 3
    for k in plain:
        assert torch.equal(plain[k], flat[k]), k


def test_fused_embedding_grad_into_flat_buffer_matches_dense():
    """FusedEmbedding scatter-adds into the flat bf16 grad view (DDP hooks registered) and equals
    torch's dense embedding gradient; repeated token ids accumulate."""
    from ray_community_amd.parallel import DistributedDataParallel
    from ray_community_amd.parallel.fused_linear import FusedEmbedding

    torch.manual_seed(0)
    emb = FusedEmbedding(1000, 256).to(device=DEV, dtype=torch.bfloat16)
    ref = torch.nn.Embedding(1000, 256).to(device=DEV, dtype=torch.bfloat16)
    ref.weight.data.copy_(emb.weight.data)
    ddp = DistributedDataParallel(torch.nn.ModuleDict({"e": emb}), precompute_grad_norm=True)
    idx = torch.randint(0, 50, (4, 300), device=DEV)  # many repeats
    g = torch.randn(4, 300, 256, device=DEV, dtype=torch.bfloat16)
    emb(idx).backward(g)
    ddp.finish_gradient_sync()
    ref(idx).backward(g)
    assert emb.weight.grad.data_ptr() == ddp.flat.grad.data_ptr() + ddp.flat.param_offset[id(emb.weight)] * 2
    assert torch.equal(emb.weight.grad, ref.weight.grad)  # same fp32-accumulating kernel, one rounding
