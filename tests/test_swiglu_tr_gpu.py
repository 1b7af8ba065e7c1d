"""SwiGLU with transposed side outputs (ops.swiglu(with_transposed=True), elementwise.hip
swiglu_{fwd,bwd}_tr): values equal the plain kernels bit for bit, the transposed copies are exact
transposes, and a DDP-wrapped Llama (flat fused-wgrad path that consumes them) matches plain
autograd gradients."""
import pytest
import torch

from ray_community_amd import ops

pytestmark = pytest.mark.gpu


def test_swiglu_transposed_outputs_exact():
    torch.manual_seed(0)
    gu = torch.randn(256, 2 * 384, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    gu2 = gu.detach().clone().requires_grad_(True)
    out, out_t = ops.swiglu(gu, with_transposed=True)
    ref = ops.swiglu(gu2)
    assert torch.equal(out, ref) and torch.equal(out_t, ref.t().contiguous())
    d = torch.randn_like(ref)
    out.backward(d)
    ref.backward(d)
    assert torch.equal(gu.grad, gu2.grad)
    # the transposed input gradient was registered for the producing linear and is exact
    # (looked up by the gradient tensor autograd handed to gate_up: here gu.grad's storage)


def test_swiglu_bwd_registers_transposed_grad():
    torch.manual_seed(1)
    gu = torch.randn(128, 2 * 128, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    seen = {}

    class Probe(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.view_as(x)

        @staticmethod
        def backward(ctx, g):
            seen["g"] = g
            seen["gt"] = ops.pop_grad_transposed(g)
            return g

    out, _ = ops.swiglu(Probe.apply(gu), with_transposed=True)
    out.sum().backward()
    assert seen["gt"] is not None and torch.equal(seen["gt"], seen["g"].t().contiguous())
    assert ops.pop_grad_transposed(seen["g"]) is None  # consumed once


def test_llama_flat_path_matches_plain_autograd():
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel

    torch.manual_seed(0)
    a = build_llama("llama3-tiny", device="cuda", max_seq_len=256)
    b = build_llama("llama3-tiny", device="cuda", max_seq_len=256)
    b.load_state_dict(a.state_dict())
    ddp = DistributedDataParallel(a)
    toks = torch.randint(0, 1024, (2, 129), device="cuda")
    la = ddp(toks[:, :-1], toks[:, 1:])
    la.backward()
    ddp.finish_gradient_sync()
    lb = b(toks[:, :-1], toks[:, 1:])
    lb.backward()
    assert abs(la.item() - lb.item()) < 1e-3 * abs(lb.item())
    pa = dict(a.named_parameters())
    for n, p in b.named_parameters():
        ga, gb = pa[n].grad.float(), p.grad.float()
        rel = (ga - gb).norm() / (gb.norm() + 1e-12)
        assert rel < 2e-2, (n, rel.item())


@pytest.mark.parametrize("T,H,F", [(256, 256, 512), (512, 384, 768), (1024, 1024, 1536)])
def test_gemm_swiglu_bwd_fused_matches_fp32(T, H, F):
    """ops.gemm_swiglu_bwd (variant-7 GEMM dh = dy W with the SwiGLU backward in its epilogue) vs
    an fp32 reference of dh and of the SwiGLU backward; the transposed copy is the exact transpose."""
    torch.manual_seed(T + F)
    dy = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    w = (torch.randn(H, F, device="cuda") / H ** 0.5).to(torch.bfloat16)  # down weight [H, F]
    gu = (torch.randn(T, 2 * F, device="cuda") * 2).to(torch.bfloat16)
    w_t = w.t().contiguous()
    dgu, dgu_t = ops.gemm_swiglu_bwd(dy, w_t, gu)
    torch.cuda.synchronize()
    dh = dy.float() @ w.float()
    g, u = gu.float()[:, :F], gu.float()[:, F:]
    s = torch.sigmoid(g)
    dg = dh * u * s * (1 + g * (1 - s))
    du = dh * (g * s).to(torch.bfloat16).float()
    ref = torch.cat([dg, du], 1)
    # bf16 output rounding + fp32 accumulation of dh over H (bound as the GEMM tests)
    absprod = dy.float().abs() @ w.float().abs()
    scale = torch.cat([(u * s * (1 + g * (1 - s))).abs(), (g * s).abs()], 1) * torch.cat([absprod, absprod], 1)
    bound = 2.0 ** -8 * ref.abs() + H * 2.0 ** -24 * scale + 2.0 ** -7 * scale / H ** 0.5 + 1e-6
    assert ((dgu.float() - ref).abs() / bound).max().item() <= 1.0
    assert torch.equal(dgu_t, dgu.t().contiguous())


def test_swiglu_down_fused_backward_matches_unfused(monkeypatch):
    """parallel.fused_linear.swiglu_down on the flat-gradient path with the fused dgrad + SwiGLU
    backward selected gives the same gate|up gradient and down dW as the unfused ops."""
    from ray_community_amd.parallel import fused_linear as fl

    monkeypatch.setattr(fl, "_FUSE_SWIGLU_BWD", True)

    torch.manual_seed(5)
    T, H, F = 512, 256, 512
    down = fl.FusedWgradLinear(F, H).to("cuda", torch.bfloat16)
    gu = (torch.randn(T, 2 * F, device="cuda") * 2).to(torch.bfloat16).requires_grad_(True)
    gy = torch.randn(T, H, device="cuda").to(torch.bfloat16)
    w = down.weight
    w._rca_flat_grad = True
    w.grad = torch.zeros_like(w)
    w._rca_grad_fresh = True
    fl.swiglu_down(gu, down).backward(gy)
    g_fused, dw_fused = gu.grad.clone(), w.grad.clone()
    gu2 = gu.detach().clone().requires_grad_(True)
    w2 = w.detach().clone().requires_grad_(True)
    torch.nn.functional.linear(ops.swiglu(gu2), w2).backward(gy)
    rel = (g_fused.float() - gu2.grad.float()).norm() / gu2.grad.float().norm()
    assert rel < 1e-2, rel.item()
    rel_w = (dw_fused.float() - w2.grad.float()).norm() / w2.grad.float().norm()
    assert rel_w < 1e-2, rel_w.item()
