"""Fused linear + cross-entropy (parallel/fused_linear.py, ops/csrc/loss_optim.hip ce_fused):
loss, dh and dW against the plain fp32 PyTorch reference, chunked, with ignored labels, and the
dW landing in a flat fused-wgrad gradient view."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(h, w, labels, ignore_index=-100):
    hf = h.detach().float().requires_grad_(True)
    wf = w.detach().float().requires_grad_(True)
    loss = F.cross_entropy(hf @ wf.t(), labels, ignore_index=ignore_index)
    loss.backward()
    return loss.detach(), hf.grad, wf.grad


@pytest.mark.parametrize("T,H,V,chunk", [(512, 256, 32000, 128), (256, 512, 128256, 0), (384, 256, 1024, 256)])
def test_linear_cross_entropy_matches_fp32(T, H, V, chunk):
    from ray_community_amd.parallel.fused_linear import linear_cross_entropy

    torch.manual_seed(0)
    h = (torch.randn(T, H, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(V, H, device="cuda") * 0.05).to(torch.bfloat16).requires_grad_(True)
    labels = torch.randint(0, V, (T,), device="cuda")
    labels[::7] = -100
    loss = linear_cross_entropy(h, w, labels, chunk_tokens=chunk)
    (loss * 2.0).backward()  # non-unit upstream gradient exercises the backward scaling
    rl, rh, rw = _ref(h, w, labels)
    assert abs(loss.item() - rl.item()) < 2e-2 * abs(rl.item()) + 1e-3
    for got, ref in ((h.grad, 2 * rh), (w.grad, 2 * rw)):
        err = (got.float() - ref).abs().max().item()
        assert err < 0.03 * ref.abs().max().item() + 1e-5, err


def test_linear_cross_entropy_into_flat_grad_view():
    from ray_community_amd.parallel import DistributedDataParallel
    from ray_community_amd.parallel.fused_linear import FusedWgradLinear, linear_cross_entropy

    torch.manual_seed(1)
    T, H, V = 256, 256, 4096
    lm = FusedWgradLinear(H, V).to("cuda", torch.bfloat16)
    ddp = DistributedDataParallel(lm)  # flat buffers, fused-wgrad views
    assert getattr(lm.weight, "_rca_flat_grad", False)
    h = (torch.randn(T, H, device="cuda") * 0.5).to(torch.bfloat16)
    labels = torch.randint(0, V, (T,), device="cuda")
    _, _, rw = _ref(h, lm.weight, labels)
    for acc in range(2):  # second pass accumulates into the view
        linear_cross_entropy(h, lm.weight, labels, chunk_tokens=64).backward()
        err = (lm.weight.grad.float() - (acc + 1) * rw).abs().max().item()
        assert err < 0.03 * rw.abs().max().item() * (acc + 1), err
    ddp.zero_grad()


@pytest.mark.parametrize("tied", [False, True])
def test_llama_fused_ce_matches_unfused(tied):
    """Same weights and tokens: the fused lm_head + CE path gives the loss and gradients of the
    materialised-logits path (DDP flat buffers, fused-wgrad lm_head)."""
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel

    toks = torch.randint(0, 1024, (2, 129), device="cuda")
    grads = []
    for fused in (False, True):
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", device="cuda", fused_ce=fused, ce_chunk=64, tie_embeddings=tied)
        ddp = DistributedDataParallel(net)
        loss = ddp(toks[:, :-1], toks[:, 1:])
        loss.backward()
        ddp.finish_gradient_sync()
        grads.append((loss.item(), ddp.flat.grad.float().clone()))
    (l0, g0), (l1, g1) = grads
    assert abs(l0 - l1) < 1e-2 * abs(l0)
    rel = (g0 - g1).norm() / g0.norm()
    assert rel < 0.02, rel.item()
