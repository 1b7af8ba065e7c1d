"""DistributedDataParallel(precompute_grad_norm=True): the per-bucket sums of squares taken on a
side stream during backward give the same clipped AdamW trajectory as the post-backward pass."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_precomputed_grad_norm_matches_post_backward():
    from ray_community_amd.models import build_llama
    from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW

    toks = torch.randint(0, 1024, (2, 129), device="cuda", generator=torch.Generator("cuda").manual_seed(1))
    outs, norms = [], []
    for pre in (False, True):
        torch.manual_seed(0)
        net = build_llama("llama3-tiny", device="cuda")
        ddp = DistributedDataParallel(net, bucket_cap_mb=0.5, precompute_grad_norm=pre)
        assert len(ddp.flat.buckets) > 2
        opt = FlatAdamW(ddp.flat, lr=1e-3, max_grad_norm=0.05)  # small: clipping is active
        opt.track_grad_norm = True
        for _ in range(3):
            loss = ddp(toks[:, :-1], toks[:, 1:])
            loss.backward()
            ddp.finish_gradient_sync()
            if pre:
                assert ddp.flat.precomputed_sumsq is not None
            opt.step(ddp.grad_scale)
            assert ddp.flat.precomputed_sumsq is None
            norms.append(opt.grad_norm())
            opt.zero_grad()
        torch.cuda.synchronize()
        outs.append(ddp.flat.data.float().clone())
    for a, b in zip(norms[:3], norms[3:]):
        assert abs(a - b) <= 1e-3 * a, (a, b)
    d = (outs[0] - outs[1]).abs()
    assert d.max() < 1e-2 and d.mean() < 1e-5
