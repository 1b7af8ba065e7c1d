"""Model-level CPU checks (no GPU)."""
import torch


def test_resnet_fold_batchnorm_matches_eval():
    from ray_community_amd.models.resnet import ResNet, fold_batchnorm

    torch.manual_seed(0)
    m = ResNet((1, 1, 1, 1), num_classes=10)
    # non-trivial running statistics and affine params
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.5, 0.5)
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
    m.eval()
    x = torch.randn(2, 3, 64, 64)
    with torch.no_grad():
        ref = m(x)
        out = fold_batchnorm(m)(x)
    assert not any(isinstance(mod, torch.nn.BatchNorm2d) for mod in m.modules())
    torch.testing.assert_close(out, ref, atol=1e-4, rtol=1e-4)
