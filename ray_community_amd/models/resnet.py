"""ResNet-50 (v1.5 bottleneck layout) for the "TorchTrainer ResNet-50 DDP bf16" benchmark config.

Reference workload: ``release/nightly_tests/dataset/multi_node_train_benchmark.py:262-370``
(torchvision ``resnet50(weights=None)``, SGD lr 0.1 momentum 0.9, 224x224 images, img/s) and the
batch-inference / Serve ResNet workloads (``release/nightly_tests/dataset/gpu_batch_inference.py``,
``release/serve_tests/workloads/serve_resnet_benchmark.py``). torchvision is not installed here, so
the network is defined directly (same layer structure and parameter count: 25.56 M).

MI355X layout: activations are NHWC (``channels_last``) end to end so MIOpen picks its NHWC
implicit-GEMM convolutions on the matrix cores; compute in bf16 under autocast with fp32
parameters (the optimizer keeps fp32 state). Every BatchNorm with its ReLU (and the bottleneck's
residual add) is ONE fused gfx950 kernel chain (``ops.batch_norm_act``: 3 launches forward,
3 backward, NHWC 16-byte streams) instead of MIOpen BN + separate elementwise kernels; the
stem's uint8 -> normalised bf16 NHWC conversion is the HIP ``image_normalize`` kernel.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class BiasAct(nn.Module):
    """What a BatchNorm becomes after ``fold_batchnorm``: its scale lives in the preceding
    convolution's weights and its shift here, applied together with the residual add and the
    ReLU in ONE in-place NHWC pass over the convolution's output (``ops.affine_act_``), instead of
    MIOpen's separate bias kernel plus torch's add and ReLU passes."""

    def __init__(self, shift: torch.Tensor):
        super().__init__()
        c = shift.numel()
        stats = torch.zeros(4, c, dtype=torch.float32, device=shift.device)
        stats[2] = 1.0
        stats[3] = shift.float()
        self.register_buffer("stats", stats)

    def _apply(self, fn, recurse=True):  # .to(dtype) must not round the fp32 shift: follow the device only
        st = self.stats
        out = super()._apply(fn, recurse)
        self.stats = st.to(self.stats.device)
        return out

    def forward(self, x, residual=None, relu=True):
        if torch.is_grad_enabled() and (x.requires_grad or (residual is not None and residual.requires_grad)):
            y = x + self.stats[3].to(x.dtype).view(1, -1, 1, 1)
            if residual is not None:
                y = y + residual
            return F.relu(y) if relu else y
        return ops.affine_act_(x, self.stats, residual, relu)


# Folded inference graph, opt-in (RCA_RESNET_GEMM_1X1=1 or GEMM_1X1[0] = True): 1x1 stride-1
# convolutions whose shape the in-tree GEMM covers run as ONE kernel with the shift / residual /
# ReLU in its epilogue (ops.conv1x1_affine_act) instead of a MIOpen convolution + the BiasAct pass.
# Off by default: the bs-256 forward measured 7.79-7.85 ms with it against 7.48-7.51 ms without
# (same process, 3 interleaved rounds, profiles/resnet_infer_r5.md) -- the GEMM's pipeline is built
# for long K, and these convolutions have K = 128-2048 with short, wide outputs.
GEMM_1X1 = [os.environ.get("RCA_RESNET_GEMM_1X1", "0") == "1"]


def conv_act(conv: nn.Conv2d, bn, x, residual=None, relu=True):
    """``act(bn(conv(x)) [+ residual])``; a folded 1x1 convolution goes through the GEMM epilogue
    when the shapes allow it and no gradient is needed."""
    if (GEMM_1X1[0] and isinstance(bn, BiasAct) and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.groups == 1 and conv.bias is None
            and not (torch.is_grad_enabled() and (x.requires_grad or conv.weight.requires_grad))
            and ops.conv1x1_affine_act_supported(x, conv.weight)):
        return ops.conv1x1_affine_act(x, conv.weight, bn.stats[3], residual, relu)
    return bn_act(bn, conv(x), residual=residual, relu=relu)


def bn_act(bn: nn.BatchNorm2d, x, residual=None, relu=True):
    """``act(bn(x) [+ residual])`` through the fused NHWC kernels (training mode) with the
    module's own parameters and running statistics. After ``fold_batchnorm`` the BN is a
    ``BiasAct`` (scale folded into the conv weights, shift + residual + ReLU in one pass)."""
    if isinstance(bn, BiasAct):
        return bn(x, residual, relu)
    if isinstance(bn, nn.Identity):
        y = x if residual is None else x + residual
        return F.relu(y, inplace=True) if relu else y
    mom = bn.momentum
    if bn.training and bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
        if mom is None:  # cumulative moving average, as nn.BatchNorm2d
            mom = 1.0 / float(bn.num_batches_tracked)
    return ops.batch_norm_act(x, bn.weight, bn.bias, bn.running_mean if bn.track_running_stats else None,
                              bn.running_var if bn.track_running_stats else None,
                              training=bn.training or not bn.track_running_stats, momentum=mom or 0.0,
                              eps=bn.eps, residual=residual, relu=relu)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_ch: int, width: int, stride: int = 1):
        super().__init__()
        out_ch = width * self.expansion
        self.conv1 = nn.Conv2d(in_ch, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)  # v1.5: stride on the 3x3
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, out_ch, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_ch)
        self.down = None
        if stride != 1 or in_ch != out_ch:
            self.down = nn.Sequential(nn.Conv2d(in_ch, out_ch, 1, stride=stride, bias=False), nn.BatchNorm2d(out_ch))

    def forward(self, x):
        idt = x if self.down is None else conv_act(self.down[0], self.down[1], x, relu=False)
        y = conv_act(self.conv1, self.bn1, x)
        y = conv_act(self.conv2, self.bn2, y)
        return conv_act(self.conv3, self.bn3, y, residual=idt)  # relu(bn3(conv3(y)) + identity)


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1000, zero_init_residual: bool = False):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        blocks = []
        in_ch = 64
        for i, n in enumerate(layers):
            width = 64 * 2 ** i
            for j in range(n):
                blocks.append(Bottleneck(in_ch, width, stride=2 if (j == 0 and i > 0) else 1))
                in_ch = width * Bottleneck.expansion
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(in_ch, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def forward(self, x):
        x = bn_act(self.bn1, self.conv1(x))
        x = F.max_pool2d(x, 3, stride=2, padding=1)
        x = self.blocks(x)
        x = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        return self.fc(x)


def resnet50(num_classes: int = 1000, device=None, channels_last: bool = True, **kw) -> ResNet:
    m = ResNet((3, 4, 6, 3), num_classes=num_classes, **kw)
    if device is not None:
        m = m.to(device)
    if channels_last:
        m = m.to(memory_format=torch.channels_last)
    return m


@torch.no_grad()
def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d):
    """(bias-free conv with the BN scale folded into its weights, fp32 per-channel shift)."""
    scale = bn.weight.float() / torch.sqrt(bn.running_var.float() + bn.eps)
    fused = nn.Conv2d(conv.in_channels, conv.out_channels, conv.kernel_size, stride=conv.stride,
                      padding=conv.padding, dilation=conv.dilation, groups=conv.groups, bias=False)
    fused = fused.to(device=conv.weight.device, dtype=conv.weight.dtype)
    fused.weight.copy_((conv.weight.float() * scale.view(-1, 1, 1, 1)).to(conv.weight.dtype))
    b0 = conv.bias.float() if conv.bias is not None else torch.zeros_like(bn.running_mean, dtype=torch.float32)
    shift = (b0 - bn.running_mean.float()) * scale + bn.bias.float()
    fused = fused.to(memory_format=torch.channels_last) if conv.weight.is_contiguous(
        memory_format=torch.channels_last) else fused
    return fused, shift


def fold_batchnorm(model: ResNet) -> ResNet:
    """Inference graph: every eval-mode BatchNorm folded into the preceding convolution
    (``w' = w * gamma / sqrt(var + eps)``, shift ``b' = (b - mean) * gamma / sqrt(var + eps) + beta``),
    so a serving replica runs a bias-free conv, then shift + residual add + ReLU in one NHWC pass
    (``BiasAct``). Returns the model, modified in place and switched to eval mode.

    (Measured, 1x MI355X, bf16 batch 256: with the shift as the conv's bias the forward took
    9.8 ms, 5.3 ms of it in three separate elementwise passes -- MIOpen's bias add, torch's
    ReLU and residual add; ``profiles/resnet_infer_r5.md``.)"""
    model.eval()
    model.conv1, shift = _fold(model.conv1, model.bn1)
    model.bn1 = BiasAct(shift)
    for blk in model.blocks:
        for i in (1, 2, 3):
            conv, shift = _fold(getattr(blk, f"conv{i}"), getattr(blk, f"bn{i}"))
            setattr(blk, f"conv{i}", conv)
            setattr(blk, f"bn{i}", BiasAct(shift))
        if blk.down is not None:
            conv, shift = _fold(blk.down[0], blk.down[1])
            blk.down = nn.Sequential(conv, BiasAct(shift))
    return model


def resnet_flops_per_image(image_size: int = 224) -> float:
    """Forward multiply-add FLOPs (x2) of ResNet-50 at 224x224: 4.09 GMAC -> 8.2 GFLOP."""
    return 2 * 4.09e9 * (image_size / 224) ** 2
