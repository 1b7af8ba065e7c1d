"""Fused crop/resize/flip/normalise (ops/csrc/image.hip) against the fp32 torch reference, and the
Data UDFs that drive it (boxes inside images, deterministic seeds, CPU path through map_batches)."""
import numpy as np
import pytest
import torch

from ray_community_amd import ops
from ray_community_amd.data.gpu import CenterCropResize, RandomResizedCropFlipNormalize, random_resized_crop_boxes


def _imgs(N=5, H=37, W=53, C=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (N, H, W, C), dtype=torch.uint8, generator=g)


def test_boxes_inside_images_and_seeded():
    b1 = random_resized_crop_boxes([100] * 64, [80] * 64, np.random.default_rng(3))
    b2 = random_resized_crop_boxes([100] * 64, [80] * 64, np.random.default_rng(3))
    assert (b1 == b2).all()
    assert (b1[:, 0] >= 0).all() and (b1[:, 1] >= 0).all() and (b1[:, 0] + b1[:, 2] <= 100).all()
    assert (b1[:, 1] + b1[:, 3] <= 80).all() and (b1[:, 2] > 0).all()
    with pytest.raises(ValueError):
        ops.crop_resize_normalize(_imgs(1), [[0, 0, 50, 10]], (8, 8))


def test_udfs_cpu_path_shapes():
    batch = {"image": _imgs(4, 40, 60).numpy(), "label": np.arange(4)}
    out = RandomResizedCropFlipNormalize(size=16, seed=0, dtype="float32")(batch)
    assert out["image"].shape == (4, 3, 16, 16) and out["image"].dtype == np.float32
    out = CenterCropResize(size=16, resize=18, dtype="float32")(batch)
    assert out["image"].shape == (4, 3, 16, 16)
    # identity box + no flip at the source size == plain normalisation
    x = _imgs(2, 8, 8)
    y = ops.crop_resize_normalize(x, [[0, 0, 8, 8]] * 2, (8, 8), None, dtype=torch.float32)
    ref = ops.reference.image_normalize_ref(x, (0.485, 0.456, 0.406), (0.229, 0.224, 0.225), torch.float32)
    assert torch.allclose(y, ref, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,channels_last", [(torch.float32, False), (torch.bfloat16, False),
                                                 (torch.bfloat16, True)])
def test_crop_resize_normalize_gpu_matches_fp32(dtype, channels_last):
    x = _imgs(6, 45, 61, 3, seed=1)
    boxes = random_resized_crop_boxes([45] * 6, [61] * 6, np.random.default_rng(0))
    boxes[0] = (0, 0, 45, 61)  # full image (downscale)
    boxes[1] = (3, 4, 7, 9)    # small box (upscale)
    flips = np.array([0, 1, 0, 1, 1, 0], dtype=np.uint8)
    ref = ops.reference.crop_resize_normalize_ref(x, torch.as_tensor(boxes), flips, (24, 32),
                                                  (0.485, 0.456, 0.406), (0.229, 0.224, 0.225))
    got = ops.crop_resize_normalize(x.cuda(), boxes, (24, 32), flips, dtype=dtype, channels_last=channels_last)
    assert got.shape == (6, 3, 24, 32)
    if channels_last:
        assert got.is_contiguous(memory_format=torch.channels_last)
    tol = 2e-4 if dtype == torch.float32 else 2e-2
    assert (got.float().cpu() - ref).abs().max().item() < tol
