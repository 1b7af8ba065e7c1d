"""GPU preprocessing UDFs for ``map_batches`` on MI355X (fused HIP kernels).

``ImageNormalize`` turns uint8 HWC image batches into normalised bf16/f32 NCHW tensors in HBM with
ONE gfx950 kernel (cast + scale + mean/std + layout transpose fused), the typical
"Data map_batches GPU preprocess -> model" hot path. Use it as a callable class so the pool
actors own a GPU:  ``ds.map_batches(ImageNormalize, num_gpus=1, concurrency=2, batch_format="numpy")``.
``RandomResizedCropFlipNormalize`` / ``CenterCropResize`` fuse crop + bilinear resize + flip +
normalise into one kernel (``ops.crop_resize_normalize``, ``ops/csrc/image.hip``).
"""
from __future__ import annotations

import numpy as np


class ImageNormalize:
    def __init__(self, column: str = "image", mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                 dtype: str = "bfloat16", keep_on_device: bool = False, channels_last: bool = False):
        import torch

        self.column = column
        self.mean = mean
        self.std = std
        self.dtype = getattr(torch, dtype)
        self.keep = keep_on_device
        self.channels_last = channels_last  # NCHW-logical tensor in NHWC memory (MIOpen NHWC convs)
        self.device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")

    def __call__(self, batch):
        import torch

        from ..ops import image_normalize

        x = torch.from_numpy(np.ascontiguousarray(batch[self.column])).to(self.device, non_blocking=True)
        y = image_normalize(x, self.mean, self.std, self.dtype, channels_last=self.channels_last)
        out = dict(batch)
        if self.keep:
            out[self.column] = y
        else:
            y = y.float() if self.dtype == torch.bfloat16 else y
            out[self.column] = y.cpu().numpy()
        return out


def random_resized_crop_boxes(heights, widths, rng, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), attempts: int = 10):
    """torchvision ``RandomResizedCrop.get_params`` per image -> int32 [N, 4] (y0, x0, h, w):
    area fraction ~ U(scale), log-aspect ~ U(log ratio), 10 tries, then the central crop with the
    aspect clamped into ``ratio``."""
    boxes = np.zeros((len(heights), 4), dtype=np.int32)
    lr = np.log(ratio)
    for i, (H, W) in enumerate(zip(heights, widths)):
        area = H * W
        for _ in range(attempts):
            ta = area * rng.uniform(scale[0], scale[1])
            ar = np.exp(rng.uniform(lr[0], lr[1]))
            w = int(round(np.sqrt(ta * ar)))
            h = int(round(np.sqrt(ta / ar)))
            if 0 < w <= W and 0 < h <= H:
                y0 = int(rng.integers(0, H - h + 1))
                x0 = int(rng.integers(0, W - w + 1))
                boxes[i] = (y0, x0, h, w)
                break
        else:
            in_ratio = W / H
            if in_ratio < ratio[0]:
                w, h = W, int(round(W / ratio[0]))
            elif in_ratio > ratio[1]:
                h, w = H, int(round(H * ratio[1]))
            else:
                w, h = W, H
            boxes[i] = ((H - h) // 2, (W - w) // 2, h, w)
    return boxes


class _CropResizeBase:
    def __init__(self, size, column, mean, std, dtype, keep_on_device, channels_last):
        import torch

        self.size = (size, size) if isinstance(size, int) else tuple(size)
        self.column = column
        self.mean, self.std = mean, std
        self.dtype = getattr(torch, dtype)
        self.keep = keep_on_device
        self.channels_last = channels_last
        self.device = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")

    def _boxes_flips(self, n, H, W):  # pragma: no cover - interface
        raise NotImplementedError

    def __call__(self, batch):
        import torch

        from ..ops import crop_resize_normalize

        imgs = np.ascontiguousarray(batch[self.column])
        N, H, W = imgs.shape[:3]
        boxes, flips = self._boxes_flips(N, H, W)
        x = torch.from_numpy(imgs).to(self.device, non_blocking=True)
        y = crop_resize_normalize(x, boxes, self.size, flips, self.mean, self.std, self.dtype,
                                  channels_last=self.channels_last)
        out = dict(batch)
        if self.keep:
            out[self.column] = y
        else:
            y = y.float() if self.dtype == torch.bfloat16 else y
            out[self.column] = y.cpu().numpy()
        return out


class RandomResizedCropFlipNormalize(_CropResizeBase):
    """ImageNet training augmentation as ONE gfx950 kernel per batch: RandomResizedCrop(size,
    scale, ratio) + RandomHorizontalFlip(p) + ToTensor + Normalize, uint8 HWC in -> bf16 NCHW out
    (boxes/flips drawn on the host, resampling on the device)."""

    def __init__(self, size=224, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3), flip_p: float = 0.5, seed=None,
                 column: str = "image", mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), dtype: str = "bfloat16",
                 keep_on_device: bool = False, channels_last: bool = False):
        super().__init__(size, column, mean, std, dtype, keep_on_device, channels_last)
        self.scale, self.ratio, self.flip_p = scale, ratio, flip_p
        self.rng = np.random.default_rng(seed)

    def _boxes_flips(self, n, H, W):
        boxes = random_resized_crop_boxes([H] * n, [W] * n, self.rng, self.scale, self.ratio)
        flips = (self.rng.random(n) < self.flip_p).astype(np.uint8)
        return boxes, flips


class CenterCropResize(_CropResizeBase):
    """Evaluation transform: the central square-ish region that ``Resize(resize)`` followed by
    ``CenterCrop(size)`` would keep, resampled once to ``size`` and normalised (single bilinear
    resample instead of resize-then-crop)."""

    def __init__(self, size=224, resize=256, column: str = "image", mean=(0.485, 0.456, 0.406),
                 std=(0.229, 0.224, 0.225), dtype: str = "bfloat16", keep_on_device: bool = False,
                 channels_last: bool = False):
        super().__init__(size, column, mean, std, dtype, keep_on_device, channels_last)
        self.resize = resize

    def _boxes_flips(self, n, H, W):
        f = self.resize / min(H, W)  # Resize(shorter side -> resize) scale
        h = max(1, min(H, int(round(self.size[0] / f))))
        w = max(1, min(W, int(round(self.size[1] / f))))
        box = np.array([(H - h) // 2, (W - w) // 2, h, w], dtype=np.int32)
        return np.tile(box, (n, 1)), None
