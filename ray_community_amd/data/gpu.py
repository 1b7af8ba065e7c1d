"""GPU preprocessing UDFs for ``map_batches`` on MI355X (fused HIP kernels).

``ImageNormalize`` turns uint8 HWC image batches into normalised bf16/f32 NCHW tensors in HBM with
ONE gfx950 kernel (cast + scale + mean/std + layout transpose fused), the typical
"Data map_batches GPU preprocess -> model" hot path. Use it as a callable class so the pool
actors own a GPU:  ``ds.map_batches(ImageNormalize, num_gpus=1, concurrency=2, batch_format="numpy")``.
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
