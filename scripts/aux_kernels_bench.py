"""Timing + bandwidth of the data-path (image.hip) and RL (rl_data.hip) HIP kernels at realistic
shapes, for `rocprofv3 --kernel-trace --stats` summaries (profiles/aux_kernels_r3.md).
Each op runs warmup + 20 timed calls; prints one JSON line per op (us/call, effective GB/s)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_community_amd import ops  # noqa: E402


def timed(name, fn, nbytes, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / iters
    print(json.dumps({"op": name, "us": round(us, 1), "GB/s": round(nbytes / us / 1e3, 1)}), flush=True)


dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
# ImageNet-style batch: 256 x 224 x 224 x 3 uint8 -> bf16 NCHW / NHWC
u8 = torch.randint(0, 256, (256, 224, 224, 3), device=dev, dtype=torch.uint8, generator=g)
n = u8.numel()
timed("image_normalize_nchw_bf16", lambda: ops.image_normalize(u8), n * 3)
timed("image_normalize_nhwc_bf16", lambda: ops.image_normalize(u8, channels_last=True), n * 3)
# RandomResizedCrop from 256 x 320 x 320 x 3 sources to 224 x 224 (+flip), channels_last bf16
src = torch.randint(0, 256, (256, 320, 320, 3), device=dev, dtype=torch.uint8, generator=g)
boxes = torch.tensor([[10, 20, 200, 260]] * 256, dtype=torch.int32)
flips = torch.arange(256) % 2
timed("crop_resize_normalize_nhwc_bf16", lambda: ops.crop_resize_normalize(src, boxes, 224, flips, channels_last=True),
      256 * 224 * 224 * 3 * 2 + 256 * 200 * 260 * 3)
# RL: GAE / V-trace over 1024 envs x 512 steps, standardize 4M advantages
B, T = 1024, 512
r = torch.randn(B, T, device=dev, generator=g)
v = torch.randn(B, T, device=dev, generator=g)
te = torch.rand(B, T, device=dev, generator=g) < 0.01
lv = torch.randn(B, device=dev, generator=g)
timed("gae_1024x512", lambda: ops.compute_gae(r, v, te, te, 0.99, 0.95, last_values=lv), B * T * (4 * 4 + 2))
timed("gae_std_1024x512", lambda: ops.compute_gae(r, v, te, te, 0.99, 0.95, last_values=lv, standardize=True),
      B * T * (4 * 6 + 2))
lr_ = torch.randn(B, T, device=dev, generator=g) * 0.1
timed("vtrace_1024x512", lambda: ops.vtrace(lr_, r, v, v, te, te), B * T * (4 * 6 + 2))
x = torch.randn(1 << 22, device=dev, generator=g)
timed("standardize_4M", lambda: ops.standardize_(x), x.numel() * 4 * 3)
parts = [torch.randn(512, 84 * 84, device=dev, generator=g) for _ in range(32)]
timed("batched_concat_32x512x7056_f32", lambda: ops.batched_concat(parts), 2 * sum(p.numel() * 4 for p in parts))
