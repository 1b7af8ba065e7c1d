"""Same-process interleaved A/B of the ResNet-50 1x1 convolutions: MIOpen conv2d vs the NHWC GEMM
(hipBLASLt) path (models/resnet.py LINEAR_1X1), for the folded bf16 serving forward at batch 256
and for the bf16 DDP training step at batch 256 / 224 px (bench_resnet.py's configuration)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_community_amd.models import resnet as R  # noqa: E402


def timeit(fn, iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    net = R.fold_batchnorm(R.resnet50().to(dev)).to(memory_format=torch.channels_last).to(torch.bfloat16)
    x = torch.randn(256, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = {}
    with torch.inference_mode():
        for flag in (False, True):
            R.LINEAR_1X1[0] = flag
            for _ in range(5):
                net(x)
            torch.cuda.synchronize()
            print("infer warm", flag, flush=True)
        for rnd in range(3):
            for flag in (False, True):
                R.LINEAR_1X1[0] = flag
                res.setdefault(("infer", flag), []).append(timeit(lambda: net(x), 20))
                print("infer", flag, f"{res[('infer', flag)][-1]:.3f} ms", flush=True)
    del net
    from ray_community_amd.train.vision import build_resnet_training

    net, ddp, opt, batch, step = build_resnet_training(batch_size=256, image_size=224)
    data = batch()
    for flag in (False, True):
        R.LINEAR_1X1[0] = flag
        for i in range(4):
            t0 = time.perf_counter()
            step(*data)
            torch.cuda.synchronize()
            print("train warmup", flag, i, f"{(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    for rnd in range(3):
        for flag in (False, True):
            R.LINEAR_1X1[0] = flag
            res.setdefault(("train", flag), []).append(timeit(lambda: step(*data), 10))
            print("train", flag, f"{res[('train', flag)][-1]:.3f} ms", flush=True)
    for (kind, flag), v in res.items():
        med = sorted(v)[len(v) // 2]
        print(f"{kind:5s} {'gemm ' if flag else 'miopen'}: " + " ".join(f"{t:.3f}" for t in v)
              + f"  median {med:.3f} ms = {256 / med * 1e3:.0f} img/s", flush=True)


if __name__ == "__main__":
    main()
