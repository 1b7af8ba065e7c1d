"""Serving forward of the folded bf16 ResNet-50 at batch 256: eager launches vs one HIP-graph
replay (static input buffer), interleaved in one process."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_community_amd.models.resnet import fold_batchnorm, resnet50  # noqa: E402


def timeit(fn, iters=30):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    net = fold_batchnorm(resnet50().to(dev)).to(memory_format=torch.channels_last).to(torch.bfloat16)
    x = torch.randn(256, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    static_x = x.clone()
    with torch.inference_mode():
        for _ in range(5):
            ref = net(x)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                net(static_x)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            static_y = net(static_x)
        g.replay()
        torch.cuda.synchronize()
        err = (static_y.float() - ref.float()).abs().max().item()
        print(f"graph vs eager max abs diff {err:.4f}", flush=True)

        def graphed():
            static_x.copy_(x)
            g.replay()
            return static_y

        for rnd in range(3):
            te = timeit(lambda: net(x))
            tg = timeit(graphed)
            print(f"round {rnd}: eager {te:.3f} ms  graph {tg:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
