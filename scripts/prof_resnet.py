"""In-process ResNet-50 training steps for kernel profiling (bench_resnet.py runs the loop inside
a Train worker actor, which rocprofv3 would not follow).

    rocprofv3 --kernel-trace --stats -d gpurun_out/profrn -o run -- python scripts/prof_resnet.py --steps 5
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_community_amd.train.vision import build_resnet_training  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    net, ddp, opt, batch, step = build_resnet_training(batch_size=a.batch_size)
    data = batch()
    for _ in range(a.warmup):
        step(*data)
    torch.cuda.synchronize()
    time.sleep(float(os.environ.get("GAP_S", 0)))  # idle gap marking the steady state in a trace
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step(*data)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    print(f"resnet50 bs{a.batch_size}: {1000 * dt:.1f} ms/step  {a.batch_size / dt:.0f} img/s  loss {loss.item():.3f}  "
          f"peak {torch.cuda.max_memory_allocated() / 1e9:.1f} GB", flush=True)


if __name__ == "__main__":
    main()
