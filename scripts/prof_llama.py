"""In-process Llama training steps for kernel profiling (rocprofv3 only sees the process it
launches; bench.py runs the loop inside a Train worker actor).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python scripts/prof_llama.py --steps 3
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_community_amd.train.llm import build_llama_training  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    net, ddp, opt, batch, step = build_llama_training(model=a.model, seq_len=a.seq_len, micro_batch=a.micro_batch)
    data = batch()
    for _ in range(a.warmup):
        step(*data)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step(*data)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    tok = a.micro_batch * a.seq_len
    print(f"{a.model}: {1000 * dt:.1f} ms/step  {tok / dt:.0f} tok/s  loss {loss.item():.4f}  "
          f"peak {torch.cuda.max_memory_allocated() / 1e9:.1f} GB", flush=True)


if __name__ == "__main__":
    main()
