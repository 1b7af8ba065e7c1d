"""Which Python lines launch the stray bf16 add kernels in the 8B step (torch.profiler with stacks
on a 2-layer model at 8B width)."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd.train.llm import build_llama_training  # noqa: E402


def main():
    net, ddp, opt, batch, step = build_llama_training(model="llama3-8b", seq_len=4096, micro_batch=2, num_layers=2)
    data = batch()
    step(*data)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step(*data)
        torch.cuda.synchronize()
    c = Counter()
    for e in prof.events():
        if e.name in ("aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::copy_", "aten::mul", "aten::mul_"):
            st = [f for f in (e.stack or []) if "ray_community_amd" in f or "torch/autograd" in f][:3]
            c[(e.name, tuple(st))] += 1
    for (name, st), n in c.most_common(25):
        print(n, name, " <- ".join(st))


if __name__ == "__main__":
    main()
