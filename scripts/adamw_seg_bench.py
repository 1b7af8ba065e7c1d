"""Split-master AdamW on the real Llama-3-8B flat layout: the flat kernel vs the segmented kernel
that also writes W^T of every fused-wgrad weight (parallel/optim.py FlatAdamW._setup_transposed).
Prints ms per step for each, the segmented kernel at several grid sizes, and checks one W^T."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_community_amd.models import build_llama  # noqa: E402
from ray_community_amd.ops._lib import lib  # noqa: E402
from ray_community_amd.parallel import DistributedDataParallel, FlatAdamW  # noqa: E402


def timed(fn, n=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    net = build_llama(os.environ.get("MODEL", "llama3-8b"), device="cuda")
    ddp = DistributedDataParallel(net)
    opt = FlatAdamW(ddp.flat, lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0)
    ddp.flat.grad.normal_()
    out = {"params": ddp.flat.numel}
    opt.transposed_weights = False
    out["flat_ms"] = round(timed(lambda: opt.step()), 3)
    opt.transposed_weights = True
    for nb in (4096, 8192, 2048, 16384):
        lib().rca_adamw_split_set_blocks(nb)
        out[f"seg@{nb}_ms"] = round(timed(lambda: opt.step()), 3)
    lib().rca_adamw_split_set_blocks(4096)
    w = net.layers[0].mlp.gate_up.weight
    out["wt_exact"] = bool(torch.equal(w._rca_wt, w.detach().t()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
