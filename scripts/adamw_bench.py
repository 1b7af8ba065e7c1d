"""AdamW kernel A/B: fp32 master (28 B/param) vs split master (26 B/param) on an 8B-sized flat
buffer (the Llama-3-8B parameter count), bf16 grads, clip on. Prints ms and effective TB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_community_amd.ops._lib import check, lib, stream_ptr  # noqa: E402

N = int(float(os.environ.get("ADAMW_N", 8.03e9)))
dev = torch.device("cuda")
g = torch.zeros(N, dtype=torch.bfloat16, device=dev)
m = torch.zeros(N, dtype=torch.float32, device=dev)
v = torch.zeros(N, dtype=torch.float32, device=dev)
hi = torch.zeros(N, dtype=torch.bfloat16, device=dev)
sumsq = torch.ones(1, device=dev)
st = stream_ptr(dev)
out = {}
kinds = ["split", "fp32"] + [f"split@{nb}" for nb in (2048, 8192, 16384)]
for kind in kinds:
    if kind.startswith("split@"):
        lib().rca_adamw_split_set_blocks(int(kind.split("@")[1]))
        kind_base = "split"
    else:
        lib().rca_adamw_split_set_blocks(4096)
        kind_base = kind
    if kind_base == "fp32":
        master = torch.zeros(N, dtype=torch.float32, device=dev)
        fn = lambda: check(lib().rca_adamw(master.data_ptr(), hi.data_ptr(), g.data_ptr(), 0, m.data_ptr(),
                                           v.data_ptr(), N, 1e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 1.0,
                                           sumsq.data_ptr(), 1.0, st), "adamw")
        bpp = 28
    else:
        lo = torch.zeros(N, dtype=torch.int16, device=dev)
        fn = lambda: check(lib().rca_adamw_split(hi.data_ptr(), lo.data_ptr(), g.data_ptr(), 0, m.data_ptr(),
                                                 v.data_ptr(), N, 1e-4, 0.9, 0.95, 1e-8, 0.1, 0.1, 0.05, 1.0,
                                                 sumsq.data_ptr(), 1.0, st), "adamw_split")
        bpp = 26
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    out[kind] = {"ms": round(ms, 3), "TB/s": round(N * bpp / ms / 1e9, 3), "bytes_per_param": bpp}
    if kind_base == "split":
        del lo
    else:
        del master
print(json.dumps({"n": N, **out}))
