"""The Data->Serve pipeline's replica work alone: bench_data_serve.Classifier on a device-resident
bf16 NHWC batch of 256, in-process (no Data, no Serve). Prints ms per batch and images/s, the
ceiling of bench_data_serve.py with one replica."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench_data_serve import Classifier  # noqa: E402

bs = int(os.environ.get("BS", 256))
layout = os.environ.get("LAYOUT", "nhwc")
c = Classifier("resnet50", 224, bs, "cuda")
x = torch.randn(bs, 3, 224, 224, device="cuda", dtype=torch.bfloat16)
if layout == "nhwc":
    x = x.contiguous(memory_format=torch.channels_last)
else:
    c.net = c.net.to(memory_format=torch.contiguous_format)
for _ in range(3):
    c(x)
torch.cuda.synchronize()
time.sleep(float(os.environ.get("GAP_S", 0)))  # an idle gap that marks the steady state in a trace
res = {}
if os.environ.get("AB_UNROLL"):  # same-process A/B of the BN apply pass: 1 vs 4 vectors in flight per lane
    from ray_community_amd.ops._lib import lib

    for rnd in range(3):
        for u in (1, 4):
            lib().rca_bn_set_unroll(u)
            ts = []
            for _ in range(15):
                t0 = time.perf_counter()
                with torch.inference_mode():
                    c.net(x)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            res.setdefault(f"unroll{u}_ms", []).append(round(ts[len(ts) // 2] * 1e3, 3))
    lib().rca_bn_set_unroll(4)
if os.environ.get("AB_GEMM"):  # same-process A/B: folded 1x1 convolutions on the GEMM epilogue vs MIOpen + BiasAct
    from ray_community_amd.models import resnet as R

    for rnd in range(3):
        for on in (False, True):
            R.GEMM_1X1[0] = on
            for _ in range(2):
                with torch.inference_mode():
                    c.net(x)
            ts = []
            for _ in range(15):
                t0 = time.perf_counter()
                with torch.inference_mode():
                    c.net(x)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            res.setdefault(f"gemm1x1_{int(on)}_ms", []).append(round(ts[len(ts) // 2] * 1e3, 3))
    R.GEMM_1X1[0] = False
for name, fn in (("forward_only", lambda: c.net(x)), ("call_with_argmax_to_host", lambda: c(x))):
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        with torch.inference_mode():
            fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2] * 1e3
    res[name] = {"ms_median": round(med, 3), "images_per_s": round(bs / med * 1e3, 1)}
print(json.dumps({"layout": layout, "bs": bs, **res}))
