"""Locate the largest kernel-vs-reference AdamW difference (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ray_community_amd.ops import reference as ref  # noqa: E402
from ray_community_amd.parallel import FlatAdamW  # noqa: E402
from ray_community_amd.parallel.flat import FlatParameters  # noqa: E402

DEV = "cuda"
n = 8 * 4096 + 5
torch.manual_seed(0)
net = torch.nn.Linear(n, 1, bias=False).to(device=DEV, dtype=torch.bfloat16)
flat = FlatParameters(net, grad_dtype=torch.bfloat16)
opt = FlatAdamW(flat, lr=1e-3, weight_decay=0.1, max_grad_norm=0.5, master_format="fp32")
print("numel", flat.numel, "decay_end", flat.decay_end)
g = torch.Generator(device=DEV).manual_seed(1)
for step in range(3):
    flat.grad.copy_(torch.randn(flat.numel, device=DEV, generator=g).to(torch.bfloat16))
    p, mr, vr, gr = opt.master.clone(), opt.m.clone(), opt.v.clone(), flat.grad.float().clone()
    p_old = p.clone()
    opt.step(0.5)
    c = min(1.0, 0.5 / (float(gr.norm()) * 0.5 + 1e-6))
    for s, e, wd in ((0, flat.decay_end, 0.1), (flat.decay_end, flat.numel, 0.0)):
        if e > s:
            ref.adamw_ref(p[s:e], gr[s:e], mr[s:e], vr[s:e], 1e-3, 0.9, 0.95, 1e-8, wd, opt.step_count,
                          grad_mul=0.5, clip=c)
    _, ex = torch.frexp(torch.maximum(p.abs(), p_old.abs()))
    ulp = torch.ldexp(torch.ones_like(p), ex - 24)
    r = (opt.master - p).abs() / ulp
    i = int(r.argmax())
    print(f"step {step+1} worst {float(r[i]):.1f} ulp at {i}: old {float(p_old[i]):.6e} ref {float(p[i]):.9e} "
          f"ker {float(opt.master[i]):.9e} g {float(gr[i]):.6e} m {float(mr[i]):.6e}/{float(opt.m[i]):.6e} "
          f"v {float(vr[i]):.6e}/{float(opt.v[i]):.6e} sumsq_k {float(opt._sumsq):.8e} sumsq_r {float(gr.pow(2).sum()):.8e}")
    print("  count > 1 ulp:", int((r > 1).sum()), "of", r.numel(), " m diff max", float((opt.m - mr).abs().max()),
          " v diff max", float((opt.v - vr).abs().max()))
