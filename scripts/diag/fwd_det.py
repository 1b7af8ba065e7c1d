"""Diagnostic: which forward op of llama3-tiny is run-to-run nondeterministic on the GPU?"""
import torch
from ray_community_amd import ops
from ray_community_amd.models import build_llama

torch.manual_seed(0)
net = build_llama("llama3-tiny", device="cuda")
toks = torch.randint(0, 1024, (2, 129), device="cuda", generator=torch.Generator("cuda").manual_seed(1))


def run():
    outs = {}
    hooks = []
    for n, m in net.named_modules():
        if n:
            hooks.append(m.register_forward_hook(lambda mod, i, o, n=n: outs.__setitem__(
                n, [t.detach().clone() for t in (o if isinstance(o, tuple) else (o,)) if torch.is_tensor(t)])))
    loss = net(toks[:, :-1], toks[:, 1:])
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    return loss.item(), outs


ref_loss, ref = run()
for trial in range(3):
    loss, o = run()
    bad = [n for n in ref if any(not torch.equal(a, b) for a, b in zip(ref[n], o[n]))]
    print("trial", trial, "loss", ref_loss, loss, "first differing modules:", bad[:6], flush=True)

# isolated ops on fixed inputs
x = torch.randn(256, 256, device="cuda", dtype=torch.bfloat16)
w = torch.randn(1024, 256, device="cuda", dtype=torch.bfloat16)
for name, fn in [("F.linear", lambda: torch.nn.functional.linear(x, w)),
                 ("mm_t", lambda: torch.mm(x, w.t())),
                 ("swiglu", lambda: ops.swiglu(torch.nn.functional.linear(x, w))),
                 ("swiglu_t", lambda: ops.swiglu(torch.nn.functional.linear(x, w), with_transposed=True)[1]),
                 ("rmsnorm", lambda: ops.rms_norm(x, torch.ones(256, device="cuda", dtype=torch.bfloat16))),
                 ]:
    a = fn()
    a = a[0] if isinstance(a, tuple) else a
    same = all(torch.equal(a, (lambda r: r[0] if isinstance(r, tuple) else r)(fn())) for _ in range(5))
    print(name, "deterministic" if same else "NONDETERMINISTIC", flush=True)
qkv = torch.randn(2 * 128, (4 + 2 * 2) * 64, device="cuda", dtype=torch.bfloat16)
a = ops.flash_attention_qkv(qkv, 2, 128, 4, 2, 64, causal=True)
print("attn fwd", "deterministic" if all(torch.equal(a, ops.flash_attention_qkv(qkv, 2, 128, 4, 2, 64, causal=True)) for _ in range(5)) else "NONDETERMINISTIC")
h = torch.randn(256, 256, device="cuda", dtype=torch.bfloat16)
lab = torch.randint(0, 1024, (256,), device="cuda")
from ray_community_amd.parallel.fused_linear import linear_cross_entropy
l0 = linear_cross_entropy(h, w, lab)
print("fused ce", "deterministic" if all(torch.equal(l0, linear_cross_entropy(h, w, lab)) for _ in range(5)) else "NONDETERMINISTIC")
