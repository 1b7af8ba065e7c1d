"""Down-projection dgrad + SwiGLU backward at the Llama-3-8B MLP shape (T 8192, H 4096, F 14336):
fused (ops.gemm_swiglu_bwd: variant-7 GEMM with the SwiGLU-backward epilogue) vs unfused
(hipBLASLt dh = dy W on the W^T copy + ops.swiglu_backward with the transposed copy) vs the
variant-7 GEMM alone (what the epilogue adds). Interleaved rounds, best of N."""
import sys

import torch

sys.path.insert(0, ".")
from ray_community_amd import ops  # noqa: E402

T, H, F = 8192, 4096, 14336
dy = torch.randn(T, H, device="cuda").to(torch.bfloat16)
w_t = (torch.randn(F, H, device="cuda") / 64).to(torch.bfloat16)
gu = torch.randn(T, 2 * F, device="cuda").to(torch.bfloat16)
dh = torch.empty(T, F, device="cuda", dtype=torch.bfloat16)
lib = ops._lib.lib()


def fused():
    ops.gemm_swiglu_bwd(dy, w_t, gu)


def unfused():
    torch.mm(dy, w_t.t(), out=dh)
    ops.swiglu_backward(gu, dh, with_transposed=True)
    ops.pop_grad_transposed(dh)


def gemm7():
    lib.rca_gemm_set_variant(7)
    ops.gemm(dy, w_t, out=dh)


def swiglu_only():
    ops.swiglu_backward(gu, dh, with_transposed=True)


def timeit(fn, reps=5):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


fns = {"fused": fused, "unfused": unfused, "gemm_v7": gemm7, "hipblaslt_dgrad": lambda: torch.mm(dy, w_t.t(), out=dh),
       "swiglu_bwd_tr": swiglu_only}
for f in fns.values():
    f()
res = {k: [] for k in fns}
for _ in range(3):
    for k, f in fns.items():
        res[k].append(timeit(f))
for k, v in res.items():
    print(f"{k:16s} {min(v) * 1000:8.1f} us")
