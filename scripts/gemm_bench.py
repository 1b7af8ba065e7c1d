"""Hand-written gfx950 GEMM (ops.gemm) vs torch/hipBLASLt on the Llama-3-8B training shapes.

For each shape: numerics vs an fp32 torch reference, then interleaved timing rounds in one
process (cdna_hip_programming.md §5.4 rule 24) of
  * ours      : ops.gemm on the natural layout (no transposed copies),
  * torch     : torch.matmul on the same natural layout (hipBLASLt picks its own kernel),
  * torch+tr  : what the model did in round 1 for backward layouts: HIP transpose copies + the
                reduction-contiguous hipBLASLt GEMM (transpose time included).
Random uniform operands (rule 25)."""
import argparse
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from ray_community_amd import ops  # noqa: E402

T = 8192
SHAPES = [  # (name, kind, M, N, K)
    ("qkv_fwd", "fwd", T, 6144, 4096), ("o_fwd", "fwd", T, 4096, 4096), ("gu_fwd", "fwd", T, 28672, 4096),
    ("down_fwd", "fwd", T, 4096, 14336), ("lm_fwd", "fwd", T, 128256, 4096),
    ("qkv_dgrad", "dgrad", T, 4096, 6144), ("gu_dgrad", "dgrad", T, 4096, 28672), ("down_dgrad", "dgrad", T, 14336, 4096),
    ("lm_dgrad", "dgrad", T, 4096, 128256),
    ("qkv_wgrad", "wgrad", 6144, 4096, T), ("gu_wgrad", "wgrad", 28672, 4096, T), ("down_wgrad", "wgrad", 4096, 14336, T),
    ("lm_wgrad", "wgrad", 128256, 4096, T),
]


def operands(kind, M, N, K, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    if kind == "fwd":      # x [M][K], w [N][K]
        a, b = r(M, K), r(N, K)
        return a, b, False, False, lambda: torch.matmul(a, b.t()), lambda: torch.matmul(a, b.t())
    if kind == "dgrad":    # dy [M][K(=n_out)], w [K][N]
        a, b = r(M, K), r(K, N)
        return a, b, False, True, lambda: torch.matmul(a, b), lambda: torch.matmul(a, ops.transpose(b).t())
    a, b = r(K, M), r(K, N)  # wgrad: dy [T=K][M], x [T=K][N]
    return a, b, True, True, lambda: torch.matmul(a.t(), b), lambda: torch.matmul(ops.transpose(a), ops.transpose(b).t())


def timeit(fn, reps):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--variants", default="2,0", help="hand-GEMM variants to time (gemm.hip launch_variant)")
    ap.add_argument("--tn", action="store_true",
                    help="also time every variant and torch on pre-transposed k-contiguous operands (keys *_tn, "
                         "transpose time excluded): the kernel-against-kernel comparison on hipBLASLt's best layout")
    args = ap.parse_args()
    dev = "cuda"
    rows = []
    for name, kind, M, N, K in SHAPES:
        if args.only and args.only not in name:
            continue
        a, b, ak, bk, f_torch, f_tr = operands(kind, M, N, K, dev)
        variants = [int(v) for v in args.variants.split(",") if v]
        lib = ops._lib.lib()
        ref = f_torch().float()
        row_err = {}
        for v in variants:
            lib.rca_gemm_set_variant(v)
            o = ops.gemm(a, b, ak, bk)
            row_err[f"v{v}_err"] = ((o.float() - ref).abs().max() / ref.abs().max()).item()
            o2 = o.clone()
            ops.gemm(a, b, ak, bk, out=o2, accumulate=True)
            row_err[f"v{v}_acc_err"] = ((o2.float() - 2 * ref).abs().max() / (2 * ref.abs().max())).item()
            del o, o2
        lib.rca_gemm_set_variant(variants[0])
        out = ops.gemm(a, b, ak, bk)
        def mk(v):
            def f():
                lib.rca_gemm_set_variant(v)
                ops.gemm(a, b, ak, bk, out=out)
            return f
        fns = {f"v{v}": mk(v) for v in variants}
        fns["torch"] = f_torch
        fns["torch+tr"] = f_tr
        if args.tn:
            at = a if not ak else ops.transpose(a)          # [M][K]
            bt = b if not bk else ops.transpose(b)          # [N][K]
            for v in variants:
                lib.rca_gemm_set_variant(v)
                o = ops.gemm(at, bt, False, False)
                row_err[f"v{v}_tn_err"] = ((o.float() - ref).abs().max() / ref.abs().max()).item()
                del o
            def mk_tn(v):
                def f():
                    lib.rca_gemm_set_variant(v)
                    ops.gemm(at, bt, False, False, out=out)
                return f
            for v in variants:
                fns[f"v{v}_tn"] = mk_tn(v)
            fns["torch_tn"] = lambda: torch.matmul(at, bt.t())
        for f in fns.values():
            f()
        res = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f, args.reps))
        lib.rca_gemm_set_variant(variants[0])
        fl = 2.0 * M * N * K
        row = {"name": name, "M": M, "N": N, "K": K, **row_err}
        for k, v in res.items():
            ms = min(v)
            row[k + "_ms"] = round(ms, 4)
            row[k + "_tf"] = round(fl / ms / 1e9, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
        del a, b, out, ref
        if args.tn:
            del at, bt
        torch.cuda.empty_cache()
    tot = {k: round(sum(r[k + "_ms"] for r in rows), 4) for k in list(res)}
    print(json.dumps({"total_ms": tot}), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"rows": rows, "total_ms": tot}, f, indent=1)


if __name__ == "__main__":
    main()
