"""Same-process, interleaved A/B of the Llama-3-8B training step (the bench.py workload, built once).

    python scripts/step_ab.py --arms base,noplan --rounds 3 --steps 10

Each arm is a named run-time toggle (TOGGLES below) applied before its steps and undone after, so
every arm runs on the same model, optimizer state, allocator state and box; arms alternate inside
each round (A B A B ...), which cancels the box's clock drift that separate processes see.
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def _lib():
    from ray_community_amd.ops import _lib
    return _lib.lib()


def _ops():
    from ray_community_amd import ops
    return ops


def _set_attr(mod, name, value):
    old = getattr(mod, name)
    setattr(mod, name, value)
    return lambda: setattr(mod, name, old)


def _set_lib(fn, value):
    f = getattr(_lib(), fn)
    old = f(value)
    return lambda: f(old)


CTX = {}  # filled after the model is built: "ddp", "opt"


def _toggles():
    from ray_community_amd.parallel import fused_linear as fl
    return {
        "base": lambda: (lambda: None),
        # gradient-norm sum of squares: per bucket on the DDP side stream during backward (default)
        # vs one pass on the compute stream before AdamW
        "norm_side": lambda: _set_attr(CTX["ddp"], "_norm", CTX["norm"]),
        "norm_main": lambda: _set_attr(CTX["ddp"], "_norm", None),
        # RoPE backward fused with the dqkv transpose (default) vs the in-place kernel + transpose
        "rope_tr": lambda: _set_attr(_ops(), "_ROPE_BWD_TR", True),
        "rope_sep": lambda: _set_attr(_ops(), "_ROPE_BWD_TR", False),
        # gate_up input gradient on hipBLASLt instead of the hand GEMM
        "noplan": lambda: _set_attr(fl, "_DGRAD_PLANS_ON", False),
        "plan": lambda: _set_attr(fl, "_DGRAD_PLANS_ON", True),
        # attention backward: 0 = delta/dQ kernel (recomputes S, P, dP) + dK/dV, 1 = delta, dK/dV + dS tiles, dQ = dS.K
        "attn_split": lambda: _set_lib("rca_attn_set_bwd_mode", 0),
        "attn_fused": lambda: _set_lib("rca_attn_set_bwd_mode", 1),
        "attn_fwd_hs": lambda: _set_lib("rca_attn_set_fwd_mode", 2),
        # wait states ahead of the hand-scheduled dK/dV kernel's asm MFMAs (s_nop 1 vs s_nop 3)
        "nop1": lambda: _set_lib("rca_attn_set_hs_nops", 1),
        "nop3": lambda: _set_lib("rca_attn_set_hs_nops", 3),
        # attention forward: 4-wave workgroups (2 per CU) vs 8-wave 256-row workgroups; dQ-from-dS
        # with 1 or 2 query blocks per wave
        "fwd_nw4": lambda: _set_lib("rca_attn_set_fwd_nw", 4),
        "nw8_qw2": lambda: _both(_set_lib("rca_attn_set_fwd_nw", 8), _set_lib("rca_attn_set_dq_qw", 2)),
        "qw1": lambda: _set_lib("rca_attn_set_dq_qw", 1),
    }


def _both(undo_a, undo_b):
    return lambda: (undo_b(), undo_a())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="base,noplan")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=2)
    a = ap.parse_args()
    from ray_community_amd.train.llm import build_llama_training

    toggles = _toggles()
    arms = a.arms.split(",")
    for arm in arms:
        if arm not in toggles:
            raise SystemExit(f"unknown arm {arm!r}; known: {sorted(toggles)}")
    net, ddp, opt, batch, step = build_llama_training(model=a.model, seq_len=a.seq_len, micro_batch=a.micro_batch,
                                                      grad_norm_side_stream=True)
    CTX.update(ddp=ddp, opt=opt, norm=ddp._norm)
    if "norm_side" not in a.arms.split(","):
        ddp._norm = None  # the shipped default: the norm pass runs on the compute stream
    data = [batch() for _ in range(2)]
    times = {arm: [] for arm in arms}
    for arm in arms:  # warm every arm's code path once (kernel loads, W^T copies, allocator)
        undo = toggles[arm]()
        for i in range(a.warmup):
            step(*data[i % 2])
        undo()
    torch.cuda.synchronize()
    for r in range(a.rounds):
        order = arms if r % 2 == 0 else arms[::-1]
        for arm in order:
            undo = toggles[arm]()
            step(*data[0])  # one untimed step after the switch
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(a.steps):
                loss = step(*data[i % 2])
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.steps
            undo()
            times[arm].append(ms)
            print(f"round {r} {arm:12s} {ms:8.2f} ms/step  loss {loss.item():.4f}", flush=True)
    print("arm          median ms   min ms   all")
    for arm in arms:
        t = times[arm]
        print(f"{arm:12s} {statistics.median(t):9.2f} {min(t):8.2f}   " + " ".join(f"{x:.2f}" for x in t))


if __name__ == "__main__":
    main()
