"""Debug: hand-scheduled attention forward (mode 2) vs the default kernel, per 32-row group."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_community_amd import ops  # noqa: E402

lib = ops._lib.lib()
torch.manual_seed(0)
for causal in (False, True):
    for S in (256, 512):
        B, H, D = 1, 1, 128
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        res = []
        for mode in (0, 2):
            lib.rca_attn_set_fwd_mode(mode)
            o, lse = ops.flash_attention_fwd_lse(q, k, v, causal) if hasattr(ops, "flash_attention_fwd_lse") else (
                ops.flash_attention(q, k, v, causal), None)
            torch.cuda.synchronize()
            res.append(o.float())
        lib.rca_attn_set_fwd_mode(0)
        d = (res[1] - res[0]).abs().amax(dim=(0, 2, 3))  # per row
        print(f"causal={causal} S={S}: per-32-row max err:",
              " ".join(f"{d[i:i + 32].max().item():.3f}" for i in range(0, S, 32)), flush=True)
        bad = (d > 0.05).nonzero().flatten().tolist()
        print("  first bad rows:", bad[:12], "nan:", torch.isnan(res[1]).any().item(), flush=True)
        # per-column check on one bad row
        if bad:
            r = bad[0]
            print("  row", r, "ref[:8]", res[0][0, r, 0, :8].tolist(), "\n  got[:8]", res[1][0, r, 0, :8].tolist())
