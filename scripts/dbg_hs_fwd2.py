"""Debug: per-half-tile probability mass of the hand-scheduled forward (mode 2) vs the default.
V[key, d] = 1 if d == key // 32 (one-hot half-tile id): O[row, d] = mass of half d / l."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402

lib = ops._lib.lib()
torch.manual_seed(0)
S, D = 256, 128
for causal in (False, True):
    q = torch.randn(1, S, 1, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(1, S, 1, D, device="cuda", dtype=torch.bfloat16)
    v = torch.zeros(1, S, 1, D, device="cuda", dtype=torch.bfloat16)
    for key in range(S):
        v[0, key, 0, key // 32] = 1.0
    outs = []
    for mode in (0, 2):
        lib.rca_attn_set_fwd_mode(mode)
        o = torch.empty(1, S, 1, D, device="cuda", dtype=torch.bfloat16)
        lse = torch.empty(1, 1, S, device="cuda", dtype=torch.float32)
        ops._attn_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), 1, S, 1, 1, D,
                      D, D, D, D, 1.0 / math.sqrt(D), causal)
        torch.cuda.synchronize()
        outs.append((o.float(), lse.clone()))
    lib.rca_attn_set_fwd_mode(0)
    for row in (0, 31, 32, 63, 64, 95, 96, 127, 130, 200, 255):
        ref = outs[0][0][0, row, 0, :8].tolist()
        got = outs[1][0][0, row, 0, :8].tolist()
        print(f"causal={causal} row {row}: lse ref {outs[0][1][0, 0, row].item():.3f} hs {outs[1][1][0, 0, row].item():.3f}")
        print("   ref mass", " ".join(f"{x:.3f}" for x in ref))
        print("   hs  mass", " ".join(f"{x:.3f}" for x in got))
