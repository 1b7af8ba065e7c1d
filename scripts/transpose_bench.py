"""ops.transpose bandwidth + exactness at the 8B training shapes (run twice: default kernel and
RCA_TRANSPOSE_TILE64=1 for the 64 x 64 kernel)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ray_community_amd import ops  # noqa: E402


def main():
    for R, C in [(8192, 4096), (8192, 6144), (8192, 14336), (6144, 4096), (28672, 4096), (4096, 14336), (8192, 128256)]:
        x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(C, R, device="cuda", dtype=torch.bfloat16)
        ops.transpose(x, out=out)
        ok = bool(torch.equal(out, x.t()))
        for _ in range(3):
            ops.transpose(x, out=out)
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            ops.transpose(x, out=out)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(json.dumps({"R": R, "C": C, "exact": ok, "us": round(dt * 1e6, 1),
                          "TBps": round(2 * x.numel() * 2 / dt / 1e12, 2),
                          "tile64": bool(os.environ.get("RCA_TRANSPOSE_TILE64"))}), flush=True)
        del x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
