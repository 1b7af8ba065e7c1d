"""RMSNorm (fused residual) fwd / fwd+bwd timing at the Llama-3-8B training shape (8192 x 4096)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ray_community_amd import ops


def main():
    rows, H = int(os.environ.get("ROWS", 8192)), int(os.environ.get("H", 4096))
    x = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(rows, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = (1 + 0.1 * torch.randn(H, device="cuda")).to(torch.bfloat16).requires_grad_(True)
    gy, gs = torch.randn_like(x), torch.randn_like(x)
    y, s = ops.rms_norm(x, w, 1e-5, r)

    def bwd():
        torch.autograd.backward([y, s], [gy, gs], retain_graph=True)

    for _ in range(5):
        bwd()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        bwd()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    gb = 4 * rows * H * 2 / 1e9  # s, dy, dres read + dx write
    print(f"{os.environ.get('RCA_KERNEL_LIB', 'new')}: rmsnorm bwd {rows}x{H}: {ms * 1e3:.1f} us/call "
          f"(incl. autograd + colsum; {gb / ms:.2f} TB/s on the 4 row streams)", flush=True)


if __name__ == "__main__":
    main()
