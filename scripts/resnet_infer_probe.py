"""ResNet-50 bf16 NHWC inference probe: whole forward time at the serving batch, and every 1x1
convolution shape timed as MIOpen conv2d vs the same contraction as a GEMM over the channel dim
(NHWC makes a stride-1 1x1 conv a [N*H*W, Cin] x [Cin, Cout] matmul with no data movement)."""
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from ray_community_amd.models.resnet import fold_batchnorm, resnet50  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = True
    bs = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    net = fold_batchnorm(resnet50().to(dev)).to(memory_format=torch.channels_last).to(torch.bfloat16).eval()
    x = torch.randn(bs, 3, 224, 224, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    shapes = []

    def hook(mod, inp, out):
        if mod.kernel_size == (1, 1):
            shapes.append((tuple(inp[0].shape), mod.weight.shape[0], mod.stride[0], mod.bias is not None))

    hs = [m.register_forward_hook(hook) for m in net.modules() if isinstance(m, torch.nn.Conv2d)]
    with torch.inference_mode():
        net(x)
    for h in hs:
        h.remove()
    with torch.inference_mode():
        ms = timeit(lambda: net(x))
    print(f"forward bs={bs}: {ms:.3f} ms  ({bs / ms * 1e3:.0f} img/s)")
    tot_conv = tot_gemm = 0.0
    seen = {}
    for (n, c, h, w), co, s, has_b in shapes:
        key = (n, c, h, w, co, s)
        seen[key] = seen.get(key, 0) + 1
    for (n, c, h, w, co, s), cnt in sorted(seen.items()):
        xi = torch.randn(n, c, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(co, c, 1, 1, device=dev, dtype=torch.bfloat16)
        b = torch.randn(co, device=dev, dtype=torch.bfloat16)
        with torch.inference_mode():
            t_conv = timeit(lambda: F.conv2d(xi, wt, b, stride=s))
            xs = xi[:, :, ::s, ::s] if s > 1 else xi
            w2 = wt.view(co, c)

            def gemm():
                a = xs.permute(0, 2, 3, 1)
                if s > 1:
                    a = a.contiguous()
                return torch.addmm(b, a.reshape(-1, c), w2.t())

            t_gemm = timeit(gemm)
            if s == 1:
                a0 = xi.permute(0, 2, 3, 1).reshape(-1, c)
                t_act = timeit(lambda: torch._addmm_activation(b, a0, w2.t()))
                conv_relu = timeit(lambda: F.relu_(F.conv2d(xi, wt, b)))
            else:
                t_act = conv_relu = float("nan")
        flops = 2 * n * (h // s) * (w // s) * c * co
        tot_conv += cnt * t_conv
        tot_gemm += cnt * t_gemm
        print(f"1x1 N{n} C{c} {h}x{w} -> {co} s{s} x{cnt}: conv {t_conv:.3f} ms ({flops / t_conv / 1e9:.0f} TF/s)"
              f"  gemm {t_gemm:.3f} ms ({flops / t_gemm / 1e9:.0f} TF/s)  gemm+bias+relu epilogue {t_act:.3f} ms"
              f"  conv+bias+relu {conv_relu:.3f} ms")
    print(f"1x1 total: conv {tot_conv:.2f} ms, gemm {tot_gemm:.2f} ms")


if __name__ == "__main__":
    main()
