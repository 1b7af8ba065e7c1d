"""Read bandwidth / conv speed on an IPC-mapped GPU object vs a local copy (diagnostic)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import ray_community_amd as ray

    ray.init(num_cpus=8, num_gpus=1)

    @ray.remote(num_gpus=0.25)
    class Reader:
        def __init__(self):
            import torch
            import torch.nn.functional as F

            self.w = torch.randn(64, 3, 7, 7, device="cuda", dtype=torch.bfloat16)
            from ray_community_amd.models.resnet import fold_batchnorm, resnet50

            torch.backends.cudnn.benchmark = True
            net = fold_batchnorm(resnet50().cuda()).to(memory_format=torch.channels_last)
            self.net = net.to(torch.bfloat16)

        def bench(self, x):
            import torch
            import torch.nn.functional as F

            def t(fn, n=5):
                fn()
                torch.cuda.synchronize()
                s = time.perf_counter()
                for _ in range(n):
                    fn()
                torch.cuda.synchronize()
                return (time.perf_counter() - s) / n * 1e3

            local = x.clone()
            out = {"mapped_is_cl": x.is_contiguous(memory_format=torch.channels_last), "ptr_mod_256": x.data_ptr() % 256}
            with torch.inference_mode():
                for name, v in (("local", local), ("mapped", x)):
                    out[name + "_sum_ms"] = round(t(lambda: v.sum()), 3)
                    out[name + "_conv_ms"] = round(t(lambda: F.conv2d(v, self.w, stride=2, padding=3)), 3)
                    out[name + "_resnet_ms"] = round(t(lambda: self.net(v), n=3), 3)
            out["nbytes"] = x.numel() * 2
            return out

    @ray.remote(num_gpus=0.25)
    class Owner:
        def run(self, r):
            import torch

            x = torch.randn(256, 3, 224, 224, device="cuda").to(torch.bfloat16)
            x = x.contiguous(memory_format=torch.channels_last)
            return ray.get(r.bench.remote(x))

    r = Reader.remote()
    print(ray.get(Owner.remote().run.remote(r)), flush=True)
    ray.shutdown()


if __name__ == "__main__":
    main()
