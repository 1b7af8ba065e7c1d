"""First-call cost of ResNet-50 inference on fresh IPC-mapped inputs, cudnn.benchmark on/off."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import ray_community_amd as ray

    ray.init(num_cpus=8, num_gpus=1)

    @ray.remote(num_gpus=0.25)
    class Reader:
        def __init__(self, bench):
            import torch

            from ray_community_amd.models.resnet import fold_batchnorm, resnet50

            torch.backends.cudnn.benchmark = bench
            self.net = fold_batchnorm(resnet50().cuda()).to(memory_format=torch.channels_last).to(torch.bfloat16)
            x = torch.randn(256, 3, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            with torch.inference_mode():
                for _ in range(3):
                    self.net(x)
            torch.cuda.synchronize()

        def run(self, x):
            import torch

            t = time.perf_counter()
            with torch.inference_mode():
                self.net(x)
            torch.cuda.synchronize()
            return round(1e3 * (time.perf_counter() - t), 1)

    @ray.remote(num_gpus=0.25)
    class Owner:
        def go(self, r, n):
            import torch

            keep, out = [], []
            for i in range(n):
                x = torch.randn(256, 3, 224, 224, device="cuda").to(torch.bfloat16).contiguous(
                    memory_format=torch.channels_last)
                keep.append(x)
                out.append(ray.get(r.run.remote(x)))
            return out

    for bench in (True, False):
        r = Reader.remote(bench)
        print("cudnn.benchmark", bench, "ms per call on fresh mapped inputs:", ray.get(Owner.remote().go.remote(r, 5)),
              flush=True)
        ray.kill(r)
    ray.shutdown()


if __name__ == "__main__":
    main()
