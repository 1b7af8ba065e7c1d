"""GPU object store timing: put / cross-actor get / by-value actor argument on one GPU."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import ray_community_amd as ray

    ray.init(num_cpus=8, num_gpus=1)

    @ray.remote(num_gpus=0.25)
    class B:
        def consume(self, x):
            import torch

            t = time.perf_counter()
            s = float(x.float().sum())
            torch.cuda.synchronize()
            return s, time.perf_counter() - t

        def get(self, refs):
            t0 = time.perf_counter()
            x = ray.get(refs[0])
            t1 = time.perf_counter()
            return float(x.float().sum()), t1 - t0

    @ray.remote(num_gpus=0.25)
    class A:
        def __init__(self, b):
            import torch

            self.b = b
            self.x = torch.randn(256, 3, 224, 224, device="cuda").to(torch.bfloat16)

        def run(self, mode):
            import torch

            out = []
            keep = []
            for i in range(4):
                t0 = time.perf_counter()
                if mode == "put_get_fresh":  # a new allocation every time (kept alive)
                    x = torch.randn(256 + 8 * i, 3, 224, 224, device="cuda").to(torch.bfloat16)
                    keep.append(x)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ref = ray.put(x)
                    t1 = time.perf_counter()
                    s, tg = ray.get(self.b.get.remote([ref]))
                elif mode == "put_get":
                    ref = ray.put(self.x)
                    t1 = time.perf_counter()
                    s, tg = ray.get(self.b.get.remote([ref]))
                else:
                    t1 = time.perf_counter()
                    s, tg = ray.get(self.b.consume.remote(self.x))
                t2 = time.perf_counter()
                out.append((round(1e3 * (t1 - t0), 1), round(1e3 * tg, 1), round(1e3 * (t2 - t1), 1)))
            return out

    b = B.remote()
    a = A.remote(b)
    for mode in ("put_get", "arg", "put_get_fresh"):
        print(mode, "(put ms, reader ms, round trip ms):", ray.get(a.run.remote(mode)), flush=True)
    ray.shutdown()


if __name__ == "__main__":
    main()
