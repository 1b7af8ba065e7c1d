"""Serve handle call with a CUDA tensor argument: where does the time go? (diagnostic)"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


class Echo:
    def __call__(self, x):
        import torch

        t = time.perf_counter()
        s = float(x.float().sum())
        torch.cuda.synchronize()
        return tuple(x.shape), time.perf_counter() - t, time.time()


def main():
    import numpy as np

    import ray_community_amd as ray
    from ray_community_amd import serve

    ray.init(num_cpus=8, num_gpus=1)
    dep = serve.deployment(Echo, name="Echo", ray_actor_options={"num_gpus": 0.5, "num_cpus": 1})
    serve.run(dep.bind(), name="echo", route_prefix=None)

    @ray.remote(num_gpus=0.25)
    class Caller:
        def __init__(self):
            self.h = serve.get_app_handle("echo")

        def run(self, numel, on_gpu):
            import torch

            out = []
            for _ in range(4):
                x = torch.ones(numel, device="cuda" if on_gpu else "cpu", dtype=torch.bfloat16)
                t0 = time.time()
                shape, tin, t_rep = self.h.remote(x).result()
                t1 = time.time()
                out.append((round(1e3 * (t1 - t0), 1), round(1e3 * (t_rep - t0), 1), round(1e3 * tin, 2)))
            return out

    c = Caller.remote()
    for numel, g in ((1024, True), (1 << 24, True), (1024, False)):
        print(f"numel={numel} gpu={g} (round trip ms, reply-stamp ms, compute ms):", ray.get(c.run.remote(numel, g)),
              flush=True)
    serve.shutdown()
    ray.shutdown()


if __name__ == "__main__":
    main()
