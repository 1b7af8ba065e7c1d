"""Timing breakdown of the Data -> Serve pipeline pieces on one GPU (diagnostic)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import ray_community_amd as ray
    from ray_community_amd import serve
    import bench_data_serve as B

    class Timed(B.Classifier):
        def __call__(self, x):
            import torch

            t0 = time.perf_counter()
            with torch.inference_mode():
                x2 = x.to(self.dev, self.dtype, non_blocking=True)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                y = self.net(x2)
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                p = y.argmax(1).cpu().numpy()
            t3 = time.perf_counter()
            return p, (round(1e3 * (t1 - t0), 1), round(1e3 * (t2 - t1), 1), round(1e3 * (t3 - t2), 1),
                       x.is_contiguous(memory_format=torch.channels_last), str(x.dtype), time.time())

    ray.init(num_cpus=8, num_gpus=1)
    dep = serve.deployment(Timed, name="Classifier", num_replicas=1, max_ongoing_requests=4,
                           ray_actor_options={"num_gpus": 0.5, "num_cpus": 1})
    h = serve.run(dep.bind("resnet50", 224, 256, "cuda"), name="classifier", route_prefix=None)

    @ray.remote(num_gpus=0.25)
    class Pre:
        def __init__(self):
            self.p = B.PreprocessAndClassify("classifier", "cuda")

        def run(self, n, mode):
            batch = B.synth_images({"id": np.arange(256)}, 224)
            ts = []
            for _ in range(n):
                t0 = time.perf_counter()
                x = self.p.norm(batch)["image"]
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                tw = time.time()
                if mode == "gpu":
                    r = self.p.handle.remote(x).result()
                elif mode == "cpu":
                    r = self.p.handle.remote(x.float().cpu()).result()
                else:
                    r = None
                t2 = time.perf_counter()
                info = None if r is None else (r[1][:5], round(1e3 * (r[1][5] - tw), 1))
                ts.append((t1 - t0, t2 - t1, info))
            return ts

    p = Pre.remote()
    for mode in ("gpu", "cpu", "none"):
        ts = ray.get(p.run.remote(6, mode))[2:]
        print(mode, "normalize ms %.1f  handle ms %.1f" % (1e3 * np.mean([a for a, _, _ in ts]),
                                                           1e3 * np.mean([b for _, b, _ in ts])),
              "replica (to, net, argmax ms, cl, dtype), reply-stamp ms:", [c for _, _, c in ts], flush=True)
    serve.shutdown()
    ray.shutdown()


if __name__ == "__main__":
    main()
