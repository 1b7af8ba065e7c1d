"""CPU policy-inference variants of the Atari NatureCNN actor-critic as the PPO env runners run it
(batch = envs per runner, one thread), interleaved rounds in one process:
  dense_nchw_w : default conv weights, channels-last input (the runner's permuted uint8 frames)
  cl_w         : conv weights in channels_last (oneDNN NHWC path, no input reorder)
  mkl_prepack  : oneDNN prepacked conv stack (torch.utils.mkldnn), uint8 permuted to NCHW first

    python scripts/runner_infer_bench.py [--batch 16] [--rounds 5]
"""
import argparse
import copy
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    torch.set_num_threads(1)
    import torch.utils.mkldnn as mk

    from ray_community_amd.rllib.core.rl_module import RLModule
    from ray_community_amd.rllib.utils.spaces import Box, Discrete

    m = RLModule(Box(0, 255, shape=(84, 84, 4), dtype=np.uint8), Discrete(6), {"vf_share_layers": True}).eval()
    obs = torch.from_numpy(np.random.randint(0, 255, (a.batch, 84, 84, 4), dtype=np.uint8))
    enc = m.encoder.net
    enc_cl = copy.deepcopy(enc).to(memory_format=torch.channels_last)
    convs_mk = mk.to_mkldnn(copy.deepcopy(enc[:6]))

    def heads(h):
        return m.pi(h), m.vf(h)

    arms = {
        "dense_nchw_w": lambda: heads(enc(obs.permute(0, 3, 1, 2).float().div_(255.0))),
        "cl_w": lambda: heads(enc_cl(obs.permute(0, 3, 1, 2).float().div_(255.0))),
        "mkl_prepack": lambda: heads(enc[6:](convs_mk(obs.permute(0, 3, 1, 2).contiguous().float().div_(255.0)
                                                       .to_mkldnn()).to_dense())),
    }
    with torch.no_grad():
        ref = arms["dense_nchw_w"]()[0]
        for k, f in arms.items():
            err = (f()[0] - ref).abs().max().item()
            print(f"{k:14s} max |dlogits| vs dense {err:.3g}", flush=True)
        res = {k: [] for k in arms}
        for r in range(a.rounds):
            for k in (list(arms) if r % 2 == 0 else list(arms)[::-1]):
                f = arms[k]
                for _ in range(10):
                    f()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    f()
                res[k].append(1e3 * (time.perf_counter() - t0) / a.iters)
    for k, v in res.items():
        print(f"{k:14s} median {statistics.median(v):.3f} ms  min {min(v):.3f}  all " + " ".join(f"{x:.3f}" for x in v))


if __name__ == "__main__":
    main()
