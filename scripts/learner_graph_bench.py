"""PPO learner update time at bench_rllib.py's learner config (NatureCNN on 84x84x4 uint8 frames,
train batch 8192 = 16 runners x 512, minibatch 1024, 2 epochs), interleaved in one process:

  eager_nchw  the round-5 learner: eager minibatch loop, NCHW conv weights
  eager       eager loop, channels-last (NHWC) conv weights and frames
  graph       NHWC + the minibatch step replayed as a HIP graph (rllib/core/learner.py _PPOStepGraph)

    python scripts/learner_graph_bench.py [--iters 6] [--rounds 3] [--arms eager_nchw,eager,graph]
"""
import argparse
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from ray_community_amd.rllib.core.learner import Learner  # noqa: E402
from ray_community_amd.rllib.policy.sample_batch import SampleBatch  # noqa: E402
from ray_community_amd.rllib.utils.spaces import Box, Discrete  # noqa: E402


def batch(N, T, seed):
    rng = np.random.default_rng(seed)
    b = SampleBatch({"obs": rng.integers(0, 256, (N, T, 84, 84, 4), dtype=np.uint8),
                     "actions": rng.integers(0, 6, (N, T)).astype(np.int64),
                     "rewards": rng.standard_normal((N, T)).astype(np.float32),
                     "terminateds": rng.random((N, T)) < 0.01, "truncateds": np.zeros((N, T), bool),
                     "vf_preds": rng.standard_normal((N, T)).astype(np.float32),
                     "next_vf_preds": rng.standard_normal((N, T)).astype(np.float32),
                     "action_logp": (-rng.random((N, T)) * 2).astype(np.float32),
                     "action_dist_inputs": rng.standard_normal((N, T, 6)).astype(np.float32)})
    b.fragment_shape = (N, T)
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--arms", default="eager_nchw,eager,graph")
    a = ap.parse_args()
    cfg = {"lr": 2.5e-4, "minibatch_size": 1024, "num_epochs": 2, "grad_clip": 0.5, "seed": 0, "kl_coeff": 0.2,
           "entropy_coeff": 0.01, "vf_clip_param": 10.0, "model": {}}
    obs, act = Box(0, 255, (84, 84, 4), np.uint8), Discrete(6)
    opts = {"eager_nchw": dict(learner_cuda_graph=False, learner_channels_last=False),
            "eager": dict(learner_cuda_graph=False), "graph": dict(learner_cuda_graph=True)}
    arms = {k: Learner(dict(cfg, **opts[k]), obs, act, use_gpu=True) for k in a.arms.split(",")}
    # device-resident batch, as the learner actor holds it after _fetch_fragments
    b = batch(16, 512, 0)
    dev = next(next(iter(arms.values())).module.parameters()).device
    bd = SampleBatch({k: torch.as_tensor(v).to(dev) for k, v in b.items()})
    bd.fragment_shape = b.fragment_shape
    for lr in arms.values():  # warm-up: MIOpen algorithm search, graph capture
        lr.update_ppo(bd)
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for r in range(a.rounds):
        order = list(arms)[r % len(arms):] + list(arms)[:r % len(arms)]
        for k in order:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                out = arms[k].update_ppo(bd)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / a.iters
            res[k].append(ms)
            print(f"round {r} {k:10s} {ms:8.2f} ms/update  minibatches {out['num_minibatches']} "
                  f"replays {out['cuda_graph_replays']} loss {out['total_loss']:.4f}", flush=True)
    for k, v in res.items():
        print(f"{k:10s} median {sorted(v)[len(v) // 2]:.2f} ms/update  all {' '.join(f'{x:.2f}' for x in v)}")


if __name__ == "__main__":
    main()
