"""Postprocessing (reference: ``rllib/evaluation/postprocessing.py``): GAE / discounted returns
backed by the gfx950 HIP scan kernel on GPU tensors."""
from __future__ import annotations

import numpy as np
import torch

from ... import ops
from ..policy.sample_batch import SampleBatch


class Postprocessing:
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"


def discount_cumsum(x: np.ndarray, gamma: float) -> np.ndarray:
    out = np.zeros_like(x, dtype=np.float64)
    run = 0.0
    for t in range(len(x) - 1, -1, -1):
        run = x[t] + gamma * run
        out[t] = run
    return out.astype(np.float32)


def compute_advantages(rollout: SampleBatch, last_r: float, gamma: float = 0.9, lambda_: float = 1.0,
                       use_gae: bool = True, use_critic: bool = True):
    """Single-trajectory API of the reference (terminal-free trajectory ending in ``last_r``)."""
    r = torch.as_tensor(np.asarray(rollout[SampleBatch.REWARDS], dtype=np.float32))
    T = r.shape[0]
    if use_gae:
        v = torch.as_tensor(np.asarray(rollout[SampleBatch.VF_PREDS], dtype=np.float32))
        z = torch.zeros(T, dtype=torch.bool)
        adv, tgt = ops.compute_gae(r, v, z, z, gamma, lambda_, last_values=torch.tensor([float(last_r)]))
        rollout[Postprocessing.ADVANTAGES] = adv.numpy()
        rollout[Postprocessing.VALUE_TARGETS] = tgt.numpy()
    else:
        rew = np.concatenate([np.asarray(rollout[SampleBatch.REWARDS]), [last_r]])
        ret = discount_cumsum(rew, gamma)[:-1]
        if use_critic:
            rollout[Postprocessing.ADVANTAGES] = ret - np.asarray(rollout[SampleBatch.VF_PREDS])
            rollout[Postprocessing.VALUE_TARGETS] = ret
        else:
            rollout[Postprocessing.ADVANTAGES] = ret
            rollout[Postprocessing.VALUE_TARGETS] = np.zeros_like(ret)
    return rollout
