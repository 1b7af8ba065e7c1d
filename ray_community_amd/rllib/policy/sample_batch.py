"""SampleBatch (reference: ``rllib/policy/sample_batch.py``).

A dict of equally-long column arrays. Rollout fragments are kept time-major per env as
``[num_envs, T]`` blocks (``SampleBatch.fragment_shape``) so GAE runs as one batched HIP scan;
``concat_samples`` stacks fragments along the env axis and can run on device in one launch.
"""
from __future__ import annotations

from typing import Dict, Iterator, List, Optional

import numpy as np


class SampleBatch(dict):
    OBS = "obs"
    NEXT_OBS = "new_obs"
    ACTIONS = "actions"
    REWARDS = "rewards"
    TERMINATEDS = "terminateds"
    TRUNCATEDS = "truncateds"
    DONES = "dones"
    INFOS = "infos"
    EPS_ID = "eps_id"
    ENV_ID = "env_id"
    T = "t"
    ACTION_DIST_INPUTS = "action_dist_inputs"
    ACTION_LOGP = "action_logp"
    VF_PREDS = "vf_preds"
    VALUES_BOOTSTRAPPED = "values_bootstrapped"
    NEXT_VF_PREDS = "next_vf_preds"
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"
    SEQ_LENS = "seq_lens"

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.fragment_shape = None  # (num_envs, T) when columns are env-major rollout blocks

    @property
    def count(self) -> int:
        for v in self.values():
            if hasattr(v, "shape") and len(v.shape) >= 1:
                if self.fragment_shape is not None:
                    return int(self.fragment_shape[0] * self.fragment_shape[1])
                return int(v.shape[0])
            if isinstance(v, list):
                return len(v)
        return 0

    def __len__(self):
        return self.count

    def env_steps(self):
        return self.count

    def agent_steps(self):
        return self.count

    def flatten(self) -> "SampleBatch":
        """[N, T, ...] fragment blocks -> [N*T, ...] rows."""
        if self.fragment_shape is None:
            return self
        N, T = self.fragment_shape
        out = SampleBatch()
        for k, v in self.items():
            if hasattr(v, "shape") and tuple(v.shape[:2]) == (N, T):
                out[k] = v.reshape((N * T,) + tuple(v.shape[2:]))
            else:
                out[k] = v
        return out

    def slice(self, start: int, end: int) -> "SampleBatch":
        return SampleBatch({k: v[start:end] for k, v in self.items()})

    def __getitem__(self, key):
        if isinstance(key, slice):
            return self.slice(key.start or 0, key.stop if key.stop is not None else self.count)
        return dict.__getitem__(self, key)

    def shuffle(self, rng=None) -> "SampleBatch":
        n = self.count
        perm = (rng or np.random).permutation(n)
        for k, v in list(self.items()):
            if hasattr(v, "shape") and v.shape[:1] == (n,):
                self[k] = v[perm] if isinstance(v, np.ndarray) else v[_to_index(perm, v)]
        return self

    def timeslices(self, size: int) -> List["SampleBatch"]:
        return [self.slice(i, min(i + size, self.count)) for i in range(0, self.count, size)]

    def minibatches(self, size: int, rng=None) -> Iterator["SampleBatch"]:
        n = self.count
        perm = (rng or np.random).permutation(n)
        for i in range(0, n - size + 1 if n >= size else 1, size):
            idx = perm[i: i + size]
            yield SampleBatch({k: (v[idx] if isinstance(v, np.ndarray) else v[_to_index(idx, v)])
                               for k, v in self.items() if hasattr(v, "shape")})

    def copy(self, shallow=False):
        out = SampleBatch({k: (v if shallow else v.copy() if hasattr(v, "copy") else v) for k, v in self.items()})
        out.fragment_shape = self.fragment_shape
        return out

    def to_device(self, device):
        import torch

        out = SampleBatch()
        for k, v in self.items():
            if isinstance(v, np.ndarray) and v.dtype != object:
                out[k] = torch.from_numpy(np.ascontiguousarray(v)).to(device, non_blocking=True)
            elif hasattr(v, "to"):
                out[k] = v.to(device)
            else:
                out[k] = v
        out.fragment_shape = self.fragment_shape
        return out

    def as_multi_agent(self, policy_id="default_policy"):
        return MultiAgentBatch({policy_id: self}, self.count)


def _to_index(idx, v):
    import torch

    return torch.as_tensor(idx, device=v.device)


def concat_samples(batches: List[SampleBatch]) -> SampleBatch:
    """Concatenate batches. Fragment blocks with equal T stack along the env axis."""
    batches = [b for b in batches if b is not None and b.count > 0]
    if not batches:
        return SampleBatch()
    if isinstance(batches[0], MultiAgentBatch):
        return MultiAgentBatch.concat_samples(batches)
    fs = [b.fragment_shape for b in batches]
    out = SampleBatch()
    keys = batches[0].keys()
    if all(f is not None for f in fs) and len({f[1] for f in fs}) == 1:
        for k in keys:
            out[k] = _cat([b[k] for b in batches])
        out.fragment_shape = (sum(f[0] for f in fs), fs[0][1])
        return out
    flat = [b.flatten() for b in batches]
    for k in keys:
        out[k] = _cat([b[k] for b in flat])
    return out


def _cat(xs):
    if isinstance(xs[0], np.ndarray):
        return np.concatenate(xs, axis=0)
    import torch

    if isinstance(xs[0], torch.Tensor):
        from ...ops import batched_concat

        return batched_concat(xs)
    if isinstance(xs[0], list):
        return sum(xs, [])
    return xs[0]


class MultiAgentBatch:
    """Per-policy SampleBatches of one sampling round (reference ``MultiAgentBatch``)."""

    def __init__(self, policy_batches: Dict[str, SampleBatch], env_steps: int):
        self.policy_batches = policy_batches
        self._env_steps = env_steps
        self.fragment_shape = None

    def __getitem__(self, pid):
        return self.policy_batches[pid]

    def __contains__(self, pid):
        return pid in self.policy_batches

    def __len__(self):
        return self._env_steps

    @property
    def count(self):
        return self._env_steps

    def env_steps(self):
        return self._env_steps

    def agent_steps(self):
        return sum(b.count for b in self.policy_batches.values())

    @staticmethod
    def concat_samples(batches):
        pids = set()
        for b in batches:
            pids |= set(b.policy_batches)
        return MultiAgentBatch({p: concat_samples([b.policy_batches[p] for b in batches if p in b.policy_batches])
                                for p in pids}, sum(b.count for b in batches))


DEFAULT_POLICY_ID = "default_policy"
