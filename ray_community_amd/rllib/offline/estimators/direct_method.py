"""Direct method (reference: ``rllib/offline/estimators/direct_method.py:23``): the target policy's
value of each episode's first state under a fitted-Q-evaluation model,
v_target = sum_a pi(a|s_0) Q(s_0, a)."""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ...policy.sample_batch import SampleBatch
from .fqe_torch_model import FQETorchModel
from .off_policy_estimator import OffPolicyEstimator


class DirectMethod(OffPolicyEstimator):
    def __init__(self, policy, gamma: float = 0.99, epsilon_greedy: float = 0.0, q_model_config: Optional[Dict] = None):
        super().__init__(policy, gamma, epsilon_greedy)
        self._q_cfg = dict(q_model_config or {})
        self.model: Optional[FQETorchModel] = None

    def _ensure_model(self, batch):
        if self.model is None:
            obs = np.asarray(batch[SampleBatch.OBS])
            A = self.action_probs_all(obs[:1]).shape[-1]
            self.model = FQETorchModel(self.action_probs_all, int(np.prod(obs.shape[1:])), A, self.gamma,
                                       **self._q_cfg)
        return self.model

    def train(self, batch: SampleBatch) -> Dict:
        b = transitions(batch)
        return self._ensure_model(b).train(b)

    def estimate_on_single_episode(self, episode: SampleBatch):
        r = np.asarray(episode[SampleBatch.REWARDS], np.float64)
        v0 = float(self._ensure_model(episode).estimate_v(np.asarray(episode[SampleBatch.OBS])[:1])[0])
        return {"v_behavior": float(np.sum(self._discounts(len(r)) * r)), "v_target": v0}


def transitions(batch: SampleBatch) -> SampleBatch:
    """(s, a, r, s', terminated) rows of a logged batch. Env-major ``[N, T]`` fragments carry no
    ``new_obs``: it is the next step's observation of the same row; steps whose successor is not
    in the fragment (its last column, truncations: the next observation belongs to a new
    episode) are dropped, terminations kept (their successor is never used)."""
    fs = getattr(batch, "fragment_shape", None)
    if fs is None:
        if SampleBatch.NEXT_OBS not in batch:
            raise ValueError("fitting the FQE model needs new_obs in flat logged batches")
        return batch
    N, T = fs
    obs = np.asarray(batch[SampleBatch.OBS])
    term = np.asarray(batch[SampleBatch.TERMINATEDS], bool)
    trunc = np.asarray(batch.get(SampleBatch.TRUNCATEDS, np.zeros_like(term)), bool)
    keep = np.ones((N, T), bool)
    keep[:, -1] = term[:, -1]
    keep &= ~(trunc & ~term)
    nobs = np.concatenate([obs[:, 1:], obs[:, -1:]], axis=1)
    cols = {SampleBatch.OBS: obs, SampleBatch.NEXT_OBS: nobs, SampleBatch.ACTIONS: batch[SampleBatch.ACTIONS],
            SampleBatch.REWARDS: batch[SampleBatch.REWARDS], SampleBatch.TERMINATEDS: term}
    return SampleBatch({k: np.asarray(v)[keep] for k, v in cols.items()})
