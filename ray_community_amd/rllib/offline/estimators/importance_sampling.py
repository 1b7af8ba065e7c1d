"""Per-decision importance sampling (reference: ``rllib/offline/estimators/importance_sampling.py:17``):
v_target = sum_t gamma^t p_t r_t with p_t = prod_{t' <= t} pi(a_t'|s_t') / mu(a_t'|s_t')."""
from __future__ import annotations

import numpy as np

from ...policy.sample_batch import SampleBatch
from .off_policy_estimator import OffPolicyEstimator


class ImportanceSampling(OffPolicyEstimator):
    def _ratios(self, episode):
        return np.cumprod(self.compute_action_probs(episode) / np.maximum(self.behavior_probs(episode), 1e-12))

    def estimate_on_single_episode(self, episode: SampleBatch):
        r = np.asarray(episode[SampleBatch.REWARDS], np.float64)
        d = self._discounts(len(r))
        p = self._ratios(episode)
        return {"v_behavior": float(np.sum(d * r)), "v_target": float(np.sum(d * p * r))}
