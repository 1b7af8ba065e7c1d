"""Doubly robust estimator (reference: ``rllib/offline/estimators/doubly_robust.py:28``): the
FQE model's value corrected, step by step from the end of the episode, by importance-weighted
residuals: v = V(s_t) + rho_t (r_t + gamma v - Q(s_t, a_t)), rho_t = pi(a_t|s_t) / mu(a_t|s_t)."""
from __future__ import annotations

import numpy as np

from ...policy.sample_batch import SampleBatch
from .direct_method import DirectMethod


class DoublyRobust(DirectMethod):
    def estimate_on_single_episode(self, episode: SampleBatch):
        m = self._ensure_model(episode)
        obs = np.asarray(episode[SampleBatch.OBS])
        r = np.asarray(episode[SampleBatch.REWARDS], np.float64)
        rho = self.compute_action_probs(episode) / np.maximum(self.behavior_probs(episode), 1e-12)
        q = m.estimate_q(obs, episode[SampleBatch.ACTIONS])
        v = m.estimate_v(obs)
        vt = 0.0
        for t in reversed(range(len(r))):
            vt = v[t] + rho[t] * (r[t] + self.gamma * vt - q[t])
        return {"v_behavior": float(np.sum(self._discounts(len(r)) * r)), "v_target": float(vt)}
