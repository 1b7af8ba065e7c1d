"""Per-decision weighted importance sampling (reference:
``rllib/offline/estimators/weighted_importance_sampling.py:19``): each cumulative ratio p_t is
normalised by w_t, the mean of the p_t of all episodes of the batch (an episode that already ended
keeps its last ratio: absorbing, zero reward), so the estimate is
sum_t gamma^t sum_i p_it r_it / sum_i p_it -- biased, far lower variance than IS."""
from __future__ import annotations

import numpy as np

from ...policy.sample_batch import SampleBatch
from .importance_sampling import ImportanceSampling


class WeightedImportanceSampling(ImportanceSampling):
    def estimate_on_episodes(self, episodes):
        ps = [self._ratios(e) for e in episodes]
        rs = [np.asarray(e[SampleBatch.REWARDS], np.float64) for e in episodes]
        H = max(len(p) for p in ps)
        P = np.stack([np.concatenate([p, np.full(H - len(p), p[-1])]) for p in ps])
        R = np.stack([np.concatenate([r, np.zeros(H - len(r))]) for r in rs])
        w = np.maximum(P.mean(0), 1e-300)
        d = self._discounts(H)
        out = []
        for i in range(len(episodes)):
            n = len(rs[i])
            out.append({"v_behavior": float(np.sum(d[:n] * rs[i])), "v_target": float(np.sum(d * P[i] / w * R[i]))})
        return out

    def estimate_on_single_episode(self, episode):
        return self.estimate_on_episodes([episode])[0]
