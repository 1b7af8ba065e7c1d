"""Fitted Q Evaluation model (reference: ``rllib/offline/estimators/fqe_torch_model.py``): a
Q-network for the TARGET policy, fitted on logged transitions by iterating
Q(s, a) <- r + gamma (1 - terminated) sum_a' pi(a'|s') Q_target(s', a') (a target network
refreshed by Polyak averaging), the model behind DirectMethod and DoublyRobust."""
from __future__ import annotations

import copy
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from ...policy.sample_batch import SampleBatch


class FQETorchModel:
    def __init__(self, policy_probs, obs_dim: int, num_actions: int, gamma: float = 0.99, *,
                 hiddens=(64, 64), lr: float = 1e-3, n_iters: int = 1, minibatch_size: int = 128,
                 polyak_coef: float = 0.05, seed: Optional[int] = None):
        if seed is not None:
            torch.manual_seed(seed)
        self.policy_probs = policy_probs  # callable: obs [B, ...] -> pi(.|s) [B, A] (numpy)
        self.gamma = gamma
        self.n_iters, self.mb, self.tau = n_iters, minibatch_size, polyak_coef
        layers, d = [], obs_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), nn.ReLU()]
            d = h
        layers.append(nn.Linear(d, num_actions))
        self.q = nn.Sequential(*layers)
        self.q_target = copy.deepcopy(self.q)
        self.opt = torch.optim.Adam(self.q.parameters(), lr=lr)
        self.rng = np.random.default_rng(seed)

    def _x(self, obs):
        return torch.as_tensor(np.asarray(obs), dtype=torch.float32).reshape(len(obs), -1)

    def train(self, batch: SampleBatch) -> Dict[str, float]:
        obs, nobs = batch[SampleBatch.OBS], batch[SampleBatch.NEXT_OBS]
        a = torch.as_tensor(np.asarray(batch[SampleBatch.ACTIONS]).astype(np.int64))
        r = torch.as_tensor(np.asarray(batch[SampleBatch.REWARDS], np.float32))
        term = torch.as_tensor(np.asarray(batch[SampleBatch.TERMINATEDS], np.float32))
        pn = torch.as_tensor(self.policy_probs(nobs), dtype=torch.float32)
        x, xn = self._x(obs), self._x(nobs)
        n = len(r)
        losses = []
        for _ in range(self.n_iters):
            for idx in np.array_split(self.rng.permutation(n), max(1, n // self.mb)):
                i = torch.as_tensor(idx)
                with torch.no_grad():
                    v_next = (self.q_target(xn[i]) * pn[i]).sum(-1)
                    y = r[i] + self.gamma * (1 - term[i]) * v_next
                q = self.q(x[i]).gather(1, a[i].unsqueeze(1)).squeeze(1)
                loss = ((q - y) ** 2).mean()
                self.opt.zero_grad()
                loss.backward()
                self.opt.step()
                losses.append(float(loss))
                with torch.no_grad():
                    for pt, p in zip(self.q_target.parameters(), self.q.parameters()):
                        pt.mul_(1 - self.tau).add_(self.tau * p)
        return {"loss": float(np.mean(losses)) if losses else 0.0}

    @torch.no_grad()
    def estimate_q(self, obs, actions) -> np.ndarray:
        q = self.q(self._x(obs))
        a = torch.as_tensor(np.asarray(actions).astype(np.int64))
        return q.gather(1, a.unsqueeze(1)).squeeze(1).numpy()

    @torch.no_grad()
    def estimate_v(self, obs) -> np.ndarray:
        q = self.q(self._x(obs)).numpy()
        return (q * self.policy_probs(obs)).sum(-1)
