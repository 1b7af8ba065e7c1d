"""SAC networks (reference: ``rllib/algorithms/sac/torch/sac_torch_rl_module.py``,
``sac_catalog.py``): tanh-squashed Gaussian policy, twin Q critics with Polyak-averaged targets,
learnable entropy temperature."""
from __future__ import annotations

import copy
import math
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn as nn

from ..utils.spaces import Box
from .rl_module import _mlp

LOG_STD_MIN, LOG_STD_MAX = -20.0, 2.0


class SACModule(nn.Module):
    def __init__(self, observation_space, action_space, model_config: Optional[Dict] = None, **_):
        super().__init__()
        if not isinstance(action_space, Box):
            raise ValueError("SAC here supports continuous (Box) action spaces")
        cfg = dict(model_config or {})
        hid = cfg.get("fcnet_hiddens", [256, 256])
        act = cfg.get("fcnet_activation", "relu")
        self.obs_dim = int(np.prod(observation_space.shape))
        self.act_dim = int(np.prod(action_space.shape))
        self.register_buffer("a_low", torch.as_tensor(action_space.low, dtype=torch.float32).reshape(-1))
        self.register_buffer("a_high", torch.as_tensor(action_space.high, dtype=torch.float32).reshape(-1))
        body, d = _mlp(self.obs_dim, hid, act)
        self.pi = nn.Sequential(body, nn.Linear(d, 2 * self.act_dim))
        q1, dq = _mlp(self.obs_dim + self.act_dim, hid, act)
        q2, _ = _mlp(self.obs_dim + self.act_dim, hid, act)
        self.q1 = nn.Sequential(q1, nn.Linear(dq, 1))
        self.q2 = nn.Sequential(q2, nn.Linear(dq, 1))
        self.q1_t = copy.deepcopy(self.q1)
        self.q2_t = copy.deepcopy(self.q2)
        for p in list(self.q1_t.parameters()) + list(self.q2_t.parameters()):
            p.requires_grad_(False)
        self.log_alpha = nn.Parameter(torch.tensor(math.log(float(cfg.get("initial_alpha", 1.0)))))
        self.dist_cls = None  # marks the SAC module for the env runner

    # ------------------------------------------------------------------ policy
    def _scale(self, u):  # [-1, 1] -> action bounds
        return self.a_low + (u + 1.0) * 0.5 * (self.a_high - self.a_low)

    def _unscale(self, a):
        return 2.0 * (a - self.a_low) / (self.a_high - self.a_low) - 1.0

    def policy(self, obs, deterministic=False):
        """Returns (squashed action in [-1, 1], log-prob)."""
        x = obs.float().reshape(obs.shape[0], -1)
        mean, log_std = self.pi(x).chunk(2, -1)
        log_std = log_std.clamp(LOG_STD_MIN, LOG_STD_MAX)
        std = log_std.exp()
        z = mean if deterministic else mean + std * torch.randn_like(mean)
        u = torch.tanh(z)
        logp = (-0.5 * ((z - mean) / std) ** 2 - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        logp = logp - (2 * (math.log(2.0) - z - nn.functional.softplus(-2 * z))).sum(-1)
        return u, logp

    def logp_of(self, obs, u):
        """Log-prob of given squashed actions ``u`` in (-1, 1) under the current policy (the
        tanh-Gaussian density through atanh; used by CQL's behaviour-cloning warm-up)."""
        x = obs.float().reshape(obs.shape[0], -1)
        mean, log_std = self.pi(x).chunk(2, -1)
        log_std = log_std.clamp(LOG_STD_MIN, LOG_STD_MAX)
        u = u.clamp(-1 + 1e-6, 1 - 1e-6)
        z = torch.atanh(u)
        logp = (-0.5 * ((z - mean) / log_std.exp()) ** 2 - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        return logp - (2 * (math.log(2.0) - z - nn.functional.softplus(-2 * z))).sum(-1)

    def q(self, obs, u, target=False):
        x = torch.cat([obs.float().reshape(obs.shape[0], -1), u], -1)
        if target:
            return self.q1_t(x).squeeze(-1), self.q2_t(x).squeeze(-1)
        return self.q1(x).squeeze(-1), self.q2(x).squeeze(-1)

    @torch.no_grad()
    def forward(self, obs):
        """(deterministic action, V(s) ~ min_i Q_i(s, mu(s))) — the value head on-policy samplers
        bootstrap from."""
        u, _ = self.policy(obs, deterministic=True)
        return self._scale(u), torch.min(*self.q(obs, u))

    @torch.no_grad()
    def forward_inference(self, obs):
        u, _ = self.policy(obs, deterministic=True)
        return self._scale(u), torch.zeros(obs.shape[0])

    @torch.no_grad()
    def forward_exploration(self, obs):
        u, lp = self.policy(obs)
        return self._scale(u), lp, torch.zeros(obs.shape[0]), None

    @torch.no_grad()
    def polyak(self, tau: float):
        for src, dst in ((self.q1, self.q1_t), (self.q2, self.q2_t)):
            for p, pt in zip(src.parameters(), dst.parameters()):
                pt.mul_(1 - tau).add_(p, alpha=tau)

    def get_state(self):
        return {k: v.detach().cpu() for k, v in self.state_dict().items()}

    def set_state(self, state):
        self.load_state_dict(state)
