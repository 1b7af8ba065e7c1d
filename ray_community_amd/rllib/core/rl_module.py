"""RLModule + catalog for torch (reference: ``rllib/core/rl_module/torch``, ``rllib/core/models``).

Encoders: MLP for vector observations, Nature-CNN for 84x84 image stacks (uint8 HWC; the
uint8 -> float NCHW conversion runs as the ``image_normalize`` HIP kernel on GPU). Heads:
policy logits (Categorical) or mean/log-std (DiagGaussian), value head; optional Q head for DQN.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..utils.spaces import Box, Discrete
from .learner_api import MultiRLModuleAPI, RLModuleAPI, StatefulFlag


class Categorical:
    def __init__(self, logits):
        self.logits = logits - logits.logsumexp(-1, keepdim=True)

    def sample(self):
        return torch.multinomial(self.logits.exp(), 1).squeeze(-1)

    def deterministic_sample(self):
        return self.logits.argmax(-1)

    def logp(self, a):
        return self.logits.gather(-1, a.long().unsqueeze(-1)).squeeze(-1)

    def entropy(self):
        p = self.logits.exp()
        return -(p * self.logits).sum(-1)

    def kl(self, other):
        p = self.logits.exp()
        return (p * (self.logits - other.logits)).sum(-1)


class DiagGaussian:
    def __init__(self, inputs):
        self.mean, log_std = inputs.chunk(2, dim=-1)
        self.log_std = log_std.clamp(-20, 2)
        self.std = self.log_std.exp()

    def sample(self):
        return self.mean + self.std * torch.randn_like(self.mean)

    def deterministic_sample(self):
        return self.mean

    def logp(self, a):
        return (-0.5 * ((a - self.mean) / self.std) ** 2 - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)

    def entropy(self):
        return (self.log_std + 0.5 * math.log(2 * math.pi * math.e)).sum(-1)

    def kl(self, other):
        return (other.log_std - self.log_std + (self.std ** 2 + (self.mean - other.mean) ** 2) /
                (2.0 * other.std ** 2) - 0.5).sum(-1)


def _act(name):
    return {"tanh": nn.Tanh, "relu": nn.ReLU, "swish": nn.SiLU, "silu": nn.SiLU, "linear": nn.Identity,
            "elu": nn.ELU}[name]


def _mlp(inp, hiddens, act):
    layers = []
    d = inp
    for h in hiddens:
        layers += [nn.Linear(d, h), _act(act)()]
        d = h
    return nn.Sequential(*layers), d


class NatureCNN(nn.Module):
    def __init__(self, in_ch, out_dim=512):
        super().__init__()
        self.net = nn.Sequential(nn.Conv2d(in_ch, 32, 8, 4), nn.ReLU(), nn.Conv2d(32, 64, 4, 2), nn.ReLU(),
                                 nn.Conv2d(64, 64, 3, 1), nn.ReLU(), nn.Flatten(), nn.Linear(64 * 7 * 7, out_dim),
                                 nn.ReLU())
        self.out_dim = out_dim

    def forward(self, x):
        return self.net(x)


def preprocess_obs(obs: torch.Tensor, channels_last: bool = False) -> torch.Tensor:
    """uint8 [B, H, W, C] frames -> float [B, C, H, W] / 255 (one HIP kernel on GPU;
    ``channels_last``: written in NHWC memory, what a channels-last conv stack consumes)."""
    if obs.dtype == torch.uint8 and obs.dim() == 4:
        if obs.is_cuda:
            from ...ops import image_normalize

            C = obs.shape[-1]
            return image_normalize(obs, mean=(0.0,) * C, std=(1.0,) * C, dtype=torch.float32,
                                   channels_last=channels_last)
        return obs.permute(0, 3, 1, 2).float().div_(255.0)
    return obs.float()


class RLModule(RLModuleAPI, nn.Module):
    """Actor-critic module used by PPO/IMPALA/APPO (and DQN via ``q_head``)."""

    def __init__(self, observation_space, action_space, model_config: Optional[Dict] = None, q_head=False):
        super().__init__()
        cfg = dict(model_config or {})
        self.obs_space = observation_space
        self.act_space = action_space
        self.model_config = cfg
        hiddens = cfg.get("fcnet_hiddens", [256, 256])
        act = cfg.get("fcnet_activation", "tanh")
        self.vf_share = cfg.get("vf_share_layers", False)
        self.is_image = len(observation_space.shape) == 3
        if isinstance(action_space, Discrete):
            self.n_out = action_space.n
            self.dist_cls = Categorical
        else:
            self.n_out = 2 * int(np.prod(action_space.shape))
            self.dist_cls = DiagGaussian
        if self.is_image:
            self.encoder = NatureCNN(observation_space.shape[-1], cfg.get("conv_out", 512))
            feat = self.encoder.out_dim
            self.vf_encoder = None
            self.vf_share = True
        else:
            inp = int(np.prod(observation_space.shape))
            self.encoder, feat = _mlp(inp, hiddens, act)
            self.vf_encoder = None if self.vf_share else _mlp(inp, hiddens, act)[0]
        self.pi = nn.Linear(feat, self.n_out)
        self.vf = nn.Linear(feat, 1)
        self.q_head = nn.Linear(feat, self.n_out) if q_head else None
        nn.init.orthogonal_(self.pi.weight, 0.01)
        nn.init.zeros_(self.pi.bias)

    def _x(self, obs):
        if self.is_image:
            w = self.encoder.net[0].weight  # channels-last weights: feed NHWC frames (no MIOpen transposes)
            return preprocess_obs(obs, channels_last=w.is_cuda and w.stride(1) == 1 and w.shape[1] > 1)
        return preprocess_obs(obs).reshape(obs.shape[0], -1)

    def forward(self, obs):
        x = self._x(obs)
        h = self.encoder(x)
        logits = self.pi(h)
        hv = h if self.vf_encoder is None else self.vf_encoder(x)
        v = self.vf(hv).squeeze(-1)
        return logits, v

    def q_values(self, obs):
        h = self.encoder(self._x(obs))
        return self.q_head(h)

    def dist(self, logits):
        return self.dist_cls(logits)

    @torch.no_grad()
    def forward_inference(self, obs):
        logits, v = self.forward(obs)
        return self.dist(logits).deterministic_sample(), v

    @torch.no_grad()
    def forward_exploration(self, obs):
        logits, v = self.forward(obs)
        d = self.dist(logits)
        a = d.sample()
        return a, d.logp(a), v, logits

    def get_state(self):
        return {k: v.detach().to("cpu", copy=True) for k, v in self.state_dict().items()}

    def set_state(self, state):
        self.load_state_dict(state)


class RecurrentRLModule(RLModuleAPI, nn.Module):
    """LSTM actor-critic (reference: the new-stack default ``use_lstm`` encoder,
    ``rllib/core/models/torch/encoder.py`` TorchLSTMEncoder): MLP encoder -> LSTM cell -> policy and
    value heads. Stateful: the env runner carries one ``(h, c)`` row per sub-env (zeroed at episode
    starts) and records the state each step entered with; the learner replays ``max_seq_len``
    chunks from the recorded chunk-start states, zeroing the state inside a chunk where a new
    episode begins (``resets``), so training sees exactly the recurrence the rollout used."""

    is_stateful = StatefulFlag(1)

    def __init__(self, observation_space, action_space, model_config: Optional[Dict] = None):
        super().__init__()
        cfg = dict(model_config or {})
        self.obs_space, self.act_space = observation_space, action_space
        if len(observation_space.shape) == 3:
            raise ValueError("use_lstm over image observations is not supported; stack frames with "
                             "FrameStackingEnvToModule instead")
        if isinstance(action_space, Discrete):
            self.n_out, self.dist_cls = action_space.n, Categorical
        else:
            self.n_out, self.dist_cls = 2 * int(np.prod(action_space.shape)), DiagGaussian
        self.cell_size = int(cfg.get("lstm_cell_size", 256))
        self.max_seq_len = int(cfg.get("max_seq_len", 20))
        hiddens = cfg.get("fcnet_hiddens", [256, 256])
        inp = int(np.prod(observation_space.shape))
        self.encoder, feat = _mlp(inp, hiddens, cfg.get("fcnet_activation", "tanh"))
        self.lstm = nn.LSTMCell(feat, self.cell_size)
        self.pi = nn.Linear(self.cell_size, self.n_out)
        self.vf = nn.Linear(self.cell_size, 1)
        nn.init.orthogonal_(self.pi.weight, 0.01)
        nn.init.zeros_(self.pi.bias)

    # ------------------------------------------------------------------ state
    def get_initial_state(self, batch_size: int = 1, device=None):
        z = torch.zeros(batch_size, 2 * self.cell_size, device=device)
        return z

    def _cell(self, x, state):
        h, c = state[:, : self.cell_size], state[:, self.cell_size:]
        h, c = self.lstm(x, (h, c))
        return h, torch.cat([h, c], 1)

    # ------------------------------------------------------------------ rollout (one step)
    def forward_step(self, obs, state):
        x = preprocess_obs(obs).reshape(obs.shape[0], -1)
        h, new_state = self._cell(self.encoder(x), state.to(x.dtype))
        return self.pi(h), self.vf(h).squeeze(-1), new_state

    @torch.no_grad()
    def forward_exploration_step(self, obs, state):
        logits, v, st = self.forward_step(obs, state)
        d = self.dist(logits)
        a = d.sample()
        return a, d.logp(a), v, logits, st

    @torch.no_grad()
    def forward_inference_step(self, obs, state):
        logits, v, st = self.forward_step(obs, state)
        return self.dist(logits).deterministic_sample(), v, st

    # ------------------------------------------------------------------ training (sequences)
    def forward_seq(self, obs, state0, resets):
        """obs [B, L, ...], state0 [B, 2H], resets [B, L] (state zeroed BEFORE step t where set)
        -> logits [B, L, A], values [B, L]."""
        B, L = obs.shape[:2]
        x = self.encoder(preprocess_obs(obs).reshape(B, L, -1))
        st = state0.to(x.dtype)
        keep = (~resets.bool()).to(x.dtype).unsqueeze(-1)
        hs = []
        for t in range(L):
            st = st * keep[:, t]
            h, st = self._cell(x[:, t], st)
            hs.append(h)
        h = torch.stack(hs, 1)
        return self.pi(h), self.vf(h).squeeze(-1)

    def forward(self, obs, state=None, resets=None):
        """``resets`` given: the sequence form (``forward_seq``; what the learner calls, so a DDP
        wrapper sees it). Otherwise one step per row from ``state`` (default: a fresh state)."""
        if resets is not None:
            return self.forward_seq(obs, state, resets)
        st = self.get_initial_state(obs.shape[0], obs.device) if state is None else state
        logits, v, _ = self.forward_step(obs, st)
        return logits, v

    def dist(self, logits):
        return self.dist_cls(logits)

    def get_state(self):
        return {k: v.detach().to("cpu", copy=True) for k, v in self.state_dict().items()}

    def set_state(self, state):
        self.load_state_dict(state)


class RLModuleSpec:
    """How to build one RLModule (reference ``rllib/core/rl_module/rl_module.py`` RLModuleSpec):
    ``module_class(observation_space, action_space, model_config)``. A custom class subclasses
    ``RLModule`` (or implements its forward_* / get_state / set_state API)."""

    def __init__(self, module_class=None, observation_space=None, action_space=None, model_config=None,
                 model_config_dict=None, catalog_class=None, load_state_path=None):
        self.module_class = module_class
        self.observation_space = observation_space
        self.action_space = action_space
        self.model_config = dict(model_config or model_config_dict or {})
        self.catalog_class = catalog_class
        self.load_state_path = load_state_path

    def build(self, observation_space=None, action_space=None, base_model_config=None):
        cls = self.module_class or RLModule
        obs = self.observation_space or observation_space
        act = self.action_space or action_space
        if obs is None or act is None:
            raise ValueError("RLModuleSpec.build needs observation_space and action_space")
        m = cls(obs, act, {**dict(base_model_config or {}), **self.model_config})
        if self.load_state_path:
            m.load_state_dict(torch.load(self.load_state_path, weights_only=True))
        return m


SingleAgentRLModuleSpec = RLModuleSpec


class MultiRLModule(MultiRLModuleAPI, nn.Module):
    """Container of per-module RLModules (reference ``rllib/core/rl_module/marl_module.py:45``
    ``MultiAgentRLModule``): one RLModule per module (policy) id, registered as torch submodules
    (``parameters()`` / ``to()`` / ``state_dict()`` cover all of them). Dict-like access
    (``m[mid]``, ``in``, ``keys`` / ``values`` / ``items``, item assignment), ``add_module`` /
    ``remove_module``, ``foreach_module``; the forward passes take and return
    ``{module_id: ...}`` dicts, each module seeing only its own batch."""

    def __init__(self, rl_modules: Optional[Dict] = None):
        super().__init__()
        self._rl_modules = nn.ModuleDict()
        self._ids: list = []  # module ids in insertion order (ModuleDict keys must be strings)
        for mid, m in (rl_modules or {}).items():
            self.add_module(mid, m)

    # -------------------------------------------------------------- container API
    def add_module(self, module_id, module, *, override: bool = False):  # noqa: D401 (shadows nn.Module's)
        if not isinstance(module, nn.Module):
            return super().add_module(module_id, module)
        key = str(module_id)
        if module_id in self._ids and not override:
            raise ValueError(f"module {module_id!r} already exists (pass override=True to replace it)")
        self._rl_modules[key] = module
        if module_id not in self._ids:
            self._ids.append(module_id)
        return self

    def remove_module(self, module_id, *, raise_err_if_not_found: bool = True):
        if module_id not in self._ids:
            if raise_err_if_not_found:
                raise KeyError(f"no module {module_id!r}")
            return None
        self._ids.remove(module_id)
        return self._rl_modules.pop(str(module_id))

    def __getitem__(self, module_id):
        if module_id not in self._ids:
            raise KeyError(module_id)
        return self._rl_modules[str(module_id)]

    def __setitem__(self, module_id, module):
        self.add_module(module_id, module, override=True)

    def __contains__(self, module_id):
        return module_id in self._ids

    def __iter__(self):
        return iter(list(self._ids))

    def __len__(self):
        return len(self._ids)

    def keys(self):
        return list(self._ids)

    def values(self):
        return [self[m] for m in self._ids]

    def items(self):
        return [(m, self[m]) for m in self._ids]

    def pop(self, module_id, *default):
        if module_id not in self._ids and default:
            return default[0]
        return self.remove_module(module_id)

    def foreach_module(self, func):
        """[func(module_id, module)] over all modules."""
        return [func(mid, m) for mid, m in self.items()]

    # -------------------------------------------------------------- forward passes
    def _each(self, method: str, batch: Dict, *args):
        return {mid: getattr(self[mid], method)(b, *args) for mid, b in batch.items() if mid in self}

    def forward(self, batch: Dict):
        return self._each("forward", batch)

    def forward_inference(self, batch: Dict):
        return self._each("forward_inference", batch)

    def forward_exploration(self, batch: Dict):
        return self._each("forward_exploration", batch)

    def forward_train(self, batch: Dict):
        return self._each("forward", batch)

    # -------------------------------------------------------------- state
    def get_state(self, module_ids=None):
        ids = self._ids if module_ids is None else [m for m in module_ids if m in self]
        return {mid: self[mid].get_state() for mid in ids}

    def set_state(self, state: Dict):
        for mid, st in state.items():
            if mid in self:
                self[mid].set_state(st)

    def as_multi_agent(self):
        return self

    def __repr__(self):
        return f"MultiRLModule({', '.join(f'{m!r}: {type(self[m]).__name__}' for m in self._ids)})"


MultiAgentRLModule = MultiRLModule


class MultiRLModuleSpec:
    """{module_id: RLModuleSpec} for multi-agent algorithms (reference MultiRLModuleSpec); ``build``
    makes the ``MultiRLModule`` (or ``multi_rl_module_class``) holding every module."""

    def __init__(self, module_specs: Optional[Dict] = None, multi_rl_module_class=None, **kw):
        self.module_specs = dict(module_specs or {})
        self.multi_rl_module_class = multi_rl_module_class

    def build(self, module_id=None):
        if module_id is not None:
            return self.module_specs[module_id].build()
        cls = self.multi_rl_module_class or MultiRLModule
        return cls({mid: spec.build() for mid, spec in self.module_specs.items()})

    def add_modules(self, module_specs: Dict, override: bool = True):
        for mid, spec in module_specs.items():
            if mid in self.module_specs and not override:
                raise ValueError(f"module spec {mid!r} already exists")
            self.module_specs[mid] = spec


MultiAgentRLModuleSpec = MultiRLModuleSpec


def _spec_for(config: Dict, module_id):
    spec = config.get("rl_module_spec")
    if spec is None:
        return None
    if isinstance(spec, MultiRLModuleSpec):
        spec = spec.module_specs
    if isinstance(spec, dict):
        spec = spec.get(module_id if module_id is not None else config.get("_module_id"),
                        spec.get("default_policy"))
    return spec if isinstance(spec, RLModuleSpec) else None


def make_module(config: Dict, observation_space, action_space, module_id=None):
    """Module factory: an ``rl_module_spec`` with a custom ``module_class`` wins (per module id in
    multi-agent configs); else keyed by ``config['module_class']`` (``"actor_critic"`` default,
    ``"sac"``); ``model.use_lstm`` selects the recurrent actor-critic (PPO)."""
    spec = _spec_for(config, module_id)
    if spec is not None and spec.module_class is not None:
        return spec.build(observation_space, action_space, config.get("model"))
    kind = config.get("module_class", "actor_critic")
    model = config.get("model") or {}
    if kind == "sac":
        if model.get("use_lstm"):
            raise ValueError("use_lstm is supported for PPO (actor-critic modules) only")
        from .sac_module import SACModule

        return SACModule(observation_space, action_space, config.get("model"))
    if model.get("use_lstm"):
        if config.get("q_head") or config.get("_algo") not in (None, "PPO"):
            raise ValueError("use_lstm is supported for PPO only")
        return RecurrentRLModule(observation_space, action_space, model)
    return RLModule(observation_space, action_space, config.get("model"), q_head=config.get("q_head", False))
