"""DreamerV3 (reference: ``rllib/algorithms/dreamerv3/`` — ``dreamerv3.py`` config/algorithm,
``dreamerv3_learner.py`` losses, ``utils/`` symlog / two-hot; Hafner et al. 2023, "Mastering
Diverse Domains through World Models").

A world model learns from replayed sequences and the actor-critic learns purely in imagination:

* world model — MLP encoder of symlog(obs); RSSM with a GRU deterministic state ``h`` and a
  categorical stochastic state ``z`` (``num_categoricals`` x ``num_classes``, 1 % uniform mix,
  straight-through samples); decoder (symlog MSE), reward head (two-hot over 255 symlog bins),
  continue head (Bernoulli); loss = pred + 0.5 * max(1, KL[sg(post) || prior]) +
  0.1 * max(1, KL[post || sg(prior)]) (free bits 1 nat);
* imagination — from every posterior state of the batch, ``horizon_H`` steps of actor samples
  through the prior; lambda-returns over predicted rewards/continues and the critic;
* actor — REINFORCE on (R - v) / max(1, S) plus ``entropy_scale`` * entropy, S an EMA
  (``return_normalization_decay``) of the 5th-95th percentile range of the returns (the
  reference backpropagates through the dynamics for continuous actions; here both action kinds
  use the score-function estimator);
* critic — two-hot cross-entropy to symlog(R) plus a regulariser toward its own EMA.

Acting runs in the driver's vectorised env (``num_envs_per_env_runner`` sub-envs, per-sub-env
RSSM state); sequences live in a per-sub-env ring replay. ``training_ratio`` = replayed steps
per env step (reference semantics): each ``train()`` samples ``env_steps_per_iteration`` steps
and runs ``training_ratio * steps / (B * T)`` updates. Runs on the GPU when
``resources(num_gpus>0)``.
"""
from __future__ import annotations

import copy
import os
import pickle
from typing import Dict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .algorithm import Algorithm
from .algorithm_config import AlgorithmConfig

# (dense units, MLP layers, GRU units, num_categoricals, num_classes) — reference model sizes, plus
# an extra-small "nano" used by tests
MODEL_SIZES = {
    "nano": (64, 1, 64, 4, 4),
    "micro": (128, 1, 128, 8, 8),
    "mini": (192, 1, 192, 16, 16),
    "XS": (256, 1, 256, 32, 32),
    "S": (512, 2, 512, 32, 32),
    "M": (640, 3, 1024, 32, 32),
    "L": (768, 4, 2048, 32, 32),
    "XL": (1024, 5, 4096, 32, 32),
}
NUM_BINS = 255


def symlog(x):
    return torch.sign(x) * torch.log1p(x.abs())


def symexp(x):
    return torch.sign(x) * torch.expm1(x.abs())


class TwoHot:
    """Two-hot targets over ``NUM_BINS`` equally spaced bins in symlog space [-20, 20]."""

    def __init__(self, device):
        self.bins = torch.linspace(-20.0, 20.0, NUM_BINS, device=device)

    def encode(self, y):  # y: symlog-space targets [...]
        y = y.clamp(-20.0, 20.0)
        k = (torch.searchsorted(self.bins, y.contiguous(), right=True) - 1).clamp(0, NUM_BINS - 2)
        lo, hi = self.bins[k], self.bins[k + 1]
        w = ((y - lo) / (hi - lo)).clamp(0.0, 1.0)
        t = torch.zeros(y.shape + (NUM_BINS,), device=y.device)
        t.scatter_(-1, k.unsqueeze(-1), (1 - w).unsqueeze(-1))
        t.scatter_add_(-1, (k + 1).unsqueeze(-1), w.unsqueeze(-1))
        return t

    def decode(self, logits):  # -> real-space value
        return symexp((logits.softmax(-1) * self.bins).sum(-1))

    def loss(self, logits, y_real):
        return -(self.encode(symlog(y_real)) * logits.log_softmax(-1)).sum(-1)


def mlp(inp, units, layers, out=None, zero_out=False):
    mods, d = [], inp
    for _ in range(layers):
        mods += [nn.Linear(d, units, bias=False), nn.LayerNorm(units), nn.SiLU()]
        d = units
    if out is not None:
        lin = nn.Linear(d, out)
        if zero_out:
            nn.init.zeros_(lin.weight)
            nn.init.zeros_(lin.bias)
        mods.append(lin)
    return nn.Sequential(*mods)


class WorldModel(nn.Module):
    def __init__(self, obs_dim, act_dim, units, layers, gru, C, K):
        super().__init__()
        self.C, self.K, self.gru_units, self.act_dim = C, K, gru, act_dim
        self.z_dim = C * K
        self.encoder = mlp(obs_dim, units, max(1, layers))
        self.img_in = mlp(self.z_dim + act_dim, units, 1)
        self.gru = nn.GRUCell(units, gru)
        self.prior = mlp(gru, units, 1, self.z_dim)
        self.post = mlp(gru + units, units, 1, self.z_dim)
        feat = gru + self.z_dim
        self.decoder = mlp(feat, units, max(1, layers), obs_dim)
        self.reward = mlp(feat, units, max(1, layers), NUM_BINS, zero_out=True)
        self.cont = mlp(feat, units, max(1, layers), 1)

    def dist_probs(self, logits):
        p = logits.view(*logits.shape[:-1], self.C, self.K).softmax(-1)
        return 0.99 * p + 0.01 / self.K

    def sample(self, probs):
        idx = torch.distributions.Categorical(probs=probs).sample()
        onehot = F.one_hot(idx, self.K).float()
        return (onehot + probs - probs.detach()).flatten(-2)  # straight-through

    def step_h(self, h, z, a):
        return self.gru(self.img_in(torch.cat([z, a], -1)), h)

    def observe(self, h, embed):
        probs = self.dist_probs(self.post(torch.cat([h, embed], -1)))
        return self.sample(probs), probs

    def imagine_z(self, h):
        probs = self.dist_probs(self.prior(h))
        return self.sample(probs), probs


class ActorCritic(nn.Module):
    def __init__(self, feat, act_dim, discrete, units, layers):
        super().__init__()
        self.discrete = discrete
        self.actor = mlp(feat, units, max(1, layers), act_dim if discrete else 2 * act_dim)
        self.critic = mlp(feat, units, max(1, layers), NUM_BINS, zero_out=True)

    def policy(self, feat):
        out = self.actor(feat)
        if self.discrete:
            p = 0.99 * out.softmax(-1) + 0.01 / out.shape[-1]
            return torch.distributions.Categorical(probs=p)
        mean, std = out.chunk(2, -1)
        std = 0.9 * torch.sigmoid(std + 2.0) + 0.1
        return torch.distributions.Independent(torch.distributions.Normal(torch.tanh(mean), std), 1)


class SequenceReplay:
    """Per-sub-env ring buffers of rows (obs_t, a_{t-1}, r_t, is_first_t, is_terminal_t), one write
    pointer per stream (a finished episode adds its terminal row to its own stream only)."""

    def __init__(self, n_streams, capacity, obs_dim, act_dim, seed=None):
        self.n, self.cap = n_streams, capacity
        self.obs = np.zeros((n_streams, capacity, obs_dim), np.float32)
        self.act = np.zeros((n_streams, capacity, act_dim), np.float32)
        self.rew = np.zeros((n_streams, capacity), np.float32)
        self.first = np.zeros((n_streams, capacity), bool)
        self.term = np.zeros((n_streams, capacity), bool)
        self.pos = np.zeros(n_streams, np.int64)
        self.sizes = np.zeros(n_streams, np.int64)
        self.rng = np.random.default_rng(seed)

    @property
    def size(self) -> int:
        return int(self.sizes.min())

    def add(self, streams, obs, prev_act, rew, first, term):
        p = self.pos[streams]
        self.obs[streams, p], self.act[streams, p], self.rew[streams, p] = obs, prev_act, rew
        self.first[streams, p], self.term[streams, p] = first, term
        self.pos[streams] = (p + 1) % self.cap
        self.sizes[streams] = np.minimum(self.sizes[streams] + 1, self.cap)

    def sample(self, B, T):
        ok = np.nonzero(self.sizes >= T)[0]
        s = ok[self.rng.integers(0, len(ok), B)]
        st = (self.rng.random(B) * (self.sizes[s] - T + 1)).astype(np.int64)
        full = self.sizes[s] == self.cap
        st = np.where(full, (st + self.pos[s]) % self.cap, st)  # full ring: offset from the oldest row
        idx = (st[:, None] + np.arange(T)[None]) % self.cap
        out = {k: getattr(self, k)[s[:, None], idx] for k in ("obs", "act", "rew", "first", "term")}
        out["first"][:, 0] = True  # every window starts from a fresh state
        return out


class DreamerV3Config(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class=algo_class or DreamerV3)
        self.model_size = "XS"
        self.training_ratio = 1024
        self.replay_buffer_config = {"type": "EpisodeReplayBuffer", "capacity": int(1e6)}
        self.world_model_lr = 1e-4
        self.actor_lr = 3e-5
        self.critic_lr = 3e-5
        self.batch_size_B = 16
        self.batch_length_T = 64
        self.horizon_H = 15
        self.gae_lambda = 0.95
        self.entropy_scale = 3e-4
        self.return_normalization_decay = 0.99
        self.train_critic = True
        self.train_actor = True
        self.world_model_grad_clip_by_global_norm = 1000.0
        self.critic_grad_clip_by_global_norm = 100.0
        self.actor_grad_clip_by_global_norm = 100.0
        self.symlog_obs = "auto"
        self.gamma = 0.997
        self.env_steps_per_iteration = 256
        self.num_steps_sampled_before_learning_starts = 512
        self.critic_ema_decay = 0.98
        self.num_env_runners = 0
        self.num_envs_per_env_runner = 4

    def training(self, **kw):
        for k in ("model_size", "training_ratio", "batch_size_B", "batch_length_T", "horizon_H", "gae_lambda",
                  "entropy_scale", "return_normalization_decay", "train_critic", "train_actor", "world_model_lr",
                  "actor_lr", "critic_lr", "world_model_grad_clip_by_global_norm", "critic_grad_clip_by_global_norm",
                  "actor_grad_clip_by_global_norm", "symlog_obs", "env_steps_per_iteration", "critic_ema_decay",
                  "num_steps_sampled_before_learning_starts"):
            if k in kw:
                setattr(self, k, kw.pop(k))
        if "replay_buffer_config" in kw:
            self.replay_buffer_config = {**self.replay_buffer_config, **kw.pop("replay_buffer_config")}
        return super().training(**kw)


class _Metrics:
    def __init__(self):
        self.new_episodes = []

    def get_metrics(self):
        eps, self.new_episodes = self.new_episodes, []
        return {"episodes": eps, "custom_metrics": []}


class DreamerV3(Algorithm):
    _default_config_cls = DreamerV3Config

    @classmethod
    def get_default_config(cls):
        return DreamerV3Config()

    def setup(self, config):
        from ..._private import worker as w
        from ..env.envs import make_vector_env

        if not w.is_initialized():
            w.init()
        if isinstance(config, dict):
            self.config = self._default_config_cls().update_from_dict(config)
        cfg = self.config
        if cfg.seed is not None:
            torch.manual_seed(int(cfg.seed))
        self.device = torch.device("cuda") if (cfg.num_gpus or 0) > 0 and torch.cuda.is_available() else \
            torch.device("cpu")
        self.env = make_vector_env(cfg.env, cfg.num_envs_per_env_runner, cfg.env_config, seed=cfg.seed)
        self.N = self.env.num_envs
        osp, asp = self.env.observation_space, self.env.action_space
        self.obs_space, self.act_space = osp, asp
        self.obs_dim = int(np.prod(osp.shape))
        self.discrete = hasattr(asp, "n")
        self.act_dim = int(asp.n) if self.discrete else int(np.prod(asp.shape))
        units, layers, gru, C, K = MODEL_SIZES[cfg.model_size]
        self.wm = WorldModel(self.obs_dim, self.act_dim, units, layers, gru, C, K).to(self.device)
        self.ac = ActorCritic(gru + C * K, self.act_dim, self.discrete, units, layers).to(self.device)
        self.critic_ema = copy.deepcopy(self.ac.critic).requires_grad_(False)
        self.opt_wm = torch.optim.Adam(self.wm.parameters(), lr=cfg.world_model_lr, eps=1e-8)
        self.opt_actor = torch.optim.Adam(self.ac.actor.parameters(), lr=cfg.actor_lr, eps=1e-5)
        self.opt_critic = torch.optim.Adam(self.ac.critic.parameters(), lr=cfg.critic_lr, eps=1e-5)
        self.twohot = TwoHot(self.device)
        self.symlog_obs = cfg.symlog_obs if isinstance(cfg.symlog_obs, bool) else True
        cap = max(cfg.batch_length_T + 1, int(cfg.replay_buffer_config.get("capacity", 1e6)) // self.N)
        self.replay = SequenceReplay(self.N, cap, self.obs_dim, self.act_dim, seed=cfg.seed)
        self.ret_scale = None
        self._updates = 0
        self._metrics = _Metrics()
        self.local_runner = self._metrics  # base train() collects episodes through get_metrics()
        self.remote_runners = []
        self.obs, _ = self.env.reset(seed=cfg.seed)
        self._reset_act_state(np.ones(self.N, bool))
        self.ep_ret = np.zeros(self.N)
        self.ep_len = np.zeros(self.N, np.int64)
        self._first = np.ones(self.N, bool)
        self._last_r = np.zeros(self.N, np.float32)
        self._rng = np.random.default_rng(cfg.seed)
        from .callbacks import build as _build_callbacks

        self.callbacks = _build_callbacks(getattr(cfg, "_callbacks", None))
        self._custom_metrics = []
        if self.callbacks is not None:
            self.callbacks.on_algorithm_init(algorithm=self)

    # ------------------------------------------------------------------ acting
    def _reset_act_state(self, mask):
        dev = self.device
        if not hasattr(self, "_h"):
            self._h = torch.zeros(self.N, self.wm.gru_units, device=dev)
            self._z = torch.zeros(self.N, self.wm.z_dim, device=dev)
            self._a = torch.zeros(self.N, self.act_dim, device=dev)
        m = torch.as_tensor(mask, device=dev)
        self._h[m] = 0
        self._z[m] = 0
        self._a[m] = 0

    def _prep_obs(self, obs):
        o = torch.as_tensor(np.asarray(obs, np.float32).reshape(len(obs), -1), device=self.device)
        return symlog(o) if self.symlog_obs else o

    def _encode_act(self, a):
        if self.discrete:
            return F.one_hot(torch.as_tensor(a, device=self.device).long(), self.act_dim).float()
        return torch.as_tensor(np.asarray(a, np.float32).reshape(len(a), -1), device=self.device)

    def _env_action(self, a_t):
        if self.discrete:
            return a_t.cpu().numpy().astype(np.int64)
        lo, hi = self.act_space.low, self.act_space.high
        a = a_t.clamp(-1, 1).cpu().numpy()
        return (lo + (a + 1.0) * 0.5 * (hi - lo)).astype(np.float32)

    @torch.no_grad()
    def _act(self, obs, explore=True, random=False):
        h = self.wm.step_h(self._h, self._z, self._a)
        z, _ = self.wm.observe(h, self.wm.encoder(self._prep_obs(obs)))
        feat = torch.cat([h, z], -1)
        if random:
            if self.discrete:
                a = torch.as_tensor(self._rng.integers(0, self.act_dim, self.N), device=self.device)
            else:
                a = torch.as_tensor(self._rng.uniform(-1, 1, (self.N, self.act_dim)), device=self.device).float()
        else:
            d = self.ac.policy(feat)
            if explore:
                a = d.sample()
            elif self.discrete:
                a = d.probs.argmax(-1)
            else:
                a = d.base_dist.mean
        self._h, self._z = h, z
        self._a = F.one_hot(a.long(), self.act_dim).float() if self.discrete else a.float()
        return a

    def _sample_env(self, steps):
        random = self._timesteps_total < self.config.num_steps_sampled_before_learning_starts
        allstreams = np.arange(self.N)
        for _ in range(max(1, steps // self.N)):
            # row for the current observation: the action and reward that led to it
            self.replay.add(allstreams, np.asarray(self.obs, np.float32).reshape(self.N, -1), self._a.cpu().numpy(),
                            self._last_r, self._first, np.zeros(self.N, bool))
            a = self._act(self.obs, explore=True, random=random)
            nobs, r, te, tr, info = self.env.step(self._env_action(a))
            r = np.asarray(r, np.float32)
            self.ep_ret += r
            self.ep_len += 1
            done = np.asarray(te | tr, bool)
            self._last_r, self._first = r, np.zeros(self.N, bool)
            if done.any():
                idx = np.nonzero(done)[0]
                fin = np.asarray(info["final_obs"], np.float32).reshape(self.N, -1)[idx]
                # terminal row of each finished stream, then its next episode starts fresh
                self.replay.add(idx, fin, self._a[torch.as_tensor(idx, device=self.device)].cpu().numpy(), r[idx],
                                np.zeros(len(idx), bool), np.asarray(te, bool)[idx])
                for i in idx:
                    self._metrics.new_episodes.append((float(self.ep_ret[i]), int(self.ep_len[i])))
                self.ep_ret[done] = 0
                self.ep_len[done] = 0
                self._first = done.copy()
                self._last_r = np.where(done, 0.0, r).astype(np.float32)
                self._reset_act_state(done)
            self.obs = nobs
            self._timesteps_total += self.N

    # ------------------------------------------------------------------ learning
    def _update(self) -> Dict:
        cfg = self.config
        B, T, H = cfg.batch_size_B, cfg.batch_length_T, cfg.horizon_H
        d = self.replay.sample(B, T)
        dev = self.device
        obs = torch.as_tensor(d["obs"], device=dev)
        obs_in = symlog(obs) if self.symlog_obs else obs
        act = torch.as_tensor(d["act"], device=dev)
        rew = torch.as_tensor(d["rew"], device=dev)
        first = torch.as_tensor(d["first"], device=dev)
        term = torch.as_tensor(d["term"], device=dev).float()
        wm = self.wm
        embed = wm.encoder(obs_in)
        h = torch.zeros(B, wm.gru_units, device=dev)
        z = torch.zeros(B, wm.z_dim, device=dev)
        hs, zs, posts, priors = [], [], [], []
        for t in range(T):
            keep = (~first[:, t]).float().unsqueeze(-1)
            h, z, a_prev = h * keep, z * keep, act[:, t] * keep
            h = wm.step_h(h, z, a_prev)
            prior_p = wm.dist_probs(wm.prior(h))
            z, post_p = wm.observe(h, embed[:, t])
            hs.append(h)
            zs.append(z)
            posts.append(post_p)
            priors.append(prior_p)
        h_all, z_all = torch.stack(hs, 1), torch.stack(zs, 1)
        post_p, prior_p = torch.stack(posts, 1), torch.stack(priors, 1)
        feat = torch.cat([h_all, z_all], -1)
        dec_loss = (wm.decoder(feat) - (symlog(obs) if self.symlog_obs else obs)).pow(2).sum(-1)
        rew_loss = self.twohot.loss(wm.reward(feat), rew)
        cont_loss = F.binary_cross_entropy_with_logits(wm.cont(feat).squeeze(-1), 1.0 - term, reduction="none")

        def kl(p, q):
            return (p * (p.log() - q.log())).sum(-1).sum(-1)

        dyn = kl(post_p.detach(), prior_p).clamp(min=1.0)
        rep = kl(post_p, prior_p.detach()).clamp(min=1.0)
        wm_loss = (dec_loss + rew_loss + cont_loss + 0.5 * dyn + 0.1 * rep).mean()
        self.opt_wm.zero_grad(set_to_none=True)
        wm_loss.backward()
        gn_wm = nn.utils.clip_grad_norm_(wm.parameters(), cfg.world_model_grad_clip_by_global_norm)
        self.opt_wm.step()

        # ---- imagination from every posterior state
        with torch.no_grad():
            h = h_all.reshape(B * T, -1).detach()
            z = z_all.reshape(B * T, -1).detach()
            c0 = (1.0 - term).reshape(B * T)
        feats, acts = [torch.cat([h, z], -1)], []
        for _ in range(H):
            with torch.no_grad():
                a = self.ac.policy(feats[-1]).sample()
                a_in = F.one_hot(a.long(), self.act_dim).float() if self.discrete else a
                h = wm.step_h(h, z, a_in)
                z, _ = wm.imagine_z(h)
            acts.append(a)
            feats.append(torch.cat([h, z], -1).detach())
        fs = torch.stack(feats, 0)  # [H+1, BT, F]
        with torch.no_grad():
            r_im = self.twohot.decode(wm.reward(fs[1:]))
            c_im = torch.sigmoid(wm.cont(fs[1:]).squeeze(-1))
            cont = torch.cat([c0.unsqueeze(0), c_im], 0)  # [H+1, BT]
            v = self.twohot.decode(self.ac.critic(fs))
            ret = [v[-1]]
            g, lam = cfg.gamma, cfg.gae_lambda
            for t in reversed(range(H)):
                ret.append(r_im[t] + g * cont[t + 1] * ((1 - lam) * v[t + 1] + lam * ret[-1]))
            R = torch.stack(ret[::-1][:-1], 0)  # [H, BT] returns for states 0..H-1
            w = torch.cumprod(torch.cat([torch.ones_like(cont[:1]), g * cont[1:-1]], 0), 0)  # [H, BT]
            lo, hi = torch.quantile(R.flatten().float(), torch.tensor([0.05, 0.95], device=dev))
            rng = (hi - lo).item()
            dcy = cfg.return_normalization_decay
            self.ret_scale = rng if self.ret_scale is None else dcy * self.ret_scale + (1 - dcy) * rng
            scale = max(1.0, self.ret_scale)
            adv = (R - v[:-1]) / scale
        out = {"world_model_loss": float(wm_loss.detach()), "decoder_loss": float(dec_loss.detach().mean()),
               "reward_loss": float(rew_loss.detach().mean()), "continue_loss": float(cont_loss.detach().mean()),
               "dyn_kl": float(dyn.detach().mean()), "rep_kl": float(rep.detach().mean()), "wm_grad_norm": float(gn_wm),
               "return_scale": scale, "imagined_return_mean": float(R.mean())}
        if cfg.train_actor:
            dist = self.ac.policy(fs[:-1])
            a_stack = torch.stack(acts, 0)
            logp = dist.log_prob(a_stack)
            ent = dist.entropy()
            actor_loss = -(w * (logp * adv + cfg.entropy_scale * ent)).mean()
            self.opt_actor.zero_grad(set_to_none=True)
            actor_loss.backward()
            nn.utils.clip_grad_norm_(self.ac.actor.parameters(), cfg.actor_grad_clip_by_global_norm)
            self.opt_actor.step()
            out.update(actor_loss=float(actor_loss.detach()), entropy=float(ent.detach().mean()))
        if cfg.train_critic:
            logits = self.ac.critic(fs[:-1])
            with torch.no_grad():
                ema_t = self.critic_ema(fs[:-1]).softmax(-1)
            crit = self.twohot.loss(logits, R) - (ema_t * logits.log_softmax(-1)).sum(-1)
            critic_loss = (w * crit).mean()
            self.opt_critic.zero_grad(set_to_none=True)
            critic_loss.backward()
            nn.utils.clip_grad_norm_(self.ac.critic.parameters(), cfg.critic_grad_clip_by_global_norm)
            self.opt_critic.step()
            with torch.no_grad():
                dcy = cfg.critic_ema_decay
                for pe, p in zip(self.critic_ema.parameters(), self.ac.critic.parameters()):
                    pe.mul_(dcy).add_(p, alpha=1 - dcy)
            out["critic_loss"] = float(critic_loss.detach())
        self._updates += 1
        return out

    def training_step(self) -> Dict:
        cfg = self.config
        steps = max(self.N, int(cfg.env_steps_per_iteration))
        before = self._timesteps_total
        self._sample_env(steps)
        sampled = self._timesteps_total - before
        info: Dict = {}
        if self._timesteps_total >= cfg.num_steps_sampled_before_learning_starts and \
                self.replay.size > cfg.batch_length_T:
            n_upd = max(1, int(round(sampled * cfg.training_ratio / (cfg.batch_size_B * cfg.batch_length_T))))
            for _ in range(n_upd):
                info = self._update()
        info["num_updates_total"] = self._updates
        info["_steps_this_iter"] = sampled
        return info

    # ------------------------------------------------------------------ API overrides
    def _evaluate(self) -> Dict:
        cfg = self.config
        from ..env.envs import make_vector_env

        env = make_vector_env(cfg.env, 1, cfg.env_config, seed=(cfg.seed or 0) + 99991)
        rets = []
        saved = (self._h, self._z, self._a, self.N)
        self.N = 1
        del self._h  # _reset_act_state re-creates the acting state for one env
        self._reset_act_state(np.ones(1, bool))
        obs, _ = env.reset()
        ret, guard = 0.0, 0
        while len(rets) < cfg.evaluation_duration and guard < 100000:
            a = self._act(obs, explore=False)
            obs, r, te, tr, info = env.step(self._env_action(a))
            ret += float(r[0])
            guard += 1
            if te[0] or tr[0]:
                rets.append(ret)
                ret = 0.0
                self._reset_act_state(np.ones(1, bool))
        self._h, self._z, self._a, self.N = saved
        m = float(np.mean(rets)) if rets else float("nan")
        return {"episode_reward_mean": m, "env_runners": {"episode_return_mean": m}, "num_episodes": len(rets)}

    def compute_single_action(self, observation, explore: bool = False, state=None, **kw):
        """Stateless convenience: one posterior step from a zero RSSM state."""
        with torch.no_grad():
            h = self.wm.step_h(torch.zeros(1, self.wm.gru_units, device=self.device),
                               torch.zeros(1, self.wm.z_dim, device=self.device),
                               torch.zeros(1, self.act_dim, device=self.device))
            z, _ = self.wm.observe(h, self.wm.encoder(self._prep_obs(np.asarray(observation)[None])))
            d = self.ac.policy(torch.cat([h, z], -1))
            a = d.sample() if explore else (d.probs.argmax(-1) if self.discrete else d.base_dist.mean)
        a = self._env_action(a)[0]
        return int(a) if self.discrete else a

    def get_weights(self):
        return {"world_model": {k: v.cpu() for k, v in self.wm.state_dict().items()},
                "actor_critic": {k: v.cpu() for k, v in self.ac.state_dict().items()}}

    def set_weights(self, w):
        self.wm.load_state_dict(w["world_model"])
        self.ac.load_state_dict(w["actor_critic"])

    def save_checkpoint(self, checkpoint_dir: str):
        import json

        os.makedirs(checkpoint_dir, exist_ok=True)
        st = {"weights": self.get_weights(), "critic_ema": {k: v.cpu() for k, v in self.critic_ema.state_dict().items()},
              "opt": [o.state_dict() for o in (self.opt_wm, self.opt_actor, self.opt_critic)],
              "iteration": self._iteration, "timesteps_total": self._timesteps_total, "ret_scale": self.ret_scale,
              "updates": self._updates, "config": self.config.to_dict()}
        with open(os.path.join(checkpoint_dir, "algorithm_state.pkl"), "wb") as f:
            pickle.dump(st, f)
        with open(os.path.join(checkpoint_dir, "rllib_checkpoint.json"), "w") as f:
            json.dump({"type": "Algorithm", "algo": "DreamerV3", "format": "rca-1"}, f)
        return checkpoint_dir

    def load_checkpoint(self, checkpoint):
        path = checkpoint if isinstance(checkpoint, str) else getattr(checkpoint, "path", checkpoint)
        with open(os.path.join(path, "algorithm_state.pkl"), "rb") as f:
            st = pickle.load(f)
        self.set_weights(st["weights"])
        self.critic_ema.load_state_dict(st["critic_ema"])
        for o, s in zip((self.opt_wm, self.opt_actor, self.opt_critic), st["opt"]):
            o.load_state_dict(s)
        self._iteration, self._timesteps_total = st["iteration"], st["timesteps_total"]
        self.ret_scale, self._updates = st["ret_scale"], st["updates"]
        if self.callbacks is not None:
            self.callbacks.on_checkpoint_loaded(algorithm=self)

    def stop(self):
        pass

    cleanup = stop
