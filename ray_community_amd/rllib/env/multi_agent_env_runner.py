"""Multi-agent env runner (reference: ``rllib/env/multi_agent_env_runner.py:24``).

Steps ``num_envs_per_env_runner`` copies of a ``MultiAgentEnv``. Every agent id is bound to a
policy by ``policy_mapping_fn(agent_id, episode, worker)`` (evaluated once per agent: the mapping
is static for the runner's lifetime); each policy has its own RLModule and all of a policy's
acting agents are batched into one forward pass per step.

Output per policy is the same env-major ``[R, T]`` fragment the single-agent PPO learner consumes
(R = sub-envs x agents mapped to that policy), with ``loss_mask`` = 0 on the steps where an agent
was not acting (it finished before the rest of its episode); those padded steps are terminal with
zero reward and value, so the batched GAE kernel never leaks returns across them. Truncated
agents bootstrap from their final observation exactly as in the single-agent runner.
"""
from __future__ import annotations

import collections
from typing import Dict, Optional

import numpy as np
import torch

from ..core.rl_module import MultiRLModule, make_module
from ..policy.sample_batch import DEFAULT_POLICY_ID, MultiAgentBatch, SampleBatch
from .multi_agent_env import make_multi_agent_env


def default_policy_mapping_fn(agent_id, episode=None, worker=None, **kw):
    return DEFAULT_POLICY_ID


class MultiAgentEnvRunner:
    def __init__(self, config: Dict, worker_index: int = 0):
        torch.set_num_threads(int(config.get("num_cpus_per_env_runner_threads", 1)))
        self.cfg = config
        self.worker_index = worker_index
        seed = config.get("seed")
        self.seed = None if seed is None else int(seed) + 1000 * worker_index
        if self.seed is not None:
            torch.manual_seed(self.seed)
        self.N = int(config.get("num_envs_per_env_runner", 1))
        self.envs = [make_multi_agent_env(config["env"], config.get("env_config")) for _ in range(self.N)]
        env0 = self.envs[0]
        self.agent_ids = list(env0.possible_agents)
        fn = config.get("policy_mapping_fn") or default_policy_mapping_fn
        self.agent_policy = {a: fn(a, None, worker=self) for a in self.agent_ids}
        declared = config.get("policies") or {DEFAULT_POLICY_ID: None}
        self.policy_ids = [p for p in (declared if isinstance(declared, (dict, list, tuple, set)) else [declared])]
        for a, p in self.agent_policy.items():
            if p not in self.policy_ids:
                raise ValueError(f"policy_mapping_fn maps agent {a!r} to unknown policy {p!r}")
        self.spaces_ = {}
        for p in self.policy_ids:
            spec = declared.get(p) if isinstance(declared, dict) else None
            agents = [a for a in self.agent_ids if self.agent_policy[a] == p]
            obs_sp = getattr(spec, "observation_space", None) or (spec[1] if isinstance(spec, tuple) and len(spec) > 2
                                                                   else None)
            act_sp = getattr(spec, "action_space", None) or (spec[2] if isinstance(spec, tuple) and len(spec) > 2
                                                              else None)
            if agents:
                obs_sp = obs_sp or env0.get_observation_space(agents[0])
                act_sp = act_sp or env0.get_action_space(agents[0])
            self.spaces_[p] = (obs_sp, act_sp)
        # one MultiRLModule holding every policy's RLModule (reference MultiAgentRLModule)
        self.modules = MultiRLModule({p: make_module(config, *self.spaces_[p], module_id=p) for p in self.policy_ids
                                      if self.spaces_[p][0]})
        for m in self.modules.values():
            m.eval()
        # fixed row layout per policy: (sub-env, agent)
        self.rows = {p: [(i, a) for i in range(self.N) for a in self.agent_ids if self.agent_policy[a] == p]
                     for p in self.modules}
        self.obs = []
        for i, e in enumerate(self.envs):
            o, _ = e.reset(seed=None if self.seed is None else self.seed + i)
            self.obs.append(dict(o))
        self.ep_ret = [collections.defaultdict(float) for _ in range(self.N)]
        self.ep_len = [0] * self.N
        self.completed = collections.deque(maxlen=int(config.get("metrics_num_episodes_for_smoothing", 100)))
        self.new_episodes = []
        self.new_agent_returns = collections.defaultdict(list)
        self.steps_sampled = 0
        self.weights_version = -1

    def spaces(self):
        return {p: sp for p, sp in self.spaces_.items()}

    def _remap(self, fn):
        """Re-bind agents to policies (runtime policy mutation); takes effect for the next
        ``sample`` call, whose per-policy row layout is rebuilt here."""
        mapping = {a: fn(a, None, worker=self) for a in self.agent_ids}
        for a, p in mapping.items():
            if p not in self.modules:
                raise ValueError(f"policy_mapping_fn maps agent {a!r} to unknown policy {p!r}")
        self.agent_policy = mapping
        self.cfg["policy_mapping_fn"] = fn
        self.rows = {p: [(i, a) for i in range(self.N) for a in self.agent_ids if self.agent_policy[a] == p]
                     for p in self.modules}

    def add_policy(self, policy_id, observation_space, action_space, weights=None, policy_mapping_fn=None):
        """Add a policy's RLModule (reference ``Algorithm.add_policy`` on every env runner)."""
        if policy_id in self.modules:
            raise KeyError(f"policy {policy_id!r} already exists")
        self.spaces_[policy_id] = (observation_space, action_space)
        self.policy_ids.append(policy_id)
        m = make_module(self.cfg, observation_space, action_space, module_id=policy_id)
        m.eval()
        if weights is not None:
            m.set_state(weights)
        self.modules[policy_id] = m
        self._remap(policy_mapping_fn or self.cfg.get("policy_mapping_fn") or default_policy_mapping_fn)
        return True

    def remove_policy(self, policy_id, policy_mapping_fn=None):
        if policy_id not in self.modules:
            raise KeyError(f"unknown policy {policy_id!r}")
        fn = policy_mapping_fn or self.cfg.get("policy_mapping_fn") or default_policy_mapping_fn
        keep = MultiRLModule(dict(self.modules.items()))
        keep.pop(policy_id)
        for a in self.agent_ids:
            if fn(a, None, worker=self) not in keep:
                raise ValueError(f"after removing {policy_id!r}, agent {a!r} would map to no policy: "
                                 f"pass a new policy_mapping_fn")
        self.modules = keep
        self.spaces_.pop(policy_id, None)
        self.policy_ids = [p for p in self.policy_ids if p != policy_id]
        self._remap(fn)
        return True

    def set_weights(self, states: Dict, version: int = 0):
        if version != self.weights_version:
            for p, st in states.items():
                if p in self.modules:
                    self.modules[p].set_state(st)
            self.weights_version = version
        return True

    def get_weights(self):
        return {p: m.get_state() for p, m in self.modules.items()}

    @torch.no_grad()
    def sample(self, num_steps: Optional[int] = None, explore: bool = True) -> MultiAgentBatch:
        T = max(1, int(num_steps or self.cfg.get("rollout_fragment_length", 64) * self.N) // self.N)
        bufs = {}
        for p, rows in self.rows.items():
            R = len(rows)
            obs_shape = self.spaces_[p][0].shape
            act_shape = tuple(self.spaces_[p][1].shape or ())
            disc = getattr(self.modules[p], "dist_cls", None) is not None and \
                self.modules[p].dist_cls.__name__ == "Categorical"
            bufs[p] = {
                "obs": np.zeros((R, T) + tuple(obs_shape), dtype=np.float32),
                "actions": np.zeros((R, T) + (() if disc else act_shape), dtype=np.int64 if disc else np.float32),
                "action_logp": np.zeros((R, T), np.float32), "vf_preds": np.zeros((R, T), np.float32),
                "rewards": np.zeros((R, T), np.float32), "terminateds": np.ones((R, T), bool),
                "truncateds": np.zeros((R, T), bool), "next_vf_preds": np.zeros((R, T), np.float32),
                "loss_mask": np.zeros((R, T), np.float32), "logits": None,
            }
        for t in range(T):
            actions = [dict() for _ in range(self.N)]
            acted = {}
            for p, rows in self.rows.items():
                live = [(r, i, a) for r, (i, a) in enumerate(rows) if a in self.obs[i]]
                if not live:
                    continue
                o = torch.as_tensor(np.stack([self.obs[i][a] for _, i, a in live]).astype(np.float32))
                m = self.modules[p]
                if explore:
                    act, lp, v, logits = m.forward_exploration(o)
                else:
                    act, v = m.forward_inference(o)
                    lp, logits = torch.zeros(len(live)), None
                B = bufs[p]
                idx = np.array([r for r, _, _ in live])
                B["obs"][idx, t] = o.numpy()
                an = act.numpy()
                B["actions"][idx, t] = an
                B["action_logp"][idx, t] = lp.numpy()
                B["vf_preds"][idx, t] = v.numpy()
                B["loss_mask"][idx, t] = 1.0
                B["terminateds"][idx, t] = False
                if logits is not None:
                    if B["logits"] is None:
                        B["logits"] = np.zeros((len(rows), T, logits.shape[-1]), np.float32)
                    B["logits"][idx, t] = logits.numpy()
                for k, (_, i, a) in enumerate(live):
                    actions[i][a] = an[k].item() if an[k].ndim == 0 else an[k]
                acted[p] = live
            # step every sub-env
            results = []
            for i, e in enumerate(self.envs):
                results.append(e.step(actions[i]) if actions[i] else ({}, {}, {"__all__": False},
                                                                       {"__all__": False}, {}))
            trunc_boot = collections.defaultdict(list)  # p -> [(row, final obs)]
            for p, live in acted.items():
                B = bufs[p]
                for r, i, a in live:
                    nobs, rew, term, trunc, _ = results[i]
                    B["rewards"][r, t] = rew.get(a, 0.0)
                    te, tr = bool(term.get(a, False)), bool(trunc.get(a, False))
                    B["terminateds"][r, t] = te
                    B["truncateds"][r, t] = tr and not te
                    if tr and not te and a in nobs:
                        trunc_boot[p].append((r, nobs[a]))
            for p, items in trunc_boot.items():
                fo = torch.as_tensor(np.stack([x[1] for x in items]).astype(np.float32))
                fv = self.modules[p].forward(fo)[1].numpy()
                for (r, _), v in zip(items, fv):
                    bufs[p]["next_vf_preds"][r, t] = v
            for i, (nobs, rew, term, trunc, _) in enumerate(results):
                for a, r_ in rew.items():
                    self.ep_ret[i][a] += r_
                self.ep_len[i] += 1 if rew else 0
                ended = {a for a in self.obs[i] if term.get(a) or trunc.get(a)}
                cur = {a: o for a, o in nobs.items() if a not in ended}
                if term.get("__all__") or trunc.get("__all__"):
                    total = float(sum(self.ep_ret[i].values()))
                    ep = (total, int(self.ep_len[i]))
                    self.completed.append(ep)
                    self.new_episodes.append(ep)
                    for a, v in self.ep_ret[i].items():
                        self.new_agent_returns[self.agent_policy.get(a, DEFAULT_POLICY_ID)].append(float(v))
                    self.ep_ret[i] = collections.defaultdict(float)
                    self.ep_len[i] = 0
                    cur, _ = self.envs[i].reset()
                    cur = dict(cur)
                self.obs[i] = cur
        # value bootstraps: next step's value of the same row where it keeps acting; the last
        # step bootstraps from the current observation
        for p, rows in self.rows.items():
            B = bufs[p]
            same_episode = (B["loss_mask"][:, 1:] > 0) & ~B["terminateds"][:, :-1] & ~B["truncateds"][:, :-1]
            B["next_vf_preds"][:, :-1] = np.where(same_episode, B["vf_preds"][:, 1:], B["next_vf_preds"][:, :-1])
            live = [(r, i, a) for r, (i, a) in enumerate(rows) if a in self.obs[i]]
            if live:
                o = torch.as_tensor(np.stack([self.obs[i][a] for _, i, a in live]).astype(np.float32))
                lv = self.modules[p].forward(o)[1].numpy()
                for (r, _, _), v in zip(live, lv):
                    if not B["terminateds"][r, -1] and not B["truncateds"][r, -1]:
                        B["next_vf_preds"][r, -1] = v
        self.steps_sampled += self.N * T
        out = {}
        for p, B in bufs.items():
            logits = B.pop("logits")
            sb = SampleBatch(B)
            if logits is not None:
                sb[SampleBatch.ACTION_DIST_INPUTS] = logits
            sb.fragment_shape = (len(self.rows[p]), T)
            out[p] = sb
        return MultiAgentBatch(out, self.N * T)

    def get_metrics(self) -> Dict:
        eps, ag = self.new_episodes, self.new_agent_returns
        self.new_episodes, self.new_agent_returns = [], collections.defaultdict(list)
        return {"episodes": eps, "num_env_steps_sampled": self.steps_sampled, "custom_metrics": [],
                "policy_returns": dict(ag)}

    def ping(self):
        return "ok"

    def apply(self, func, *args, **kwargs):
        """``func(self, *args)`` (``EnvRunnerGroup.foreach_env_runner`` with a callable)."""
        return func(self, *args, **kwargs)
