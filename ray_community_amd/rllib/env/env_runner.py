"""Env runners (reference: ``rllib/env/single_agent_env_runner.py``, ``evaluation/rollout_worker.py``).

Each runner owns a natively vectorised env (N sub-envs stepped as one numpy batch) and a CPU
copy of the RLModule; it returns rollout fragments as env-major ``[N, T]`` column blocks with
the value bootstraps needed for exact GAE under auto-reset and truncation (``next_vf_preds``).
"""
from __future__ import annotations

import collections
import time
from typing import Dict, Optional

import numpy as np
import torch

from ..core.rl_module import make_module
from ..policy.sample_batch import SampleBatch
from .envs import make_vector_env


class EnvRunner:
    def __init__(self, config: Dict, worker_index: int = 0):
        torch.set_num_threads(int(config.get("num_cpus_per_env_runner_threads", 1)))
        self.cfg = config
        self.worker_index = worker_index
        seed = config.get("seed")
        self.seed = None if seed is None else int(seed) + 1000 * worker_index
        if self.seed is not None:
            torch.manual_seed(self.seed)
        self.env = make_vector_env(config["env"], config.get("num_envs_per_env_runner", 1), config.get("env_config"),
                                   seed=self.seed)
        self.N = self.env.num_envs
        self.module = make_module(config, self.env.observation_space, self.env.action_space)
        self.module.eval()
        # GPU inference (num_gpus_per_env_runner > 0): the module lives on the runner's GPU share,
        # observations go up once per step and ONE packed [N, 3 + A] tensor comes back
        self.device = torch.device("cpu")
        if float(config.get("num_gpus_per_env_runner", 0) or 0) > 0 and torch.cuda.is_available():
            self.device = torch.device("cuda", torch.cuda.current_device())
            self.module.to(self.device)
        self.obs, _ = self.env.reset(seed=self.seed)
        self.ep_ret = np.zeros(self.N)
        self.ep_len = np.zeros(self.N, dtype=np.int64)
        self.completed = collections.deque(maxlen=int(config.get("metrics_num_episodes_for_smoothing", 100)))
        self.new_episodes = []
        self.steps_sampled = 0
        self.weights_version = -1
        self._rng = np.random.default_rng(self.seed)
        from ..algorithms.callbacks import Episode, build, overrides

        self._Episode = Episode
        self.callbacks = build(config.get("callbacks_class"))
        self._cb_step = overrides(self.callbacks, "on_episode_step")
        self.new_custom_metrics = []
        if self.callbacks is not None:
            self.callbacks.on_environment_created(env_runner=self, env=self.env, env_context=config.get("env_config"))
            self._eps = [Episode(i) for i in range(self.N)]
            for i, ep in enumerate(self._eps):
                self.callbacks.on_episode_start(episode=ep, env_runner=self, env_index=i)

    def spaces(self):
        return self.env.observation_space, self.env.action_space

    def set_weights(self, state, version: int = 0):
        if version != self.weights_version:
            self.module.set_state(state)
            self.weights_version = version
        return True

    def get_weights(self):
        return self.module.get_state()

    def _track(self, rew, term, trunc, info=None):
        self.ep_ret += rew
        self.ep_len += 1
        done = term | trunc
        cb = self.callbacks
        if cb is not None and self._cb_step:
            for i, ep in enumerate(self._eps):
                ep.total_reward, ep.length, ep.last_info = float(self.ep_ret[i]), int(self.ep_len[i]), info
                cb.on_episode_step(episode=ep, env_runner=self, env_index=i)
        if done.any():
            for i in np.nonzero(done)[0]:
                ep = (float(self.ep_ret[i]), int(self.ep_len[i]))
                self.completed.append(ep)
                self.new_episodes.append(ep)
                if cb is not None:
                    e = self._eps[i]
                    e.total_reward, e.length = ep
                    cb.on_episode_end(episode=e, env_runner=self, env_index=int(i))
                    if e.custom_metrics:
                        self.new_custom_metrics.append(dict(e.custom_metrics))
                    self._eps[i] = self._Episode(int(i))
                    cb.on_episode_start(episode=self._eps[i], env_runner=self, env_index=int(i))
            self.ep_ret[done] = 0
            self.ep_len[done] = 0

    def _to_host(self, a, lp, v, logits):
        """One device->host copy per step for the policy outputs (discrete actions travel as f32)."""
        if a.dim() != 1 or a.dtype not in (torch.int64, torch.int32):
            return a.cpu(), lp.cpu(), v.cpu(), None if logits is None else logits.cpu()
        cols = [a.float().unsqueeze(1), lp.float().unsqueeze(1), v.float().unsqueeze(1)]
        if logits is not None:
            cols.append(logits.float())
        h = torch.cat(cols, 1).cpu()
        return h[:, 0].long(), h[:, 1], h[:, 2], (h[:, 3:] if logits is not None else None)

    def _value(self, obs):
        o = torch.from_numpy(obs)
        if self.device.type == "cuda":
            o = o.to(self.device, non_blocking=True)
        return self.module.forward(o)[1].float().cpu().numpy()

    @torch.no_grad()
    def sample(self, num_steps: Optional[int] = None, explore: bool = True) -> SampleBatch:
        """On-policy fragment of T = num_steps // N steps per sub-env (PPO / IMPALA)."""
        T = max(1, int(num_steps or self.cfg.get("rollout_fragment_length", 64) * self.N) // self.N)
        N = self.N
        obs_buf = np.empty((N, T) + self.obs.shape[1:], dtype=self.obs.dtype)
        dist = getattr(self.module, "dist_cls", None)  # None: SAC-style module with its own squashed policy
        act_shape = () if dist is not None and dist.__name__ == "Categorical" else self.env.action_space.shape
        acts = np.empty((N, T) + tuple(act_shape), dtype=np.int64 if act_shape == () else np.float32)
        logp = np.empty((N, T), dtype=np.float32)
        vf = np.empty((N, T), dtype=np.float32)
        rew = np.empty((N, T), dtype=np.float32)
        term = np.empty((N, T), dtype=bool)
        trunc = np.empty((N, T), dtype=bool)
        logits_buf = None
        trunc_fix = []  # (t, env indices, final obs)
        gpu = self.device.type == "cuda"
        for t in range(T):
            o = torch.from_numpy(self.obs)
            if gpu:
                o = o.to(self.device, non_blocking=True)
            if explore:
                a, lp, v, logits = self.module.forward_exploration(o)
            else:
                a, v = self.module.forward_inference(o)
                lp = torch.zeros(N, device=o.device)
                logits = None
            if gpu:
                a, lp, v, logits = self._to_host(a, lp, v, logits)
            if logits is not None:
                if logits_buf is None:
                    logits_buf = np.empty((N, T, logits.shape[-1]), dtype=np.float32)
                logits_buf[:, t] = logits.numpy()
            obs_buf[:, t] = self.obs
            an = a.numpy()
            acts[:, t] = an
            logp[:, t] = lp.numpy()
            vf[:, t] = v.numpy()
            nobs, r, te, tr, info = self.env.step(an)
            rew[:, t] = r
            term[:, t] = te
            trunc[:, t] = tr
            if tr.any():
                idx = np.nonzero(tr)[0]
                trunc_fix.append((t, idx, info["final_obs"][idx]))
            self._track(r, te, tr, info)
            self.obs = nobs
        last_v = self._value(self.obs)
        next_vf = np.empty_like(vf)
        next_vf[:, :-1] = vf[:, 1:]
        next_vf[:, -1] = last_v
        if trunc_fix:
            fo = np.concatenate([x[2] for x in trunc_fix], axis=0)
            fv = self._value(fo)
            k = 0
            for t, idx, _ in trunc_fix:
                next_vf[idx, t] = fv[k: k + len(idx)]
                k += len(idx)
        self.steps_sampled += N * T
        b = SampleBatch({SampleBatch.OBS: obs_buf, SampleBatch.ACTIONS: acts, SampleBatch.ACTION_LOGP: logp,
                         SampleBatch.VF_PREDS: vf, SampleBatch.REWARDS: rew, SampleBatch.TERMINATEDS: term,
                         SampleBatch.TRUNCATEDS: trunc, SampleBatch.NEXT_VF_PREDS: next_vf})
        if logits_buf is not None:
            b[SampleBatch.ACTION_DIST_INPUTS] = logits_buf
        b.fragment_shape = (N, T)
        if self.cfg.get("output"):
            if getattr(self, "_writer", None) is None:
                from ..offline import JsonWriter

                self._writer = JsonWriter(self.cfg["output"])
            self._writer.write(b)
        if self.callbacks is not None:
            self.callbacks.on_sample_end(env_runner=self, samples=b)
        return b

    @torch.no_grad()
    def sample_transitions(self, num_steps: int, epsilon: float = 0.0) -> SampleBatch:
        """Off-policy transitions (DQN): epsilon-greedy on the Q head."""
        N = self.N
        T = max(1, int(num_steps) // N)
        out = {k: [] for k in ("obs", "actions", "rewards", "new_obs", "terminateds")}
        continuous = not hasattr(self.module, "q_values")
        space = self.env.action_space
        for _ in range(T):
            if continuous:  # SAC: stochastic policy; epsilon = probability of a uniform random action
                a = self.module.forward_exploration(torch.from_numpy(self.obs))[0].numpy().astype(np.float32)
                rnd = self._rng.random(N) < epsilon
                if rnd.any():
                    a[rnd] = self._rng.uniform(space.low, space.high, size=(int(rnd.sum()),) + space.shape)
            else:
                q = self.module.q_values(torch.from_numpy(self.obs))
                a = q.argmax(-1).numpy()
                rnd = self._rng.random(N) < epsilon
                if rnd.any():
                    a[rnd] = self._rng.integers(0, space.n, int(rnd.sum()))
            nobs, r, te, tr, info = self.env.step(a)
            done = te | tr
            nxt = np.where(done.reshape((-1,) + (1,) * (nobs.ndim - 1)), info["final_obs"], nobs)
            out["obs"].append(self.obs)
            out["actions"].append(a)
            out["rewards"].append(r)
            out["new_obs"].append(nxt)
            out["terminateds"].append(te)
            self._track(r, te, tr, info)
            self.obs = nobs
        self.steps_sampled += N * T
        b = SampleBatch({k: np.concatenate(v, axis=0) if k in ("obs", "new_obs") else np.concatenate(v) for k, v
                         in out.items()})
        if self.callbacks is not None:
            self.callbacks.on_sample_end(env_runner=self, samples=b)
        return b

    def get_metrics(self) -> Dict:
        eps, cms = self.new_episodes, self.new_custom_metrics
        self.new_episodes, self.new_custom_metrics = [], []
        return {"episodes": eps, "num_env_steps_sampled": self.steps_sampled, "custom_metrics": cms}

    def ping(self):
        return "ok"
