"""Algorithm base (reference: ``rllib/algorithms/algorithm.py``). An Algorithm is also a Tune
class trainable (``step() -> train()``)."""
from __future__ import annotations

import json
import os
import pickle
import time
from collections import deque
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ...tune.tuner import Trainable
from ..env.env_runner import EnvRunner
from ..policy.sample_batch import SampleBatch, concat_samples
from .algorithm_config import AlgorithmConfig


class Algorithm(Trainable):
    _default_config_cls = AlgorithmConfig
    multi_agent = False      # set in setup() from the config
    learner_groups = None
    _supports_lstm = False   # recurrent RLModules (model.use_lstm): PPO

    def __init__(self, config: Optional[AlgorithmConfig] = None, env=None, **kw):
        if isinstance(config, dict):
            config = self._default_config_cls().update_from_dict(config)
        self.config = config or self._default_config_cls()
        if env is not None:
            self.config.env = env
        self._iteration = 0
        self._timesteps_total = 0
        self._episodes_total = 0
        self._weights_version = 0
        self._recent = deque(maxlen=self.config.metrics_num_episodes_for_smoothing)
        self.setup(self.config)

    # Tune class-trainable path: Trainable.__init__ is bypassed (config already built)
    def setup(self, config):
        from ..._private import worker as w

        if not w.is_initialized():
            w.init()
        if isinstance(config, dict):
            self.config = self._default_config_cls().update_from_dict(config)
        cfg = self.config
        rd = cfg.runner_dict()
        rd.update(self._runner_extra())
        rd["_algo"] = "PPO" if self._supports_lstm else type(self).__name__
        self.multi_agent = cfg.is_multi_agent
        if self.multi_agent and (cfg.model or {}).get("use_lstm"):
            raise ValueError("use_lstm is supported for single-agent PPO only")
        runner_cls = EnvRunner
        if self.multi_agent:
            from ..env.multi_agent_env_runner import MultiAgentEnvRunner

            runner_cls = MultiAgentEnvRunner
        # the local runner (index 0) never takes the runners' GPU share
        self.local_runner = runner_cls(dict(rd, num_gpus_per_env_runner=0), 0)
        self.remote_runners = []
        if cfg.num_env_runners > 0:
            from ...actor import ActorClass

            opts = {"num_cpus": cfg.num_cpus_per_env_runner}
            if getattr(cfg, "num_gpus_per_env_runner", 0):
                opts["num_gpus"] = cfg.num_gpus_per_env_runner
            cls = ActorClass(runner_cls, opts)
            self.remote_runners = [cls.remote(rd, i + 1) for i in range(cfg.num_env_runners)]
        from ..core.learner import LearnerGroup

        ld = cfg.to_dict()
        ld.update(cfg._connector_dict())
        ld.update(self._runner_extra())
        ld["_algo"] = rd["_algo"]
        if self.multi_agent:
            # one learner group (RLModule + optimizer, possibly several GPU learners) per policy
            sp = self.local_runner.spaces()
            self.learner_groups = {p: LearnerGroup(ld, *sp[p]) for p in self.local_runner.modules}
            self.policies_to_train = list(cfg.policies_to_train or self.learner_groups)
            first = next(iter(self.learner_groups))
            self.obs_space, self.act_space = sp[first]
            self.learner_group = self.learner_groups[first]
        else:
            self.obs_space, self.act_space = self.local_runner.spaces()
            self.learner_group = LearnerGroup(ld, self.obs_space, self.act_space)
            self.learner_groups = None
        self._sync_weights()
        from .callbacks import build as _build_callbacks

        self.callbacks = _build_callbacks(getattr(cfg, "_callbacks", None))
        self._custom_metrics = []
        if self.callbacks is not None:
            self.callbacks.on_algorithm_init(algorithm=self)

    def _runner_extra(self):
        return {}

    # ------------------------------------------------------------------ rollouts
    def _sync_weights(self):
        from ..._private.worker import get, put

        st = ({p: g.get_weights() for p, g in self.learner_groups.items()} if self.multi_agent
              else self.learner_group.get_weights())
        self._weights_version += 1
        self.local_runner.set_weights(st, self._weights_version)
        if self.remote_runners:
            ref = put(st)
            get([r.set_weights.remote(ref, self._weights_version) for r in self.remote_runners])
        self._sync_connector_states()

    def _sync_connector_states(self):
        """Merge every env runner's env-to-module connector state (e.g. MeanStdFilter statistics)
        and broadcast the merged state back (reference: ``EnvRunnerGroup.sync_env_runner_states``)."""
        from ..._private.worker import get

        if self.multi_agent or not getattr(self.local_runner, "has_stateful_connectors", False):
            return
        states = [self.local_runner.get_connector_state()]
        if self.remote_runners:
            states += get([r.get_connector_state.remote() for r in self.remote_runners])
        merged = self.local_runner.env_to_module.merge_states(states)
        self.local_runner.set_connector_state(merged)
        if self.remote_runners:
            get([r.set_connector_state.remote(merged) for r in self.remote_runners])

    def _sample_fragments(self, steps_total: int) -> List[SampleBatch]:
        from ..._private.worker import get

        if self.remote_runners:
            per = max(1, steps_total // len(self.remote_runners))
            return get([r.sample.remote(per) for r in self.remote_runners])
        return [self.local_runner.sample(steps_total)]

    def _sample(self, steps_total: int) -> SampleBatch:
        return concat_samples(self._sample_fragments(steps_total))

    def _collect_metrics(self):
        from ..._private.worker import get

        ms = [self.local_runner.get_metrics()]
        if self.remote_runners:
            ms += get([r.get_metrics.remote() for r in self.remote_runners])
        eps = [e for m in ms for e in m["episodes"]]
        self._custom_metrics = [c for m in ms for c in m.get("custom_metrics", ())]
        if self.multi_agent:
            if not hasattr(self, "_policy_recent"):
                self._policy_recent = {}
            for m in ms:
                for p, rets in m.get("policy_returns", {}).items():
                    dq = self._policy_recent.setdefault(p, deque(maxlen=self.config.metrics_num_episodes_for_smoothing))
                    dq.extend(rets)
        for e in eps:
            self._recent.append(e)
        self._episodes_total += len(eps)
        return eps

    # ------------------------------------------------------------------ API
    def training_step(self) -> Dict:
        raise NotImplementedError

    def step(self):
        return self.train()

    def train(self) -> Dict:
        t0 = time.perf_counter()
        info = self.training_step()
        eps = self._collect_metrics()
        self._iteration += 1
        rets = [e[0] for e in self._recent]
        lens = [e[1] for e in self._recent]
        dt = time.perf_counter() - t0
        res = {
            "training_iteration": self._iteration,
            "episode_reward_mean": float(np.mean(rets)) if rets else float("nan"),
            "episode_reward_max": float(np.max(rets)) if rets else float("nan"),
            "episode_reward_min": float(np.min(rets)) if rets else float("nan"),
            "episode_len_mean": float(np.mean(lens)) if lens else float("nan"),
            "episodes_this_iter": len(eps),
            "episodes_total": self._episodes_total,
            "timesteps_total": self._timesteps_total,
            "num_env_steps_sampled": self._timesteps_total,
            "num_env_steps_sampled_this_iter": info.pop("_steps_this_iter", 0),
            "time_this_iter_s": dt,
            "info": {"learner": info if self.multi_agent else {"default_policy": info}},
        }
        if self.multi_agent:
            res["policy_reward_mean"] = {p: float(np.mean(d)) for p, d in getattr(self, "_policy_recent", {}).items()
                                         if d}
        res["env_steps_per_sec"] = res["num_env_steps_sampled_this_iter"] / dt if dt > 0 else 0.0
        res["env_runners"] = {"episode_return_mean": res["episode_reward_mean"],
                              "episode_return_max": res["episode_reward_max"],
                              "episode_return_min": res["episode_reward_min"],
                              "episode_len_mean": res["episode_len_mean"],
                              "num_episodes": len(eps)}
        if self._custom_metrics:
            from .callbacks import aggregate_custom_metrics

            res["custom_metrics"] = aggregate_custom_metrics(self._custom_metrics)
            res["env_runners"]["custom_metrics"] = res["custom_metrics"]
        iv = self.config.evaluation_interval
        if iv and self._iteration % iv == 0:
            res["evaluation"] = self.evaluate()
        if getattr(self, "callbacks", None) is not None:
            self.callbacks.on_train_result(algorithm=self, result=res)
        return res

    def evaluate(self) -> Dict:
        cb = getattr(self, "callbacks", None)
        if cb is not None:
            cb.on_evaluate_start(algorithm=self)
        out = self._evaluate()
        if cb is not None:
            cb.on_evaluate_end(algorithm=self, evaluation_metrics=out)
        return out

    def _evaluate(self) -> Dict:
        cfg = self.config
        rd = cfg.runner_dict()
        rd.update(self._runner_extra())
        rd.update(cfg.evaluation_config or {})
        rd["seed"] = (cfg.seed or 0) + 99991
        if not hasattr(self, "_eval_runner"):
            self._eval_runner = EnvRunner(rd, 10_000)
        self._eval_runner.set_weights(self.learner_group.get_weights(), self._weights_version)
        self._eval_runner.get_metrics()
        eps = []
        guard = 0
        while len(eps) < cfg.evaluation_duration and guard < 10000:
            self._eval_runner.sample(self._eval_runner.N * 64, explore=False)
            eps += self._eval_runner.get_metrics()["episodes"]
            guard += 1
        rets = [e[0] for e in eps]
        return {"episode_reward_mean": float(np.mean(rets)) if rets else float("nan"),
                "env_runners": {"episode_return_mean": float(np.mean(rets)) if rets else float("nan")},
                "num_episodes": len(eps)}

    def compute_single_action(self, observation, state=None, explore: bool = False, policy_id=None, **kw):
        """One action for one observation. Recurrent modules: pass ``state`` (None = initial) and
        get ``(action, state_out, {})`` back, as in the reference API."""
        obs = torch.as_tensor(np.asarray(observation)[None])
        m0 = self.local_runner.module if not self.multi_agent else None
        if m0 is not None and getattr(m0, "is_stateful", False):
            m0.set_state(self.learner_group.get_weights())
            st = m0.get_initial_state(1) if state is None else torch.as_tensor(np.asarray(state))[None].float()
            if explore:
                a, _, _, _, st2 = m0.forward_exploration_step(obs, st)
            else:
                a, _, st2 = m0.forward_inference_step(obs, st)
            a = a[0].numpy()
            return (int(a) if a.ndim == 0 else a), st2[0].numpy(), {}
        if self.multi_agent:
            pid = policy_id or next(iter(self.learner_groups))
            m = self.local_runner.modules[pid]
            m.set_state(self.learner_groups[pid].get_weights())
        else:
            m = self.local_runner.module
            m.set_state(self.learner_group.get_weights())
        if explore:
            a, _, _, _ = m.forward_exploration(obs)
        else:
            a, _ = m.forward_inference(obs)
        a = a[0].numpy()
        return int(a) if a.ndim == 0 else a

    def get_module(self, module_id=None):
        """The (weight-synced) RLModule; multi-agent: the one of ``module_id`` (default: first)."""
        if self.multi_agent:
            pid = module_id or next(iter(self.learner_groups))
            m = self.local_runner.modules[pid]
            m.set_state(self.learner_groups[pid].get_weights())
            return m
        m = self.local_runner.module
        m.set_state(self.learner_group.get_weights())
        return m

    def get_policy(self, policy_id=None):
        """Old-API-stack view (reference ``Algorithm.get_policy``): a ``TorchPolicy`` over the
        current module (``compute_actions`` / ``get_weights`` / ``set_weights``)."""
        from ..policy.policy import TorchPolicy

        m = self.get_module(policy_id)
        if self.multi_agent:
            pid = policy_id or next(iter(self.learner_groups))
            obs_sp, act_sp = self.local_runner.spaces_[pid]
        else:
            obs_sp = self.local_runner.env_to_module.observation_space
            act_sp = self.local_runner.env.action_space
        return TorchPolicy(obs_sp, act_sp, self.config.to_dict(), model=m)

    def compute_actions(self, observations, state=None, explore: bool = False, policy_id=None, **kw):
        """Batched ``compute_single_action``: a dict {agent/env key: obs} gives a dict of actions,
        an array batch gives an array (reference ``Algorithm.compute_actions``)."""
        if isinstance(observations, dict):
            return {k: self.compute_single_action(o, explore=explore, policy_id=policy_id)
                    for k, o in observations.items()}
        acts, _, _ = self.get_policy(policy_id).compute_actions(np.asarray(observations), explore=explore)
        return acts

    def export_policy_model(self, export_dir: str, policy_id=None):
        """Save the policy network's ``state_dict`` (``model.pt``, loadable with
        ``torch.load(..., weights_only=True)``) plus its class name."""
        os.makedirs(export_dir, exist_ok=True)
        m = self.get_module(policy_id)
        torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, os.path.join(export_dir, "model.pt"))
        with open(os.path.join(export_dir, "model_info.json"), "w") as f:
            json.dump({"module_class": type(m).__name__, "policy_id": policy_id}, f)
        return export_dir

    def get_weights(self, policies=None):
        if self.multi_agent:
            return {p: g.get_weights() for p, g in self.learner_groups.items() if policies is None or p in policies}
        return self.learner_group.get_weights()

    def set_weights(self, w):
        if self.multi_agent:
            for p, st in w.items():
                self.learner_groups[p].call("set_weights", st)
        else:
            self.learner_group.call("set_weights", w)
        self._sync_weights()

    def save_checkpoint(self, checkpoint_dir: str):
        os.makedirs(checkpoint_dir, exist_ok=True)
        learner = ({p: g.call("get_state") for p, g in self.learner_groups.items()} if self.multi_agent
                   else self.learner_group.call("get_state"))
        st = {"learner": learner, "iteration": self._iteration, "multi_agent": self.multi_agent,
              "timesteps_total": self._timesteps_total, "config": self.config.to_dict(),
              "extra": self._extra_state()}
        with open(os.path.join(checkpoint_dir, "algorithm_state.pkl"), "wb") as f:
            pickle.dump(st, f)
        with open(os.path.join(checkpoint_dir, "rllib_checkpoint.json"), "w") as f:
            json.dump({"type": "Algorithm", "algo": type(self).__name__, "format": "rca-1"}, f)
        return checkpoint_dir

    def load_checkpoint(self, checkpoint):
        path = checkpoint if isinstance(checkpoint, str) else getattr(checkpoint, "path", checkpoint)
        with open(os.path.join(path, "algorithm_state.pkl"), "rb") as f:
            st = pickle.load(f)
        if st.get("multi_agent"):
            for p, ls in st["learner"].items():
                self.learner_groups[p].call("set_state", ls)
        else:
            self.learner_group.call("set_state", st["learner"])
        self._iteration = st["iteration"]
        self._timesteps_total = st["timesteps_total"]
        self._load_extra_state(st.get("extra") or {})
        self._sync_weights()
        if getattr(self, "callbacks", None) is not None:
            self.callbacks.on_checkpoint_loaded(algorithm=self)

    def _extra_state(self):
        return {}

    def _load_extra_state(self, st):
        pass

    def save(self, checkpoint_dir: Optional[str] = None):
        from ...train._checkpoint import Checkpoint

        d = checkpoint_dir or os.path.join(os.path.expanduser("~/rca_results"), "rllib", f"{type(self).__name__}_"
                                           f"{int(time.time())}", f"checkpoint_{self._iteration:06d}")
        self.save_checkpoint(d)
        return _SaveResult(Checkpoint.from_directory(d))

    def restore(self, checkpoint):
        self.load_checkpoint(checkpoint)

    @classmethod
    def from_checkpoint(cls, checkpoint):
        path = checkpoint if isinstance(checkpoint, str) else checkpoint.path
        with open(os.path.join(path, "algorithm_state.pkl"), "rb") as f:
            st = pickle.load(f)
        algo = cls(config=cls._default_config_cls().update_from_dict(st["config"]))
        algo.load_checkpoint(path)
        return algo

    def stop(self):
        from ..._private.worker import kill

        for r in self.remote_runners:
            try:
                kill(r)
            except Exception:
                pass
        self.remote_runners = []
        for g in (self.learner_groups.values() if self.multi_agent else [self.learner_group]):
            g.shutdown()

    cleanup = stop

    @property
    def iteration(self):
        return self._iteration


class _SaveResult:
    def __init__(self, checkpoint):
        self.checkpoint = checkpoint

    def __fspath__(self):
        return self.checkpoint.path

    def __str__(self):
        return self.checkpoint.path
