"""Algorithm base (reference: ``rllib/algorithms/algorithm.py``). An Algorithm is also a Tune
class trainable (``step() -> train()``)."""
from __future__ import annotations

import json
import os
import pickle
import time
from collections import deque
from typing import Any, Dict, List, Optional

import cloudpickle
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
        if callable(cfg.input_):  # a reader factory (PolicyServerInput): no env to step
            from ..env.env_runner import ExternalInputRunner

            runner_cls = ExternalInputRunner
            rd["input_"] = cfg.input_
        if self.multi_agent:
            from ..env.multi_agent_env_runner import MultiAgentEnvRunner

            runner_cls = MultiAgentEnvRunner
        # the local runner (index 0) never takes the runners' GPU share
        self.local_runner = runner_cls(dict(rd, num_gpus_per_env_runner=0), 0)
        from ..env.env_runner_group import EnvRunnerGroup

        opts = {"num_cpus": cfg.num_cpus_per_env_runner, "max_restarts": 0}
        if getattr(cfg, "num_gpus_per_env_runner", 0):
            opts["num_gpus"] = cfg.num_gpus_per_env_runner
        self._runner_cls = runner_cls
        self.env_runner_group = EnvRunnerGroup(runner_cls, rd, cfg, self.local_runner, int(cfg.num_env_runners), opts)
        self._counters = {"total_num_restored_workers": 0}
        from ..core.learner import LearnerGroup

        ld = cfg.to_dict()
        ld.update(cfg._connector_dict())
        ld.update(self._runner_extra())
        ld["_algo"] = rd["_algo"]
        from ..execution import _update_kind

        try:  # the fused Learner update this algorithm trains with (LearnerGroup.update_from_batch)
            ld["_update_kind"] = _update_kind(self)
        except ValueError:  # DreamerV3 trains its world model without a Learner update kind
            pass
        self._learner_dict = ld
        if self.multi_agent:
            # one learner group (RLModule + optimizer, possibly several GPU learners) per policy
            sp = self.local_runner.spaces()
            self.learner_groups = {p: LearnerGroup(dict(ld, _module_id=p), *sp[p]) for p in self.local_runner.modules}
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

    # ------------------------------------------------------------------ env runners
    @property
    def workers(self):
        """The env runner group (reference name ``Algorithm.workers`` / ``env_runner_group``)."""
        return getattr(self, "env_runner_group", None)

    @property
    def remote_runners(self) -> List:
        """The HEALTHY remote env runner actors."""
        g = getattr(self, "env_runner_group", None)
        if g is None:
            return list(self.__dict__.get("_remote_runners_override", []))
        return g.healthy_env_runners()

    @remote_runners.setter
    def remote_runners(self, value):
        if getattr(self, "env_runner_group", None) is not None and not value:
            self.env_runner_group.stop()
        else:
            self.__dict__["_remote_runners_override"] = list(value or [])

    def _foreach_runner(self, method: str, *args, local_fallback: bool = True) -> List:
        """``method(*args)`` on every healthy remote runner (failures handled by the group's
        fault-tolerance policy); with no remote runner left, on the local one."""
        g = getattr(self, "env_runner_group", None)
        out = g.foreach_env_runner(method, *args) if g is not None and g.num_remote_env_runners() else []
        if not out and local_fallback:
            out = [getattr(self.local_runner, method)(*args)]
        return out

    def restore_workers(self, workers=None) -> List[int]:
        """Bring recreated / recovered env runners up to date (reference ``algorithm.py:1429``):
        probe the unhealthy ones, push the current weights and connector state to those that
        answer, mark them healthy and fire ``on_workers_recreated``."""
        from ..._private.worker import get, put

        workers = workers or getattr(self, "env_runner_group", None)
        if workers is None:
            return []
        restored = workers.probe_unhealthy_env_runners()
        if not restored:
            return []
        st = ({p: g.get_weights() for p, g in self.learner_groups.items()} if self.multi_agent
              else self.learner_group.get_weights())
        ref = put(st)
        actors = workers.manager.actors()
        calls = [actors[i].set_weights.remote(ref, self._weights_version) for i in restored]
        if not self.multi_agent and getattr(self.local_runner, "has_stateful_connectors", False):
            cs = self.local_runner.get_connector_state()
            calls += [actors[i].set_connector_state.remote(cs) for i in restored]
        ok = []
        try:
            get(calls, timeout=workers.restore_timeout)
            ok = restored
        except Exception:  # noqa  (a runner that dies while being restored stays unhealthy)
            for i in restored:
                try:
                    get(actors[i].ping.remote(), timeout=workers.probe_timeout)
                    ok.append(i)
                except Exception:  # noqa
                    pass
        workers.mark_healthy(ok)
        self._counters["total_num_restored_workers"] += len(ok)
        if ok and getattr(self, "callbacks", None) is not None:
            self.callbacks.on_workers_recreated(algorithm=self, worker_set=workers, worker_ids=ok,
                                                is_evaluation=False)
        return ok

    # ------------------------------------------------------------------ rollouts
    def _sync_weights(self):
        from ..._private.worker import get, put

        st = ({p: g.get_weights() for p, g in self.learner_groups.items()} if self.multi_agent
              else self.learner_group.get_weights())
        self._weights_version += 1
        self.local_runner.set_weights(st, self._weights_version)
        if self.remote_runners:
            self._foreach_runner("set_weights", put(st), self._weights_version, local_fallback=False)
        self._sync_connector_states()

    def _sync_connector_states(self):
        """Merge every env runner's env-to-module connector state (e.g. MeanStdFilter statistics)
        and broadcast the merged state back (reference: ``EnvRunnerGroup.sync_env_runner_states``)."""
        from ..._private.worker import get

        if self.multi_agent or not getattr(self.local_runner, "has_stateful_connectors", False):
            return
        states = [self.local_runner.get_connector_state()]
        if self.remote_runners:
            states += self._foreach_runner("get_connector_state", local_fallback=False)
        merged = self.local_runner.env_to_module.merge_states(states)
        self.local_runner.set_connector_state(merged)
        if self.remote_runners:
            self._foreach_runner("set_connector_state", merged, local_fallback=False)

    def _sample_fragments(self, steps_total: int) -> List[SampleBatch]:
        n = len(self.remote_runners)
        if n:
            return self._foreach_runner("sample", max(1, steps_total // n))
        return [self.local_runner.sample(steps_total)]

    def _sample_fragment_refs(self, steps_total: int, wait_ready: bool = True):
        """``(fragment refs, env steps)`` when the fragments can go to remote learners by reference
        (remote runners, learner actors whose count divides the fragments, the default fail-fast
        runner policy), else None. With ``wait_ready`` the driver waits for the fragments to be
        ready (never fetching them); without, the refs go out at once and each learner copies the
        fragments to its device as they arrive, overlapping the host->device transfer with the
        runners still sampling."""
        g = getattr(self, "env_runner_group", None)
        lg = getattr(self, "learner_group", None)
        n = len(self.remote_runners)
        if (not n or g is None or lg is None or getattr(lg, "local", None) is not None or g.ignore
                or n % max(1, getattr(lg, "n", 1)) or os.environ.get("RCA_RLLIB_FRAGMENT_REFS", "1") == "0"):
            return None
        from ..._private.worker import wait

        per = max(1, steps_total // n)
        res = g.manager.foreach_actor("sample", per, return_obj_refs=True)
        refs = [r.get() for r in res.ignore_errors()]
        if len(refs) != n:
            return None
        if wait_ready:
            wait(refs, num_returns=len(refs))
        envs = int(self.config.num_envs_per_env_runner or 1)
        steps = n * envs * max(1, per // envs)
        return refs, steps

    def _sample(self, steps_total: int) -> SampleBatch:
        return concat_samples(self._sample_fragments(steps_total))

    def _collect_metrics(self):
        from ..._private.worker import get

        ms = [self.local_runner.get_metrics()]
        if self.remote_runners:
            ms += self._foreach_runner("get_metrics", local_fallback=False)
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
        self.restore_workers()
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
        g = getattr(self, "env_runner_group", None)
        if g is not None:
            res["num_healthy_workers"] = g.num_healthy_remote_env_runners()
            res["num_remote_worker_restarts"] = g.num_remote_env_runner_restarts()
            res["num_env_runner_failures"] = len(g.failures)
            res["counters"] = dict(getattr(self, "_counters", {}))
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
        if getattr(self.config, "off_policy_estimation_methods", None) and getattr(self, "reader", None) is not None:
            out = self._evaluate()
            out["off_policy_estimator"] = self.estimate_off_policy()
        else:
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

    def estimate_off_policy(self, batches: int = 8) -> Dict:
        """Off-policy estimates of the current policy's value from ``batches`` offline batches,
        one entry per ``config.off_policy_estimation_methods`` (reference:
        ``Algorithm._run_offline_evaluation`` with ``rllib/offline/estimators``)."""
        from ..policy.sample_batch import concat_samples

        from ..offline.estimators import split_by_episode

        methods = self.config.off_policy_estimation_methods or {}
        stored = getattr(self.reader, "batches", None)  # JsonReader: the logged batches, in order (no repeats)
        data = list(stored[:batches]) if stored is not None else [self.reader.next() for _ in range(batches)]
        # episodes whole: with eps_id an episode logged across several batches is joined, and
        # pieces the log cut off (no terminal step) are left out
        flat = [b.flatten() if getattr(b, "fragment_shape", None) is not None else b for b in data]
        joined = concat_samples(flat) if len(flat) > 1 else flat[0]
        episodes = split_by_episode(joined, complete_only=True) or split_by_episode(joined)
        module = self.get_module()
        out = {}
        for name, spec in methods.items():
            spec = dict(spec)
            cls = spec.pop("type")
            est = cls(module, gamma=spec.pop("gamma", self.config.gamma), **spec)
            for b in data:
                est.train(b)
            out[name] = est.estimate_episodes(episodes)
        return out

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

    # ------------------------------------------------------------------ runtime policy mutation
    def add_policy(self, policy_id, policy_cls=None, policy=None, *, observation_space=None, action_space=None,
                   config=None, policy_state=None, policy_mapping_fn=None, policies_to_train=None,
                   module_spec=None, evaluation_workers=True, **kw):
        """Add a policy (its RLModule + learner group) to a running multi-agent algorithm and to
        every env runner (reference ``algorithm.py:1929``; league / self-play training).
        ``policy_state``: initial weights (e.g. a frozen copy of another policy's
        ``get_weights()``); ``policy_mapping_fn``: the new agent -> policy mapping;
        ``policies_to_train``: the new trainable set. Returns the new policy's ``TorchPolicy``."""
        if not self.multi_agent:
            raise ValueError("add_policy needs a multi-agent algorithm (config.multi_agent(policies=...))")
        if policy_id in self.learner_groups:
            raise KeyError(f"policy {policy_id!r} already exists")
        from ..core.learner import LearnerGroup

        sp = self.local_runner.spaces()
        if observation_space is None or action_space is None:
            if module_spec is not None and module_spec.observation_space is not None:
                observation_space = observation_space or module_spec.observation_space
                action_space = action_space or module_spec.action_space
            else:
                fn = policy_mapping_fn or self.config.policy_mapping_fn
                env0 = self.local_runner.envs[0]
                agents = [a for a in self.local_runner.agent_ids if fn is not None and fn(a, None, worker=None) ==
                          policy_id]
                if agents:
                    observation_space = observation_space or env0.get_observation_space(agents[0])
                    action_space = action_space or env0.get_action_space(agents[0])
                else:
                    first = next(iter(sp.values()))
                    observation_space, action_space = observation_space or first[0], action_space or first[1]
        if module_spec is not None:
            from ..core.rl_module import MultiRLModuleSpec

            spec = self._learner_dict.get("rl_module_spec")
            if isinstance(spec, MultiRLModuleSpec):
                specs = dict(spec.module_specs)
            elif isinstance(spec, dict):
                specs = dict(spec)
            else:
                specs = {} if spec is None else {"default_policy": spec}
            specs[policy_id] = module_spec
            self._learner_dict["rl_module_spec"] = specs
            self.env_runner_group._runner_config["rl_module_spec"] = specs
            self.local_runner.cfg["rl_module_spec"] = specs
        ld = dict(self._learner_dict, **(config or {}), _module_id=policy_id)
        g = LearnerGroup(ld, observation_space, action_space)
        if policy_state is not None:
            g.call("set_weights", policy_state)
        self.learner_groups[policy_id] = g
        w = g.get_weights()
        self.local_runner.add_policy(policy_id, observation_space, action_space, w, policy_mapping_fn)
        if self.remote_runners:
            self._foreach_runner("add_policy", policy_id, observation_space, action_space, w, policy_mapping_fn,
                                 local_fallback=False)
        self.env_runner_group._runner_config["policies"] = dict.fromkeys(self.learner_groups)
        if policy_mapping_fn is not None:
            self.config.policy_mapping_fn = policy_mapping_fn
            self.env_runner_group._runner_config["policy_mapping_fn"] = policy_mapping_fn
        pols = dict(self.config.policies or {})
        pols[policy_id] = None
        self.config.policies = pols
        if policies_to_train is not None:
            self.policies_to_train = [p for p in policies_to_train if p in self.learner_groups]
        else:
            self.policies_to_train = list(self.policies_to_train) + [policy_id]
        self.config.policies_to_train = list(self.policies_to_train)
        self._sync_weights()
        return self.get_policy(policy_id)

    def remove_policy(self, policy_id, *, policy_mapping_fn=None, policies_to_train=None, evaluation_workers=True,
                      **kw):
        """Remove a policy from the learners and every env runner (reference ``algorithm.py:2126``)."""
        if not self.multi_agent or policy_id not in self.learner_groups:
            raise KeyError(f"unknown policy {policy_id!r}")
        if len(self.learner_groups) == 1:
            raise ValueError("cannot remove the last policy")
        self.local_runner.remove_policy(policy_id, policy_mapping_fn)
        if self.remote_runners:
            self._foreach_runner("remove_policy", policy_id, policy_mapping_fn, local_fallback=False)
        self.learner_groups.pop(policy_id).shutdown()
        if self.learner_group is None or policy_id not in self.learner_groups:
            first = next(iter(self.learner_groups))
            self.learner_group = self.learner_groups[first]
            self.obs_space, self.act_space = self.local_runner.spaces()[first]
        pols = dict(self.config.policies or {})
        pols.pop(policy_id, None)
        self.config.policies = pols
        self.env_runner_group._runner_config["policies"] = dict.fromkeys(self.learner_groups)
        if policy_mapping_fn is not None:
            self.config.policy_mapping_fn = policy_mapping_fn
            self.env_runner_group._runner_config["policy_mapping_fn"] = policy_mapping_fn
        self.policies_to_train = [p for p in (policies_to_train or self.policies_to_train) if p != policy_id]
        self.config.policies_to_train = list(self.policies_to_train)

    def add_module(self, module_id, module_spec=None, *, config_overrides=None, new_agent_to_module_mapping_fn=None,
                   new_should_module_be_updated=None, add_to_learners=True, add_to_env_runners=True, **kw):
        """New-API-stack name of ``add_policy`` (reference ``algorithm.py:2054``)."""
        return self.add_policy(module_id, module_spec=module_spec, config=config_overrides,
                               policy_mapping_fn=new_agent_to_module_mapping_fn,
                               policies_to_train=new_should_module_be_updated)

    def remove_module(self, module_id, *, new_agent_to_module_mapping_fn=None, new_should_module_be_updated=None,
                      **kw):
        return self.remove_policy(module_id, policy_mapping_fn=new_agent_to_module_mapping_fn,
                                  policies_to_train=new_should_module_be_updated)

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
        if self.multi_agent:
            keep = (set(self.policies_to_train) if self.config.checkpoint_trainable_policies_only
                    else set(self.learner_groups))
            learner = {p: g.call("get_state") for p, g in self.learner_groups.items() if p in keep}
        else:
            learner = self.learner_group.call("get_state")
        if self.config.export_native_model_files:
            for p in (list(learner) if self.multi_agent else [None]):
                self.export_policy_model(os.path.join(checkpoint_dir, "native_models", str(p or "default_policy")), p)
        st = {"learner": learner, "iteration": self._iteration, "multi_agent": self.multi_agent,
              "timesteps_total": self._timesteps_total, "config": self.config.to_dict(),
              "extra": self._extra_state()}
        if not self.multi_agent and getattr(self.local_runner, "has_stateful_connectors", False):
            st["connector_state"] = self.local_runner.get_connector_state()  # e.g. MeanStd statistics
        with open(os.path.join(checkpoint_dir, "algorithm_state.pkl"), "wb") as f:
            cloudpickle.dump(st, f)  # configs hold user callables (policy_mapping_fn, ...)
        with open(os.path.join(checkpoint_dir, "rllib_checkpoint.json"), "w") as f:
            json.dump({"type": "Algorithm", "algo": type(self).__name__, "format": "rca-1"}, f)
        return checkpoint_dir

    def load_checkpoint(self, checkpoint):
        path = checkpoint if isinstance(checkpoint, str) else getattr(checkpoint, "path", checkpoint)
        with open(os.path.join(path, "algorithm_state.pkl"), "rb") as f:
            st = pickle.load(f)
        if st.get("multi_agent"):
            for p, ls in st["learner"].items():
                if p in self.learner_groups:
                    self.learner_groups[p].call("set_state", ls)
        else:
            self.learner_group.call("set_state", st["learner"])
        self._iteration = st["iteration"]
        self._timesteps_total = st["timesteps_total"]
        self._load_extra_state(st.get("extra") or {})
        if st.get("connector_state") is not None and getattr(self.local_runner, "has_stateful_connectors", False):
            self.local_runner.set_connector_state(st["connector_state"])
            if self.remote_runners:
                self._foreach_runner("set_connector_state", st["connector_state"], local_fallback=False)
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
        g = getattr(self, "env_runner_group", None)
        if g is not None:
            g.stop()
        reader = getattr(getattr(self, "local_runner", None), "reader", None)
        if reader is not None and hasattr(reader, "stop"):  # e.g. a PolicyServerInput's HTTP server
            reader.stop()
        for g in (self.learner_groups.values() if self.multi_agent else [self.learner_group]):
            g.shutdown()

    cleanup = stop

    @property
    def iteration(self):
        return self._iteration

    # ------------------------------------------------------------------ reference API surface
    @classmethod
    def get_default_config(cls):
        return cls._default_config_cls()

    def get_default_policy_class(self, config=None):
        """Old-API-stack policy class of this algorithm: the torch policy view over its RLModule."""
        from ..policy.policy import TorchPolicy

        return TorchPolicy

    @staticmethod
    def validate_env(env, env_context=None) -> None:
        """An env must expose observation and action spaces (reference hook; algorithms override)."""
        if env is None:
            return
        if getattr(env, "observation_space", None) is None or getattr(env, "action_space", None) is None:
            raise ValueError(f"env {env!r} has no observation_space / action_space")

    def validate_config(self, config=None) -> None:
        (config or self.config).validate()

    @classmethod
    def merge_algorithm_configs(cls, config1, config2, _allow_unknown_configs=None) -> Dict:
        """Deep-merge two config dicts (``config2`` wins; nested dicts merge key by key)."""
        def to_d(c):
            return c.to_dict() if isinstance(c, AlgorithmConfig) else dict(c or {})

        def merge(a, b):
            out = dict(a)
            for k, v in b.items():
                out[k] = merge(out[k], v) if isinstance(out.get(k), dict) and isinstance(v, dict) else v
            return out

        base, over = to_d(config1), to_d(config2)
        if _allow_unknown_configs is False:
            unknown = set(over) - set(base)
            if unknown:
                raise KeyError(f"unknown config keys {sorted(unknown)}")
        return merge(base, over)

    @classmethod
    def default_resource_request(cls, config):
        """The placement group one trial of this algorithm needs under Tune: the driver (plus its
        GPU when it trains locally), one bundle per env runner, one per GPU learner."""
        from ...tune import PlacementGroupFactory

        c = config if isinstance(config, AlgorithmConfig) else cls._default_config_cls().update_from_dict(dict(config))
        n_learn = int(c.num_learners)
        head = {"CPU": 1.0}
        if n_learn == 0 and float(c.num_gpus or 0) > 0:
            head["GPU"] = float(c.num_gpus)
        bundles = [head]
        for _ in range(int(c.num_env_runners)):
            b = {"CPU": float(c.num_cpus_per_env_runner)}
            if float(c.num_gpus_per_env_runner or 0) > 0:
                b["GPU"] = float(c.num_gpus_per_env_runner)
            bundles.append(b)
        for _ in range(n_learn):
            b = {"CPU": 1.0}
            if float(c.num_gpus_per_learner or 0) > 0:
                b["GPU"] = float(c.num_gpus_per_learner)
            bundles.append(b)
        return PlacementGroupFactory(bundles, strategy="PACK")

    @classmethod
    def resource_help(cls, config) -> str:
        return ("\n\nYou can adjust the resource requests of RLlib Algorithms by calling "
                "`AlgorithmConfig.env_runners(num_env_runners=.., num_cpus_per_env_runner=.., "
                "num_gpus_per_env_runner=..)` and `AlgorithmConfig.learners(num_learners=.., "
                "num_gpus_per_learner=..)`. This trial asks for "
                f"{cls.default_resource_request(config).bundles}.")

    def get_auto_filled_metrics(self, now=None, time_this_iter=None, timestamp=None, debug_metrics_only=False) -> Dict:
        import datetime

        now = now or datetime.datetime.now()
        out = {"training_iteration": self._iteration, "timesteps_total": self._timesteps_total,
               "episodes_total": self._episodes_total}
        if not debug_metrics_only:
            out.update({"date": now.strftime("%Y-%m-%d_%H-%M-%S"), "timestamp": int(timestamp or time.time()),
                        "time_this_iter_s": time_this_iter, "pid": os.getpid()})
        return out

    def log_result(self, result: Dict) -> None:
        """Record a result dict (reference: Trainable.log_result, after the callbacks saw it)."""
        self._last_result = dict(result)

    def get_state(self) -> Dict:
        """Learner states, counters and the config: everything ``from_state`` / ``set_state`` need."""
        if self.multi_agent:
            learner = {p: g.call("get_state") for p, g in self.learner_groups.items()}
        else:
            learner = self.learner_group.call("get_state")
        return {"learner": learner, "iteration": self._iteration, "multi_agent": self.multi_agent,
                "timesteps_total": self._timesteps_total, "config": self.config.to_dict(),
                "algorithm_class": type(self), "extra": self._extra_state()}

    def set_state(self, state: Dict) -> None:
        if state.get("multi_agent"):
            for p, ls in state["learner"].items():
                if p in self.learner_groups:
                    self.learner_groups[p].call("set_state", ls)
        else:
            self.learner_group.call("set_state", state["learner"])
        self._iteration = state.get("iteration", self._iteration)
        self._timesteps_total = state.get("timesteps_total", self._timesteps_total)
        self._load_extra_state(state.get("extra") or {})
        self._sync_weights()

    @staticmethod
    def from_state(state: Dict) -> "Algorithm":
        """A new Algorithm built from ``get_state()`` output (class, config, weights, counters)."""
        cls = state.get("algorithm_class")
        if cls is None:
            raise ValueError("state has no algorithm_class")
        algo = cls(config=cls._default_config_cls().update_from_dict(state["config"]))
        algo.set_state(state)
        return algo

    def export_policy_checkpoint(self, export_dir: str, policy_id=None) -> str:
        """A policy checkpoint: the module's weights (``policy_state.pt``, ``weights_only``-loadable)
        plus its spaces / config summary (``policy_info.json``)."""
        os.makedirs(export_dir, exist_ok=True)
        m = self.get_module(policy_id)
        torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, os.path.join(export_dir, "policy_state.pt"))
        info = {"policy_id": policy_id or "default_policy", "module_class": type(m).__name__,
                "algorithm": type(self).__name__, "model": self.config.model}
        with open(os.path.join(export_dir, "policy_info.json"), "w") as f:
            json.dump(info, f, default=str)
        with open(os.path.join(export_dir, "rllib_checkpoint.json"), "w") as f:
            json.dump({"type": "Policy", "format": "rca-1"}, f)
        from ..policy.policy import TorchPolicy  # + policy_state.pkl: Policy.from_checkpoint(export_dir)

        obs_space = getattr(m, "obs_space", None) or self.obs_space
        act_space = getattr(m, "act_space", None) or self.act_space
        TorchPolicy(obs_space, act_space, {"model": self.config.model}, model=m).export_checkpoint(export_dir)
        return export_dir

    def import_model(self, import_file: str):
        """Load policy weights exported by ``export_policy_model`` / ``export_policy_checkpoint``
        (``model.pt`` / ``policy_state.pt``; Keras h5 files are TensorFlow-only)."""
        if str(import_file).endswith(".h5"):
            return self.import_policy_model_from_h5(import_file)
        path = import_file
        if os.path.isdir(path):
            for name in ("policy_state.pt", "model.pt"):
                if os.path.exists(os.path.join(path, name)):
                    path = os.path.join(path, name)
                    break
        sd = torch.load(path, weights_only=True)
        m = self.get_module()
        m.load_state_dict(sd)
        self.set_weights(m.get_state() if hasattr(m, "get_state") else {k: v for k, v in sd.items()})

    def import_policy_model_from_h5(self, import_file: str, policy_id=None):
        raise NotImplementedError("Keras .h5 policy models are TensorFlow-only; export/import torch "
                                  "state_dicts with export_policy_model / import_model")


class _SaveResult:
    def __init__(self, checkpoint):
        self.checkpoint = checkpoint

    def __fspath__(self):
        return self.checkpoint.path

    def __str__(self):
        return self.checkpoint.path
